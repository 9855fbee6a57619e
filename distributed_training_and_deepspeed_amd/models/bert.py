"""BERT for masked-LM pre-training (HF ``BertForMaskedLM`` equivalent, random init).

Reference usage: ``BertForMaskedLM.from_pretrained('bert-base-cased'|'bert-large-cased')`` and
``model(input_ids, labels=...).loss`` (data_parallel_training.py:30-31,53-54).  Architecture
per SURVEY.md D15: word+position+token-type embeddings -> LN(1e-12) -> dropout 0.1;
N post-LN encoder layers (fused q/k/v projection: identical parameter count to HF's three
Linears); MLM head dense -> GELU(erf) -> LN -> decoder tied to the word embeddings + bias;
cross entropy with ignore_index -100 over all labelled positions.  No attention mask is
applied (the reference never passes one), and there is no pooler (add_pooling_layer=False).
Parameter count for bert-base-cased: 108,340,804.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
from torch import nn

from .config import BERT_BASE, TransformerConfig, get_config
from .layers import Embeddings, MLMHead
from .transformer import Runtime, TransformerLayer, prefetch_masks, stage_dgrad_transposes


@dataclass
class MaskedLMOutput:
    loss: torch.Tensor | None = None
    logits: torch.Tensor | None = None


class BertForMaskedLM(nn.Module):
    def __init__(self, cfg: TransformerConfig = BERT_BASE, rt: Runtime | None = None, sparse_mlm_head: bool = True):
        super().__init__()
        self.config = self.cfg = cfg
        self.rt = rt or Runtime()
        self.embeddings = Embeddings(cfg, self.rt)
        self.layers = nn.ModuleList([TransformerLayer(cfg, self.rt) for _ in range(cfg.num_layers)])
        self.head = MLMHead(cfg, self.rt, self.embeddings.word, sparse=sparse_mlm_head)

    @classmethod
    def from_config(cls, name: str, **kw) -> "BertForMaskedLM":
        return cls(get_config(name), **kw)

    def zero3_units(self):
        """Parameter-gathering units for ZeRO-3, in forward order."""
        return [self.embeddings, *self.layers, self.head]

    def zero3_persistent(self):
        """Parameters shared between units (tied decoder / word embeddings)."""
        return [self.embeddings.word] if self.head.decoder_w is None else []

    def encode(self, input_ids: torch.Tensor) -> torch.Tensor:
        if input_ids.is_cuda and self.training:
            prefetch_masks(self.layers, input_ids)
        x = self.embeddings(input_ids)
        for layer in self.layers:
            x = layer(x)
        stage_dgrad_transposes(self.layers, x)
        return x

    def forward(self, input_ids: torch.Tensor, labels: torch.Tensor | None = None,
                return_logits: bool = False) -> MaskedLMOutput:
        x = self.encode(input_ids)
        out = MaskedLMOutput()
        if labels is not None:
            out.loss = self.head(x, labels)
        if labels is None or return_logits:
            out.logits = self.head(x)   # module call: ZeRO-3 / staged-optimizer hooks fire
        return out
