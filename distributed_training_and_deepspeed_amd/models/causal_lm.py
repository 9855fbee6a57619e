"""Decoder-only causal LMs (HF ``AutoModelForCausalLM`` equivalents, random init).

Reference usage: ``AutoModelForCausalLM.from_pretrained('bigscience/bloom-560m')`` with
``model(input_ids, labels=labels).loss`` (zero_dp_training.py:24,85); the multi-node script
intends ``facebook/opt-125m`` (scripts/launch-multinode.sh:5) and BASELINE.json names
gpt2-medium.  SURVEY.md D17:
  * BLOOM: word embeddings -> embedding LN, pre-LN blocks with fused QKV, ALiBi, tanh-GELU,
    final LN, tied LM head, vocab 250,880 (559,214,592 parameters for bloom-560m);
  * OPT: word + learned positions (offset 2), pre-LN, ReLU, final LN, tied head;
  * GPT-2: wte + wpe, pre-LN, tanh-GELU, final LN, tied head.
Loss: shifted next-token cross entropy (labels = input_ids, ignore_index -100).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
from torch import nn

from .config import BLOOM_560M, TransformerConfig, get_config
from .layers import Embeddings, LayerNorm, LMHead
from .transformer import Runtime, TransformerLayer, prefetch_masks, stage_dgrad_transposes


@dataclass
class CausalLMOutput:
    loss: torch.Tensor | None = None
    logits: torch.Tensor | None = None


class CausalLM(nn.Module):
    def __init__(self, cfg: TransformerConfig = BLOOM_560M, rt: Runtime | None = None):
        super().__init__()
        self.config = self.cfg = cfg
        self.rt = rt or Runtime()
        self.embeddings = Embeddings(cfg, self.rt)
        self.layers = nn.ModuleList([TransformerLayer(cfg, self.rt) for _ in range(cfg.num_layers)])
        self.final_ln = LayerNorm(cfg.hidden_size, cfg.ln_eps, self.rt) if cfg.final_ln else None
        self.head = LMHead(cfg, self.rt, self.embeddings.word)

    @classmethod
    def from_config(cls, name: str, **kw) -> "CausalLM":
        return cls(get_config(name), **kw)

    def zero3_units(self):
        """Parameter-gathering units for ZeRO-3, in forward order."""
        return [self.embeddings, *self.layers] + ([self.final_ln] if self.final_ln is not None else [])

    def zero3_persistent(self):
        """Parameters shared between units (LM head tied to the word embeddings)."""
        return [self.embeddings.word]

    def encode(self, input_ids: torch.Tensor) -> torch.Tensor:
        if input_ids.is_cuda and self.training:
            prefetch_masks(self.layers, input_ids)
        x = self.embeddings(input_ids)
        for layer in self.layers:
            x = layer(x)
        stage_dgrad_transposes(self.layers, x)
        if self.final_ln is not None:
            x = self.final_ln(x)
        return x

    def forward(self, input_ids: torch.Tensor, labels: torch.Tensor | None = None,
                return_logits: bool = False) -> CausalLMOutput:
        x = self.encode(input_ids)
        out = CausalLMOutput()
        if labels is not None:
            out.loss = self.head(x, labels)
        if labels is None or return_logits:
            out.logits = self.head.logits(x)
        return out
