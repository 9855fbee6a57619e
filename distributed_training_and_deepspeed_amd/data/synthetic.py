"""Synthetic token datasets with the reference's schema and masking law.

The reference tokenizes wikitext-2 (util.py:38-60): rows padded/truncated to 512 tokens, then
either *static* MLM masking via HF DataCollatorForLanguageModeling.torch_mask_tokens
(p = 0.15 over non-special tokens; of those 80% -> [MASK], 10% -> random token, 10% kept;
unmasked labels -100 -- SURVEY.md D19) or causal labels = input_ids (pads included).
There is no network on the MI355X boxes, so rows here are random token ids with the same
shape, framing ([CLS] ... [SEP] for BERT) and the same masking law, generated
deterministically from a seed.  ``pad_fraction`` optionally right-pads rows with the pad id
to mimic short wikitext lines.
"""
from __future__ import annotations

import torch
from torch.utils.data import Dataset

from ..models.config import TransformerConfig

IGNORE_INDEX = -100


def mlm_mask_tokens(input_ids: torch.Tensor, special_mask: torch.Tensor, vocab_size: int, mask_token_id: int,
                    generator: torch.Generator, mlm_probability: float = 0.15):
    """HF ``torch_mask_tokens`` law.  Returns (masked inputs, labels)."""
    labels = input_ids.clone()
    prob = torch.full(labels.shape, mlm_probability)
    prob.masked_fill_(special_mask, 0.0)
    masked = torch.bernoulli(prob, generator=generator).bool()
    labels[~masked] = IGNORE_INDEX
    inputs = input_ids.clone()
    replaced = torch.bernoulli(torch.full(labels.shape, 0.8), generator=generator).bool() & masked
    inputs[replaced] = mask_token_id
    rnd = torch.bernoulli(torch.full(labels.shape, 0.5), generator=generator).bool() & masked & ~replaced
    inputs[rnd] = torch.randint(vocab_size, labels.shape, dtype=inputs.dtype, generator=generator)[rnd]
    return inputs, labels


def synthetic_token_rows(n: int, seq_len: int, cfg: TransformerConfig, generator: torch.Generator,
                         pad_fraction: float = 0.0):
    """Random rows (+ special-token mask).  BERT rows are framed [CLS] x ... x [SEP]."""
    specials = set(cfg.special_token_ids)
    lo = max(specials) + 1 if cfg.family == "bert" and specials else 0
    lo = min(lo, cfg.vocab_size - 1)
    ids = torch.randint(lo, cfg.vocab_size, (n, seq_len), generator=generator, dtype=torch.int64)
    if cfg.family == "bert":
        ids[:, 0] = 101
        ids[:, -1] = 102
    if pad_fraction > 0:
        lengths = torch.randint(2, seq_len + 1, (n,), generator=generator)
        padded = torch.rand(n, generator=generator) < pad_fraction
        for i in torch.nonzero(padded).flatten().tolist():
            L = int(lengths[i])
            if cfg.family == "bert":
                ids[i, L - 1] = 102
            ids[i, L:] = cfg.pad_token_id
    special = torch.zeros_like(ids, dtype=torch.bool)
    for s in specials:
        special |= ids == s
    return ids, special


class SyntheticLMDataset(Dataset):
    """Map-style dataset of {'input_ids', 'labels'} rows, statically masked like util.py."""

    def __init__(self, cfg: TransformerConfig, num_samples: int, seq_len: int = 512, mlm: bool | None = None,
                 seed: int = 0, pad_fraction: float = 0.0):
        self.cfg = cfg
        self.mlm = (cfg.family == "bert") if mlm is None else mlm
        g = torch.Generator().manual_seed(seed)
        ids, special = synthetic_token_rows(num_samples, seq_len, cfg, g, pad_fraction)
        if self.mlm:
            self.input_ids, self.labels = mlm_mask_tokens(ids, special, cfg.vocab_size, cfg.mask_token_id, g)
        else:
            self.input_ids, self.labels = ids, ids.clone()  # util.py:54-58: pads included

    def __len__(self):
        return self.input_ids.shape[0]

    def __getitem__(self, i):
        return {"input_ids": self.input_ids[i], "labels": self.labels[i]}

    def select(self, indices) -> "SyntheticLMDataset":
        """HF ``Dataset.select`` parity (data_parallel_training.py:36)."""
        idx = torch.as_tensor(list(indices), dtype=torch.int64)
        out = object.__new__(SyntheticLMDataset)
        out.cfg, out.mlm = self.cfg, self.mlm
        out.input_ids, out.labels = self.input_ids[idx], self.labels[idx]
        return out


def load_synthetic(cfg: TransformerConfig, num_samples: int, seq_len: int = 512, mlm: bool | None = None,
                   seed: int = 0) -> SyntheticLMDataset:
    """Stand-in for ``util.load_wikitext`` (same columns, same masking law)."""
    return SyntheticLMDataset(cfg, num_samples, seq_len, mlm=mlm, seed=seed)
