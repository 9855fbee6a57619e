"""Offline text dataset loader with the reference's ``util.load_wikitext`` contract.

Reference (util.py:38-60): load wikitext-2-v1 train, batch-tokenize with
``padding='max_length', truncation=True, return_special_tokens_mask=True``, then either apply
*static* MLM masking once (``collator.torch_mask_tokens``: 15% / 80-10-10) or, for causal LMs,
``labels = input_ids`` -- pads included, because the collator is bypassed (quirk 8) -- and keep
no attention mask.

There is no network on the MI355X boxes, so this loader reads a LOCAL copy: a directory saved with
``datasets.Dataset.save_to_disk`` / ``DatasetDict.save_to_disk`` (split ``train``, column ``text``),
a parquet / arrow / json(l) file, or plain text files (one example per line, like the raw wikitext
``wiki.train.raw``).  The tokenizer is any HF tokenizer object (e.g. loaded from a local directory
with ``AutoTokenizer.from_pretrained(path)``).  The masking law is the same function the synthetic
datasets use (``synthetic.mlm_mask_tokens``), seeded for reproducibility.
"""
from __future__ import annotations

import os

import torch

from .synthetic import SyntheticLMDataset, mlm_mask_tokens


def read_text_lines(path: str, split: str = "train", column: str = "text") -> list[str]:
    """Lines of a local corpus (see module docstring for the accepted layouts)."""
    if os.path.isdir(path):
        if any(os.path.exists(os.path.join(path, f)) for f in ("dataset_info.json", "dataset_dict.json", "state.json")):
            import datasets
            ds = datasets.load_from_disk(path)
            if isinstance(ds, datasets.DatasetDict):
                ds = ds[split]
            return list(ds[column])
        files = sorted(os.path.join(path, f) for f in os.listdir(path)
                       if f.endswith((".txt", ".raw", ".tokens")) and split in f)
        if not files:
            raise FileNotFoundError(f"no '{split}' text files in {path}")
        lines: list[str] = []
        for f in files:
            lines += read_text_lines(f)
        return lines
    if path.endswith((".parquet", ".arrow", ".json", ".jsonl")):
        import datasets
        kind = {"parquet": "parquet", "arrow": "arrow", "json": "json", "jsonl": "json"}[path.rsplit(".", 1)[1]]
        return list(datasets.load_dataset(kind, data_files=path, split="train")[column])
    with open(path, encoding="utf-8") as f:
        return [ln.rstrip("\n") for ln in f]


class TokenizedLMDataset(SyntheticLMDataset):
    """Same container as the synthetic datasets ({'input_ids', 'labels'} rows, ``select``)."""

    def __init__(self, input_ids: torch.Tensor, labels: torch.Tensor, mlm: bool, cfg=None):  # noqa: D107
        self.cfg, self.mlm = cfg, mlm
        self.input_ids, self.labels = input_ids, labels


def load_wikitext(tokenizer, collator=None, max_length: int | None = None, *, path: str, mlm: bool | None = None,
                  mlm_probability: float | None = None, seed: int = 0, limit: int | None = None) -> TokenizedLMDataset:
    """``util.load_wikitext`` parity on a local corpus.  ``collator`` (optional) supplies
    ``mlm`` / ``mlm_probability`` like HF's DataCollatorForLanguageModeling."""
    if mlm is None:
        mlm = bool(getattr(collator, "mlm", True))
    if mlm_probability is None:
        mlm_probability = float(getattr(collator, "mlm_probability", 0.15))
    lines = read_text_lines(path)
    if limit is not None:
        lines = lines[:limit]
    max_length = max_length or getattr(tokenizer, "model_max_length", 512)
    enc = tokenizer(lines, padding="max_length", truncation=True, max_length=max_length,
                    return_special_tokens_mask=True, return_tensors="pt")
    ids = enc["input_ids"].to(torch.int64)
    if mlm:
        special = enc["special_tokens_mask"].bool()
        g = torch.Generator().manual_seed(seed)
        inputs, labels = mlm_mask_tokens(ids, special, len(tokenizer), tokenizer.mask_token_id, g, mlm_probability)
    else:
        inputs, labels = ids, ids.clone()          # util.py:54-58: pads included, no attention mask
    return TokenizedLMDataset(inputs, labels, mlm)
