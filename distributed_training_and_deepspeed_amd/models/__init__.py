"""Model zoo: BERT-MLM, decoder-only causal LMs, the model-parallel BERT and the
instrumented transformer block -- all random-init from built-in configs."""
from __future__ import annotations

import torch

from .bert import BertForMaskedLM, MaskedLMOutput  # noqa: F401
from .causal_lm import CausalLM, CausalLMOutput  # noqa: F401
from .config import PRESETS, TransformerConfig, get_config  # noqa: F401
from .transformer import Runtime, TransformerLayer  # noqa: F401


def build_model(name: str, impl: str = "auto", dtype: torch.dtype = torch.float32, device="cpu", seed: int = 0,
                **kw):
    """Instantiate a preset by name (``base``/``large``/``tiny`` or a hub-style id)."""
    from ..ops.rng import RngState
    cfg = get_config(name)
    torch.manual_seed(seed)
    rt = Runtime(impl=impl, rng=RngState(seed=seed, device=device))
    cls = BertForMaskedLM if cfg.family == "bert" else CausalLM
    model = cls(cfg, rt=rt, **kw)
    return model.to(device=device, dtype=dtype)


def count_parameters(model: torch.nn.Module) -> int:
    return sum(p.numel() for p in model.parameters())
