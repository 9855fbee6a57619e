"""Training-memory estimators, re-derived for MI355X (288 GB HBM3E per GPU).

Reference parity (estimate_nn_memory.py, estimate_transformer_memory.py):
* ``get_model_memory(model)``: sum numel * element_size over parameters;
* ``ActivationCounter`` + ``register_hooks_recursive``: bytes of every submodule's forward
  output, Dropout outputs counted as a 1-byte/element mask (estimate_nn_memory.py:27-37);
* ``get_optimizer_memory``: Adam/AdamW 8 B/param (two fp32 moments), SGD+momentum 4, SGD 0;
  the framework's ``FusedAdam`` additionally keeps an fp32 master copy when the model is bf16;
* ``project_transformer_memory``: the reference's fp32 formula
  model = 4*L*h*(13 + 12h), grad = model, activations = L*b*s*h*(67 + 9*a*s/h) bytes
  (Korthikanti et al. 2205.05198 adapted to fp32), optimizer from the optimizer type.  The
  reference reads a *global* ``model`` for the optimizer term (quirk 3); here the parameter
  count is passed explicitly.

MI355X-first extensions:
* ``project_training_memory`` covers bf16 mixed precision (bf16 params/grads + fp32 master +
  Adam moments), the flash-attention activation path (no a*s/h score term: scores never
  materialise), dropout masks regenerated instead of stored, and the ZeRO stage partitioning
  of params/grads/optimizer state over N ranks;
* ``max_hidden_for_capacity`` inverts the projection against a capacity (288 GB default).
"""
from __future__ import annotations

import math
from dataclasses import asdict, dataclass

import torch

MI355X_HBM_BYTES = 288 * 10 ** 9


def get_model_memory(model: torch.nn.Module) -> int:
    return sum(p.numel() * p.element_size() for p in model.parameters())


class ActivationCounter:
    """Accumulates activation bytes seen by forward hooks."""

    def __init__(self):
        self.activation_bytes = 0

    def add_activations(self, tensor: torch.Tensor) -> None:
        self.activation_bytes += tensor.numel() * tensor.element_size()

    def add_activation_bytes(self, n: int) -> None:
        self.activation_bytes += n


def activation_counter_hook(counter: ActivationCounter):
    def hook(module, _inp, output):
        outs = output if isinstance(output, (tuple, list)) else (output,)
        for o in outs:
            if not torch.is_tensor(o):
                continue
            if module.__class__.__name__ == "Dropout":
                counter.add_activation_bytes(o.data.numel())  # only the (bool) mask is kept
            else:
                counter.add_activations(o.data)
    return hook


def register_hooks_recursive(model: torch.nn.Module, counter: ActivationCounter) -> list:
    handles = []
    for module in model.children():
        handles.append(module.register_forward_hook(activation_counter_hook(counter)))
        handles += register_hooks_recursive(module, counter)
    return handles


def optimizer_bytes_per_param(optimizer) -> int:
    name = type(optimizer).__name__
    if isinstance(optimizer, torch.optim.SGD):
        return 4 if any(g.get("momentum", 0) != 0 for g in optimizer.param_groups) else 0
    if isinstance(optimizer, (torch.optim.Adam, torch.optim.AdamW)):
        return 8
    if name == "FusedAdam":
        master = 0 if getattr(optimizer, "lowp", None) is None else 4
        return 8 + master
    raise ValueError(f"Unsupported optimizer: {optimizer}")


def get_optimizer_memory(model: torch.nn.Module, optimizer) -> int:
    """Bytes of optimizer state for ``model``'s parameters (reference :18-36)."""
    n = sum(p.numel() for p in model.parameters())
    return n * optimizer_bytes_per_param(optimizer)


def block_params(layers: int, h: int, ffn: int | None = None) -> int:
    ffn = 4 * h if ffn is None else ffn
    return layers * (4 * h * h + 4 * h + 2 * h * ffn + ffn + h + 4 * h)


def project_transformer_memory(layers: int, hidden_size: int, num_attention_heads: int, batch_size: int,
                               sequence_length: int, optimizer_bytes_per_param: int = 8, num_params: int | None = None) -> int:
    """The reference's fp32 projection (estimate_transformer_memory.py:39-54), in bytes."""
    h, a, b, s = hidden_size, num_attention_heads, batch_size, sequence_length
    model_memory = 4 * layers * h * (13 + 12 * h)
    gradient_memory = model_memory
    activation_memory = layers * b * s * h * (67 + (9 * a * s) / h)
    n = num_params if num_params is not None else model_memory // 4
    return int(model_memory + gradient_memory + activation_memory + n * optimizer_bytes_per_param)


@dataclass
class MemoryProjection:
    params: int
    weights: float
    grads: float
    optimizer: float
    activations: float
    total: float
    fits: bool
    capacity: float

    def as_dict(self):
        return asdict(self)


def project_training_memory(layers: int, hidden_size: int, num_heads: int, batch_size: int, seq_len: int,
                            ffn_size: int | None = None, precision: str = "bf16", flash_attention: bool = True,
                            zero_stage: int = 0, world_size: int = 1, capacity: float = MI355X_HBM_BYTES,
                            extra_params: int = 0, keep_ffn_act: bool = True) -> MemoryProjection:
    """Per-GPU bytes for one training replica on MI355X.

    precision 'fp32': fp32 weights + grads + Adam moments (the reference's setting).
    precision 'bf16': bf16 weights + bf16 grads + fp32 master + fp32 Adam moments (16 B/param
    of model state before partitioning).  Activations per layer per token (bytes):
    fp32 eager: h*(67 + 9*a*s/h)  (reference formula);
    bf16 + flash attention (this framework's fused layer): the tensors it saves --
    layer input, qkv, context, two LN sums (2 B/elt), FFN pre-activation (ffn wide) and
    fp32 row statistics, plus the FFN activation itself when ``keep_ffn_act`` (the fused
    layer's default, ``Runtime.keep_ffn_act``); dropout masks are regenerated, scores are
    never stored.
    """
    h, a, s, b = hidden_size, num_heads, seq_len, batch_size
    ffn = 4 * h if ffn_size is None else ffn_size
    n = block_params(layers, h, ffn) + extra_params
    if precision == "fp32":
        w, g, o = 4.0 * n, 4.0 * n, 8.0 * n
        act_per_tok = h * (67 + 9 * a * s / h) if not flash_attention else h * 34 + 4 * ffn
    else:
        w, g, o = 2.0 * n, 2.0 * n, 12.0 * n
        if flash_attention:
            act_per_tok = 2 * (h + 3 * h + h + h + h + ffn) + 4 * 6 + 4 * a  # saved bf16 tensors + stats/LSE
            if keep_ffn_act:
                act_per_tok += 2 * ffn
        else:
            act_per_tok = h * (34 + 5 * a * s / h)  # Korthikanti 16-bit form
    N = max(1, world_size)
    if zero_stage >= 1:
        o /= N
    if zero_stage >= 2:
        g /= N
    if zero_stage >= 3:
        w /= N
    act = layers * b * s * act_per_tok
    total = w + g + o + act
    return MemoryProjection(n, w, g, o, act, total, total <= capacity, capacity)


def max_hidden_for_capacity(capacity: float = MI355X_HBM_BYTES, layers: int = 1, heads_per_128: bool = True,
                            batch_size: int = 4, seq_len: int = 512, fp32_reference: bool = True) -> int:
    """Largest hidden size h (multiple of 128, heads = h/128, ffn = 4h) whose projected training
    memory fits ``capacity`` -- the 288 GB question of SURVEY.md section 6."""
    def fits(k: int) -> bool:
        h = 128 * k
        a = k if heads_per_128 else 16
        if fp32_reference:
            need = project_transformer_memory(layers, h, a, batch_size, seq_len, 8, num_params=block_params(layers, h))
        else:
            need = project_training_memory(layers, h, a, batch_size, seq_len).total
        return need <= capacity

    lo, hi = 1, 1 << 13  # in units of 128
    while lo < hi:
        mid = (lo + hi + 1) // 2
        if fits(mid):
            lo = mid
        else:
            hi = mid - 1
    return 128 * lo
