"""Counter-based dropout RNG shared by the HIP kernels and the PyTorch reference.

A dropout keep-decision is a pure function of (seed, step, stream id, element index), so
  * backward passes regenerate masks instead of storing them (no mask tensors in memory),
  * activation recompute in the pipeline engine reproduces the forward's masks exactly
    (the reference relies on torch Pipe's RNG-state save/restore for this),
  * the HIP kernel and this module produce bit-identical masks, so kernel-vs-reference
    numerics tests can run with dropout on.
The {seed, step} pair lives in device memory and ``advance()`` bumps the step with a device
op, which keeps masks fresh under hipGraph replay.
Hash: the same mix32 construction as ``ops/csrc/common.h`` (DropoutRng).
"""
from __future__ import annotations

import itertools

import torch

M32 = 0xFFFFFFFF
_SID = itertools.count(1)


def new_stream_id() -> int:
    """Unique id for one dropout call site (module instance); 20 bits, shifted left by 10."""
    return next(_SID) & 0xFFFFF


def _mix32(h: torch.Tensor) -> torch.Tensor:
    h = h & M32
    h = h ^ (h >> 16)
    h = (h * 0x7FEB352D) & M32
    h = h ^ (h >> 15)
    h = (h * 0x846CA68B) & M32
    h = h ^ (h >> 16)
    return h


def _mix32_int(h: int) -> int:
    h &= M32
    h ^= h >> 16
    h = (h * 0x7FEB352D) & M32
    h ^= h >> 15
    h = (h * 0x846CA68B) & M32
    h ^= h >> 16
    return h


def _keys(seed: int, step: int, sid: int) -> tuple[int, int]:
    k0 = _mix32_int((seed & M32) ^ _mix32_int(((seed >> 32) + 0x9E3779B9) & M32))
    k1 = _mix32_int(((step & M32) * 0x85EBCA6B & M32) ^ _mix32_int((sid + 0x632BE5AB) & M32) ^ k0)
    return k0, k1


def keep_threshold(p: float) -> int:
    t = p * 65536.0
    return 65536 if t >= 65536.0 else int(t + 0.5)


def keep_mask(numel: int, p: float, seed: int, step: int, sid: int, device="cpu") -> torch.Tensor:
    """Bool keep-mask for a flat tensor of ``numel`` elements (identical to the HIP kernels)."""
    k0, k1 = _keys(seed, step, sid)
    e = torch.arange(numel, dtype=torch.int64, device=device)
    i = e >> 1
    lo = i & M32
    hi = i >> 32
    b = _mix32(((lo ^ k0) + (((hi * 0xC2B2AE35) & M32) ^ k1)) & M32)
    h16 = torch.where((e & 1) == 1, b >> 16, b & 0xFFFF)
    return h16 >= keep_threshold(p)


def _xorshift32(x: torch.Tensor) -> torch.Tensor:
    x = x ^ ((x << 13) & M32)
    x = x ^ (x >> 17)
    x = x ^ ((x << 5) & M32)
    return x


def attn_keep_mask(B: int, H: int, S: int, p: float, seed: int, step: int, sid: int, device="cpu") -> torch.Tensor:
    """Bool keep-mask [B, H, S, S] of attention-probability dropout (identical to the HIP mask
    generator, ops/csrc/attention.hip ``attn_mask_kernel``).

    Per (batch*head, query, 32-key word) one counter hash seeds an xorshift32 stream; its 16
    outputs give the 32 keep decisions of the word (low / high 16 bits of output n -> keys
    2n / 2n+1, keep iff >= the 16-bit threshold).  B*H*S*S decisions per layer make the
    generator VALU-bound, so only one of every 16 32-bit draws pays for the full (two-multiply)
    mix; the rest are three shift-xor pairs."""
    k0, k1 = _keys(seed, step, sid)
    W = (S + 31) // 32
    ctr = torch.arange(B * H * S * W, dtype=torch.int64, device=device)
    lo, hi = ctr & M32, ctr >> 32
    x = _mix32(((lo ^ k0) + (((hi * 0xC2B2AE35) & M32) ^ k1)) & M32)
    x = torch.where(x == 0, torch.full_like(x, 0x6D2B79F5), x)
    thr = keep_threshold(p)
    outs = []
    for n in range(16):
        if n:
            x = _xorshift32(x)
        outs.append((x & 0xFFFF) >= thr)
        outs.append((x >> 16) >= thr)
    keep = torch.stack(outs, -1).view(B, H, S, W * 32)
    return keep[..., :S].contiguous()


class RngState:
    """Device-resident {seed, step} for the dropout kernels plus the host-side micro-batch id."""

    def __init__(self, seed: int = 0, device=None):
        self.seed = int(seed) & 0x7FFFFFFFFFFFFFFF
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.state = torch.tensor([self.seed, 0], dtype=torch.int64, device=self.device)
        self.micro = 0  # micro-batch index (gradient accumulation / pipeline chunks)

    def to(self, device) -> "RngState":
        self.device = torch.device(device)
        self.state = self.state.to(self.device)
        return self

    def reseed(self, seed: int) -> "RngState":
        """New dropout seed, in place (keeps the device tensor, so captured graphs stay valid).
        Data-parallel trainers offset it by rank: replicas then draw independent masks, as
        unseeded per-process RNGs do in the reference's torch DDP runs."""
        self.seed = int(seed) & 0x7FFFFFFFFFFFFFFF
        self.state.copy_(torch.tensor([self.seed, 0], dtype=torch.int64))
        return self

    def advance(self) -> None:
        """Next training step (device op: graph-capturable)."""
        self.state[1:2].add_(1)

    def sid(self, base: int) -> int:
        return ((base & 0xFFFFF) << 10) | (self.micro & 0x3FF)

    def host_step(self) -> int:
        return int(self.state[1].item())


_DEFAULT: dict = {}


def default_rng(device) -> RngState:
    key = str(torch.device(device))
    if key not in _DEFAULT:
        _DEFAULT[key] = RngState(seed=torch.initial_seed(), device=device)
    return _DEFAULT[key]


def set_default_rng(rng: RngState) -> None:
    _DEFAULT[str(rng.device)] = rng
