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


def _rotl32(x: torch.Tensor, r: int) -> torch.Tensor:
    return ((x << r) & M32) | (x >> (32 - r))


ATTN_MASK_ROT = 13   # ops/csrc/attention.hip kMaskRot


def attn_keep_mask(B: int, H: int, S: int, p: float, seed: int, step: int, sid: int, device="cpu") -> torch.Tensor:
    """Bool keep-mask [B, H, S, S] of attention-probability dropout (identical to the HIP mask
    generator, ops/csrc/attention.hip ``attn_mask_kernel``).

    One stream per (batch*head, query): a counter hash of (bh * S + q) expanded by xorshift32 into
    a 16-word state; per 32-key word one additive lagged-Fibonacci round with rotation
    (``s[i] += rotl(s[(i + 11) & 15], 13)``, i ascending, in place).  The 16 words are bit planes:
    key j's 16-bit draw has bit i = bit j of s[i], and keep iff draw >= the 16-bit threshold --
    evaluated for all 32 keys at once by an LSB-first bitwise comparator (the GPU form spends one
    majority op per plane; B*H*S*S decisions per layer make the generator VALU-bound)."""
    k0, k1 = _keys(seed, step, sid)
    W = (S + 31) // 32
    ctr = torch.arange(B * H * S, dtype=torch.int64, device=device)
    lo, hi = ctr & M32, ctr >> 32
    x = _mix32(((lo ^ k0) + (((hi * 0xC2B2AE35) & M32) ^ k1)) & M32)
    x = torch.where(x == 0, torch.full_like(x, 0x6D2B79F5), x)
    st = [x]
    for _ in range(15):
        st.append(_xorshift32(st[-1]))
    thr = keep_threshold(p)
    words = []
    for _ in range(W):
        acc = torch.full_like(x, M32)
        for i in range(16):
            st[i] = (st[i] + _rotl32(st[(i + 11) & 15], ATTN_MASK_ROT)) & M32
            acc = (st[i] & acc) if (thr >> i) & 1 else (st[i] | acc)
        words.append(acc if thr < 65536 else torch.zeros_like(acc))
    bits = (torch.stack(words, -1).unsqueeze(-1) >> torch.arange(32, dtype=torch.int64, device=device)) & 1
    return bits.view(B, H, S, W * 32)[..., :S].bool().contiguous()


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
