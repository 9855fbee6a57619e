"""Hand-written MFMA GEMM with fused FFN epilogues (``ops/csrc/gemm.hip``).

``C = A . B^T`` with both operands K-contiguous (a Linear weight [out, in] is exactly B):

* ``linear_gelu(x, w, b)``   -> (u, a): u = x W^T + b, a = gelu(u); the up-projection of the FFN
  forward with the activation computed in the GEMM epilogue (no re-read of u).
* ``gelu_bwd_gemm(dy, w_t, u, dbias)`` -> du = (dy . w_t^T) * gelu'(u) plus the column sums of du
  (the up-projection's bias gradient); the FFN backward's down-projection dgrad with the GELU
  derivative applied in the epilogue (no round trip of da through HBM).
* ``gemm_bt(a, b, bias)``    -> plain product (tests / benchmarks).

Status (measured on MI355X, ``scripts/bench_gemm_fused.py``, profiles/r1_gemm_fused_vs_hipblaslt.jsonl):
the main loop reaches 630-660 TF/s at the FFN shape vs hipBLASLt's 940-970 on the same box, so
the fused epilogues do not yet beat hipBLASLt + the bandwidth-bound activation kernels and the
model keeps the unfused path; the kernels are tested building blocks for the deeper-pipelined
(8-phase, cdna_hip_programming.md §5) main loop they need.

Shapes must tile by 256 x 128 x 64 (256 x 256 x 64 with DTD_GEMM_BN=256) (``supported``); callers fall back to hipBLASLt + the
elementwise kernels otherwise.  bf16 only.
"""
from __future__ import annotations

import torch

from . import _lib

EPI_STORE, EPI_BIAS_GELU, EPI_GELU_BWD = 0, 1, 2


def supported(M: int, N: int, K: int, *tensors) -> bool:
    if not all(t is not None and t.is_cuda and t.dtype == torch.bfloat16 for t in tensors):
        return False
    if not _lib.has("dtd_gemm_bt"):
        return False
    return bool(_lib.lib().dtd_gemm_bt_supported(M, N, K))


def _ld(t: torch.Tensor) -> int:
    assert t.dim() == 2 and t.stride(1) == 1, "operands must be row-major with unit inner stride"
    return t.stride(0)


def _call(epi, a, b, c, c2=None, u=None, bias=None, part=None):
    M, K = a.shape
    N = b.shape[0]
    _lib.call("dtd_gemm_bt", epi, a.data_ptr(), _ld(a), b.data_ptr(), _ld(b), c.data_ptr(), _ld(c), _lib.ptr(c2),
              _lib.ptr(u), _ld(u) if u is not None else 0, _lib.ptr(bias), _lib.ptr(part), M, N, K, _lib.stream())


def gemm_bt(a: torch.Tensor, b: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    c = torch.empty((a.shape[0], b.shape[0]), dtype=a.dtype, device=a.device)
    _call(EPI_STORE, a, b, c, bias=bias)
    return c


def linear_gelu(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None):
    """(u, a) = (x W^T + b, gelu(u)) in one kernel."""
    M, N = x.shape[0], w.shape[0]
    u = torch.empty((M, N), dtype=x.dtype, device=x.device)
    a = torch.empty_like(u)
    _call(EPI_BIAS_GELU, x, w, u, c2=a, bias=b)
    return u, a


def gelu_bwd_gemm(dy: torch.Tensor, w_t: torch.Tensor, u: torch.Tensor, dbias=None, acc: bool = False):
    """du = (dy . w_t^T) * gelu'(u); ``w_t`` is the down-projection weight transposed to
    [ffn, hidden] (K-contiguous).  ``dbias`` (dst, acc) receives the column sums of du."""
    from .functional import _finalize
    M, N = dy.shape[0], w_t.shape[0]
    du = torch.empty((M, N), dtype=dy.dtype, device=dy.device)
    nrows = _lib.lib().dtd_gemm_bt_part_rows(M)
    part = torch.empty((nrows, N), dtype=torch.float32, device=dy.device) if dbias is not None else None
    _call(EPI_GELU_BWD, dy, w_t, du, u=u, part=part)
    if part is not None:
        _finalize(part, nrows, N, dbias, acc)
    return du
