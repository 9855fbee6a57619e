"""Hand-written MFMA GEMM with fused transformer epilogues (``ops/csrc/gemm.hip``).

``C = A . B^T`` with both operands K-contiguous (a Linear weight [out, in] is exactly B; the
input-gradient product uses the transposed weight, ``transpose``):

* ``linear(x, w, b)``              -> x W^T + b                      (Linear forward)
* ``linear_gelu(x, w, b)``         -> (u, a): u = x W^T + b, a = gelu(u) computed in the epilogue
                                      (FFN up-projection: no separate activation pass over u)
* ``matmul_nt(a, b_t)``            -> a b_t^T                        (dgrad with b_t = W^T)
* ``matmul_nt_add_(c, a, b_t)``    -> c += a b_t^T in place          (residual-branch dgrad)
* ``gelu_bwd_gemm(dy, w_t, u, dbias)`` -> du = (dy w_t^T) * gelu'(u) plus the column sums of du
                                      (FFN down-projection dgrad with the GELU derivative and the
                                      up-projection's bias gradient in the epilogue)
* ``linear_act_grad(x, w, b)``     -> (g, a): a = gelu(u) and g = gelu'(u) (u = x W^T + b) from one
                                      exponential; g is stored instead of u
* ``mul_bwd_gemm(dy, w_t, g, dbias)`` -> du = (dy w_t^T) * g plus the column sums of du (the
                                      backward partner of ``linear_act_grad``: a multiply instead of
                                      the derivative's transcendental math)
* ``wgrad_tn(dy, x)``              -> fp32 split-K partials of dy^T x (weight gradient of a Linear:
                                      both operands row-major over the token dim; ``ops/csrc/wgrad.hip``,
                                      a ring-pipelined TN kernel with transposing LDS reads; one wave
                                      of workgroups; ``grad.splitk_reduce`` sums)

The kernel is the 256x256 8-phase LDS-DMA pipeline of cdna_hip_programming.md §5 (see the .hip
header).  Shapes must tile by 256 x 256 x 64 (``supported``); callers fall back to hipBLASLt +
the elementwise kernels otherwise.  bf16 only.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

import torch

from . import _lib

EPI_STORE, EPI_BIAS_GELU, EPI_GELU_BWD, EPI_ADD = 0, 1, 2, 3
EPI_BIAS_GELU_TANH, EPI_GELU_TANH_BWD, EPI_BIAS_RELU, EPI_RELU_BWD = 4, 5, 6, 7
EPI_BIAS_GELU_G, EPI_BIAS_GELU_TANH_G, EPI_MUL_BWD = 8, 9, 10
# activations with fused GEMM epilogues: erf GELU (BERT), its tanh approximation (GPT-2 / BLOOM
# "gelu_new") and ReLU (OPT) -> (forward epilogue, backward epilogue)
_ACT_EPI = {"gelu": (EPI_BIAS_GELU, EPI_GELU_BWD), "gelu_tanh": (EPI_BIAS_GELU_TANH, EPI_GELU_TANH_BWD),
            "relu": (EPI_BIAS_RELU, EPI_RELU_BWD)}
FUSED_ACTS = tuple(_ACT_EPI)
# activations whose forward epilogue can store the derivative instead of the pre-activation
_ACT_GRAD_EPI = {"gelu": EPI_BIAS_GELU_G, "gelu_tanh": EPI_BIAS_GELU_TANH_G}
GRAD_ACTS = tuple(_ACT_GRAD_EPI)

# DTD_GEMM=0 keeps every product on hipBLASLt (A/B runs); the model path checks ``enabled()``.
_ENABLED = [os.environ.get("DTD_GEMM", "1") == "1"]


# Which model products take the kernel (same-box A/B switches): the FFN up-projection forward with
# the GELU epilogue, and the FFN down-projection dgrad with the GELU-backward epilogue.
_FFN_FWD = [os.environ.get("DTD_GEMM_FFN_FWD", "1") == "1"]
_FFN_BWD = [os.environ.get("DTD_GEMM_FFN_BWD", "1") == "1"]
# The FFN up-projection stores gelu'(u) instead of u (the derivative's exp / rcp shared with the
# forward GELU; the backward epilogue is a multiply).  One extra bf16 rounding of the derivative.
_FFN_STORE_GRAD = [os.environ.get("DTD_GEMM_FFN_STORE_GRAD", "1") == "1"]
# Weight gradients on the ring-pipelined TN kernel (ops/csrc/wgrad.hip), default on: 1.2-1.29 PF/s
# against the library split-K bmm's 0.89-1.05 on the BERT-base weights (profiles/r5_s2_wgrad.jsonl),
# +4.6 % whole step (profiles/r5_s3_results.jsonl).  DTD_GEMM_WGRAD=0 keeps them on hipBLASLt.
_WGRAD = [os.environ.get("DTD_GEMM_WGRAD", "1") == "1"]
# DTD_GEMM_ALL=1: every transformer-layer projection on the hand-written kernels -- forward
# (gemm_bt + bias), input gradients (gemm_bt on the transposed weight), weight gradients (TN
# kernel, fp32 split-K partials) -- no vendor GEMM in the layers.  Off by default: the NT main loop
# runs at 0.86-0.92x of hipBLASLt's kernels on the plain products
# (profiles/r3_gemm_u2_experiment.jsonl); kept as the fully native compute path and for A/B runs.
_ALL = [os.environ.get("DTD_GEMM_ALL", "0") == "1"]
# Tile order of the persistent kernel: "dynamic" (default) claims tiles from a per-stream atomic
# queue, so workgroups delayed by CUs that another stream holds (RCCL on the comm stream, the
# attention-mask generator) take fewer tiles; "static" is the fixed round-robin order (A/B runs).
_SCHED = [os.environ.get("DTD_GEMM_SCHED", "dynamic")]
assert _SCHED[0] in ("dynamic", "static"), _SCHED[0]
_QUEUES: dict = {}
# epilogues whose dynamic-queue instantiation spills VGPRs in the main loop keep the static order
_STATIC_EPIS = frozenset({EPI_GELU_TANH_BWD})


def enabled() -> bool:
    return _ENABLED[0]


# The fused FFN kernels run one 256 x 256 tile per workgroup: below about one tile per CU (batch 1-4
# at seq 512: 32-96 tiles) most of the chip idles, and hipBLASLt's small-tile kernels plus the
# separate activation pass are faster (DTD_GEMM_FFN_MIN_TILES; default: the CU count).
_FFN_MIN_TILES = [int(os.environ.get("DTD_GEMM_FFN_MIN_TILES", "0")) or None]


def ffn_tiles_ok(M: int, N: int) -> bool:
    if _FFN_MIN_TILES[0] is None:
        _FFN_MIN_TILES[0] = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
    return (M // 256) * (N // 256) >= _FFN_MIN_TILES[0]


def ffn_fwd_enabled() -> bool:
    return _ENABLED[0] and _FFN_FWD[0]


def ffn_bwd_enabled() -> bool:
    return _ENABLED[0] and _FFN_BWD[0]


def ffn_store_grad_enabled() -> bool:
    return _ENABLED[0] and _FFN_FWD[0] and _FFN_BWD[0] and _FFN_STORE_GRAD[0]


def wgrad_enabled() -> bool:
    return _ENABLED[0] and (_WGRAD[0] or _ALL[0])


def set_wgrad(on: bool) -> None:
    _WGRAD[0] = bool(on)


def all_enabled() -> bool:
    return _ENABLED[0] and _ALL[0]


def set_all(on: bool) -> None:
    _ALL[0] = bool(on)


# fp32 (reference-precision) products on the hand-written f32-MFMA kernels (ops/csrc/gemm_f32.hip).
# DTD_GEMM_F32 = "wgrad" (default): the split-K weight gradients; "fwd": the forward products too;
# "1"/"all": every fp32 product; "0": none.  Round 5 (profiles/r5_s49_f32_gemm.jsonl, BERT-base fp32 b32 on one MI355X): the register-
# direct kernels run the weight gradients at 107-135 TF/s vs hipBLASLt's 98-132 at 16k tokens (118-131
# vs 64 at 32k) and the forward products at 121-146 vs 117-149 -- in the step the weight-gradient
# mode is at parity or better (190.1-191.4 k vs 189.9-190.7 k tokens/s) while every-product mode is
# 2 % behind (186.4 k; "fwd" mode 187.7-187.9 k vs 189.5 k): in the step the hand NT products take
# 41.6 ms against the library's 40.0 although they win in isolation, so forward / input gradients
# stay on the library by default.
_F32_MODE = os.environ.get("DTD_GEMM_F32", "wgrad")
_F32 = [_F32_MODE in ("1", "all", "fwd")]
_F32_WGRAD = [_F32_MODE in ("1", "all", "wgrad", "fwd")]
_F32_DG = [_F32_MODE in ("1", "all")]        # "fwd": forward + weight gradients, input gradients on the library
# fp32 input gradients: NT on the step's batched W^T copies (default; both operands in the blocked
# [row][k] layout, 0.86-0.89 MFMA-busy) or NN straight from W (DTD_GEMM_F32_DGRAD=nn: the [k][n]
# operand costs it 1-2 % of the step even with its loads landing in place, 183.2 k vs 186.5 k,
# profiles/r5_s49_f32_gemm.jsonl s66)
_F32_DGRAD_NN = os.environ.get("DTD_GEMM_F32_DGRAD", "nt") == "nn"


def set_f32(on: bool, wgrad: bool | None = None) -> None:
    """All fp32 products on the hand kernel (on) or none; ``wgrad`` sets the weight gradients
    separately (default: follow ``on``)."""
    _F32[0] = _F32_DG[0] = bool(on)
    _F32_WGRAD[0] = bool(on) if wgrad is None else bool(wgrad)


def set_f32_kernel(form: str = "auto") -> None:
    """Which hand-written fp32 form runs: "reg" (register-direct, one wave per workgroup), "lds"
    (LDS-staged, 2 workgroups per CU) or "auto" (the register form where its grid fills a round;
    ``DTD_GEMM_F32_KERNEL`` sets the process default)."""
    _lib.call("dtd_gemm_f32_set_kernel", {"auto": 0, "lds": 1, "reg": 2}[form])


def _ok32(t: torch.Tensor) -> bool:
    return (t is not None and t.is_cuda and t.dtype == torch.float32 and t.dim() == 2 and t.stride(1) == 1
            and t.stride(0) % 4 == 0 and t.data_ptr() % 16 == 0)


def f32_supported(M: int, N: int, K: int, *tensors, wgrad: bool = False) -> bool:
    if not ((_F32_WGRAD[0] if wgrad else _F32[0]) and all(_ok32(t) for t in tensors) and _lib.has("dtd_gemm_f32_nt")):
        return False
    return bool(_lib.lib().dtd_gemm_f32_supported(M, N, K))


def gemm_f32_nt(a: torch.Tensor, b: torch.Tensor, bias: torch.Tensor | None = None,
                out: torch.Tensor | None = None) -> torch.Tensor:
    """a . b^T (+ bias), fp32, exact f32 MFMA products; with ``out``: out += a . b^T (+ bias)."""
    M, K = a.shape
    N = b.shape[0]
    c = torch.empty((M, N), dtype=torch.float32, device=a.device) if out is None else out
    _lib.call("dtd_gemm_f32_nt", a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), c.data_ptr(), c.stride(0),
              _lib.ptr(bias), M, N, K, int(out is not None), _lib.stream())
    return c


def gemm_f32_nn(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """a . b for b [K, N] (the input gradient dY W straight from a Linear weight, no transposed
    copy), fp32; with ``out``: out += a . b."""
    M, K = a.shape
    N = b.shape[1]
    c = torch.empty((M, N), dtype=torch.float32, device=a.device) if out is None else out
    _lib.call("dtd_gemm_f32_nn", a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), c.data_ptr(), c.stride(0),
              M, N, K, int(out is not None), _lib.stream())
    return c


def gemm_f32_tn(a: torch.Tensor, b: torch.Tensor, splits: int | None = None) -> torch.Tensor:
    """fp32 partials [splits, M, N] of a^T b (a [K, M], b [K, N]) over contiguous K ranges."""
    K, M = a.shape
    N = b.shape[1]
    if splits is None:
        splits = _lib.lib().dtd_gemm_f32_tn_splits(M, N, K)
    part = torch.empty((splits, M, N), dtype=torch.float32, device=a.device)
    _lib.call("dtd_gemm_f32_tn", a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), part.data_ptr(), M, N, K,
              splits, _lib.stream())
    return part


# Plain bf16 products -- the Linear forward with bias, the NT input gradients, the residual-add input
# gradient -- on the one-wave-per-SIMD kernel (ops/csrc/gemm_w4.hip: 128 x 128 per wave, whole K-step
# fragment sets in registers, LDS-DMA into the buffer being drained, persistent across tiles).
# DTD_GEMM_W4=0 keeps them on hipBLASLt.  The residual-add form (EPI_ADD, the qkv input gradient) is
# opt-in (DTD_GEMM_W4_ADD=1): its epilogue must read the C tile, and with one wave per SIMD that
# read's latency is exposed (0.83x the library at T = 524288, profiles/r6_w4_sched.jsonl).
# The persistent grid is one workgroup per CU: with fewer than a few tiles per CU the tail and the
# one-tile prologue dominate and hipBLASLt's smaller macro tiles fill the chip better, so the dispatch
# takes the kernel only from DTD_GEMM_W4_MIN_TILES 256 x 256 tiles (default 4 per CU) up.
_W4 = [os.environ.get("DTD_GEMM_W4", "1") == "1"]
_W4_ADD = [os.environ.get("DTD_GEMM_W4_ADD", "0") == "1"]
_W4_MIN_TILES = [int(os.environ.get("DTD_GEMM_W4_MIN_TILES", "0")) or None]
# Long-K products (K = 3072: the fc2 forward and the fc1 input gradient) run 0.95-0.96x the library
# on it on every box measured (profiles/r6_w4_sched.jsonl, profiles/r6_w4nt.jsonl) while the
# K <= 2304 ones run 1.0-1.18x: the dispatch keeps K above DTD_GEMM_W4_MAX_K on hipBLASLt.
_W4_MAX_K = [int(os.environ.get("DTD_GEMM_W4_MAX_K", "2304"))]


def w4_enabled() -> bool:
    return _ENABLED[0] and _W4[0]


def set_w4(on: bool, add: bool | None = None) -> None:
    _W4[0] = bool(on)
    if add is not None:
        _W4_ADD[0] = bool(add)


def w4_supported(M: int, N: int, K: int, *tensors) -> bool:
    if not (all(_ok(t) for t in tensors) and _lib.has("dtd_gemm_w4")):
        return False
    return bool(_lib.lib().dtd_gemm_w4_supported(M, N, K))


def w4_min_tiles() -> int:
    if _W4_MIN_TILES[0] is None:
        _W4_MIN_TILES[0] = 4 * torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
    return _W4_MIN_TILES[0]


@contextlib.contextmanager
def hand_kernels_at_any_size(library: bool = True):
    """Within the block the one-wave-per-SIMD kernel and the fused FFN kernels take every product
    they tile, whatever its tile count (and with ``library=False`` the 8-wave kernel the rest it
    tiles): the prewarm's batch-1 step (utils/prewarm.py) then launches the kernels the real step
    will use."""
    prev = (_W4_MIN_TILES[0], _FFN_MIN_TILES[0], _ALL[0])
    _W4_MIN_TILES[0] = 1
    _FFN_MIN_TILES[0] = 1
    if not library:
        _ALL[0] = True
    try:
        yield
    finally:
        _W4_MIN_TILES[0], _FFN_MIN_TILES[0], _ALL[0] = prev


def _w4_pick(M: int, N: int, K: int, *tensors) -> bool:
    """The dispatch rule: kernel on, shape tiles, and enough tiles to fill the persistent grid."""
    return (w4_enabled() and K <= _W4_MAX_K[0] and (M // 256) * (N // 256) >= w4_min_tiles()
            and w4_supported(M, N, K, *tensors))


def gemm_w4(a: torch.Tensor, b: torch.Tensor, bias: torch.Tensor | None = None,
            out: torch.Tensor | None = None) -> torch.Tensor:
    """a . b^T (+ bias) on gemm_w4.hip; with ``out``: out += a . b^T in place (fp32 sum, one bf16
    rounding; no bias)."""
    M, K = a.shape
    N = b.shape[0]
    assert b.shape[1] == K, (a.shape, b.shape)
    if out is None:
        c = torch.empty((M, N), dtype=a.dtype, device=a.device)
        epi = EPI_STORE
    else:
        assert out.shape == (M, N) and bias is None, (out.shape, bias is None)
        c, epi = out, EPI_ADD
    _lib.call("dtd_gemm_w4", epi, a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), c.data_ptr(), c.stride(0),
              _lib.ptr(bias), M, N, K, _lib.stream())
    return c


def _bias_ok(b) -> bool:
    return b is None or (b.is_cuda and b.dtype == torch.bfloat16 and b.is_contiguous() and b.data_ptr() % 16 == 0)


def linear_any(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None) -> torch.Tensor:
    """F.linear, or a hand-written kernel: the fp32 one for fp32 operands, the bf16 one-wave-per-SIMD
    kernel (default) or the 8-wave one (all-native mode), when the shape tiles."""
    if (x.dtype == torch.float32 and x.dim() == 2 and f32_supported(x.shape[0], w.shape[0], x.shape[1], x, w)
            and (b is None or _ok1d32(b))):
        return gemm_f32_nt(x, w, b)
    if x.dim() == 2 and _bias_ok(b) and _w4_pick(x.shape[0], w.shape[0], x.shape[1], x, w):
        return gemm_w4(x, w, b)
    if all_enabled() and x.dim() == 2 and supported(x.shape[0], w.shape[0], x.shape[1], x, w) and (
            b is None or (b.is_cuda and b.dtype == torch.bfloat16 and b.is_contiguous())):
        return linear(x, w, b)
    return torch.nn.functional.linear(x, w, b)


def set_enabled(on: bool) -> None:
    _ENABLED[0] = bool(on)


# Projection GEMM + bias + hidden dropout + residual + LayerNorm in one kernel (ops/csrc/gemm_ln.hip)
# for the post-LN output sublayers (attention output, FFN output) at hidden size 768.
_LN_FUSED = [os.environ.get("DTD_GEMM_LN", "0") == "1"]


def set_ln_fused(on: bool) -> None:
    _LN_FUSED[0] = bool(on)


def ln_fused_enabled() -> bool:
    return _LN_FUSED[0]


def linear_ln_supported(x: torch.Tensor, w: torch.Tensor, r: torch.Tensor, *vecs) -> bool:
    """Shape / layout contract of ``linear_ln``: bf16, 16-byte aligned rows, N = 768, M % 128 == 0."""
    if not (_ok(x) and _ok(w) and _ok(r) and _lib.has("dtd_gemm_ln")):
        return False
    if not all(v is None or (v.is_cuda and v.dtype == torch.bfloat16 and v.is_contiguous()
                             and v.data_ptr() % 16 == 0) for v in vecs):
        return False
    M, K = x.shape
    return (w.shape[1] == K and r.shape == (M, w.shape[0]) and
            bool(_lib.lib().dtd_gemm_ln_supported(M, w.shape[0], K, x.stride(0), w.stride(0), r.stride(0),
                                                   w.shape[0])))


def linear_ln(x, w, b, r, gamma, beta, eps: float, p: float, rng, sid: int, store_z: bool = False):
    """``out = LayerNorm(r + dropout(x @ w.T + b))`` in one kernel; the dropout keep law and the
    (z, out, mean, rstd) result of ``ops.functional.ln_fwd(x @ w.T + b, r, ...)``, with the projection
    output rounded to bf16 once, as a stored Linear output would be."""
    M = x.shape[0]
    N = w.shape[0]
    out = torch.empty((M, N), dtype=x.dtype, device=x.device)
    z = torch.empty_like(out) if store_z else None
    mean = torch.empty(M, dtype=torch.float32, device=x.device)
    rstd = torch.empty_like(mean)
    _lib.call("dtd_gemm_ln", x.data_ptr(), w.data_ptr(), _lib.ptr(b), r.data_ptr(), gamma.data_ptr(),
              beta.data_ptr(), out.data_ptr(), _lib.ptr(z), mean.data_ptr(), rstd.data_ptr(), M, N, x.shape[1],
              x.stride(0), w.stride(0), r.stride(0), N, float(eps), float(p), rng.state.data_ptr(), sid,
              _lib.stream())
    return z, out, mean, rstd


def _ok(t: torch.Tensor) -> bool:
    return (t is not None and t.is_cuda and t.dtype == torch.bfloat16 and t.dim() == 2 and t.stride(1) == 1
            and t.stride(0) % 8 == 0 and t.data_ptr() % 16 == 0)


def supported(M: int, N: int, K: int, *tensors) -> bool:
    if not all(_ok(t) for t in tensors):
        return False
    if not _lib.has("dtd_gemm_bt"):
        return False
    return bool(_lib.lib().dtd_gemm_bt_supported(M, N, K))


def set_sched(mode: str) -> None:
    assert mode in ("dynamic", "static"), mode
    _SCHED[0] = mode


def _queue() -> int | None:
    """The current stream's tile queue (9 int32, zero at rest: the kernel's last workgroup
    re-zeroes it).  One queue per (device, stream): launches on one stream are ordered, launches
    on different streams may overlap and must not share counters."""
    if _SCHED[0] != "dynamic":
        return None
    s = torch.cuda.current_stream()   # the stream the kernel is launched on (_lib.stream())
    key = (s.device_index, s.cuda_stream)
    q = _QUEUES.get(key)
    if q is None:
        q = _QUEUES[key] = torch.zeros(16, dtype=torch.int32, device=torch.device("cuda", s.device_index))
    return q.data_ptr()


def _call(epi, a, b, c, c2=None, u=None, bias=None, part=None):
    M, K = a.shape
    N = b.shape[0]
    assert b.shape[1] == K and c.shape == (M, N), (a.shape, b.shape, c.shape)
    _lib.call("dtd_gemm_bt", epi, a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), c.data_ptr(), c.stride(0),
              _lib.ptr(c2), _lib.ptr(u), u.stride(0) if u is not None else 0, _lib.ptr(bias), _lib.ptr(part),
              M, N, K, None if epi in _STATIC_EPIS else _queue(), _lib.stream())


def gemm_bt(a: torch.Tensor, b: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    c = torch.empty((a.shape[0], b.shape[0]), dtype=a.dtype, device=a.device)
    _call(EPI_STORE, a, b, c, bias=bias)
    return c


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None) -> torch.Tensor:
    return gemm_bt(x, w, b)


def matmul_nt(a: torch.Tensor, b_t: torch.Tensor) -> torch.Tensor:
    return gemm_bt(a, b_t)


def matmul_nt_add_(c: torch.Tensor, a: torch.Tensor, b_t: torch.Tensor) -> torch.Tensor:
    """c += a . b_t^T (fp32 sum of the product and c, one bf16 rounding)."""
    _call(EPI_ADD, a, b_t, c)
    return c


def linear_gelu(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None, act: str = "gelu"):
    """(u, a) = (x W^T + b, act(u)) in one kernel (the activation of the stored bf16 u, as the
    unfused activation kernel computes it); ``act`` one of FUSED_ACTS."""
    assert act in FUSED_ACTS, act
    M, N = x.shape[0], w.shape[0]
    u = torch.empty((M, N), dtype=x.dtype, device=x.device)
    a = torch.empty_like(u)
    _call(_ACT_EPI[act][0], x, w, u, c2=a, bias=b)
    return u, a


def linear_act_grad(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None, act: str = "gelu"):
    """(g, a) = (act'(u), act(u)) with u = bf16(x W^T + b), in one kernel; ``act`` one of
    GRAD_ACTS.  u itself is not stored: the backward takes g (``mul_bwd_gemm``)."""
    assert act in GRAD_ACTS, act
    M, N = x.shape[0], w.shape[0]
    g = torch.empty((M, N), dtype=x.dtype, device=x.device)
    a = torch.empty_like(g)
    _call(_ACT_GRAD_EPI[act], x, w, g, c2=a, bias=b)
    return g, a


def mul_bwd_gemm(dy: torch.Tensor, w_t: torch.Tensor, g: torch.Tensor, dbias=None):
    """du = bf16(dy . w_t^T) * g with g = act'(u) from ``linear_act_grad``; ``dbias`` as in
    ``gelu_bwd_gemm``."""
    return _act_bwd_gemm(EPI_MUL_BWD, dy, w_t, g, dbias)


def gelu_bwd_gemm(dy: torch.Tensor, w_t: torch.Tensor, u: torch.Tensor, dbias=None, act: str = "gelu"):
    """du = bf16(dy . w_t^T) * act'(u); ``w_t`` is the down-projection weight transposed to
    [ffn, hidden] (K-contiguous).  ``dbias`` (dst, acc) receives the column sums of du; ``act``
    one of FUSED_ACTS."""
    assert act in FUSED_ACTS, act
    return _act_bwd_gemm(_ACT_EPI[act][1], dy, w_t, u, dbias)


def _act_bwd_gemm(epi: int, dy: torch.Tensor, w_t: torch.Tensor, u: torch.Tensor, dbias):
    from .functional import _finalize
    M, N = dy.shape[0], w_t.shape[0]
    du = torch.empty((M, N), dtype=dy.dtype, device=dy.device)
    part = None
    if dbias is not None:
        nrows = _lib.lib().dtd_gemm_bt_part_rows(M)
        part = torch.empty((nrows, N), dtype=torch.float32, device=dy.device)
    _call(epi, dy, w_t, du, u=u, part=part)
    if part is not None:
        dst, acc = dbias
        _finalize(part, part.shape[0], N, (dst, acc), acc)
    return du


def transpose(w: torch.Tensor) -> torch.Tensor:
    """w^T as a new contiguous bf16 tensor (LDS-tiled transpose kernel)."""
    assert w.dim() == 2 and w.is_contiguous() and w.dtype == torch.bfloat16
    out = torch.empty((w.shape[1], w.shape[0]), dtype=w.dtype, device=w.device)
    _lib.call("dtd_transpose_bf16", w.data_ptr(), out.data_ptr(), w.shape[0], w.shape[1], _lib.stream())
    return out


# Input-gradient products as "NT" GEMMs (DTD_DGRAD_NT=0: dy @ W): dX = dY W computed as
# F.linear(dY, W^T) with W^T materialised by `transpose` (~1-4 us a BERT-base weight), so hipBLASLt
# runs its forward-layout kernels instead of the NN ones -- at BERT-base b256 the qkv / o / fc1
# input gradients take 322-335 / 126-135 / 428-441 us that way vs 390 / 159-166 / 501-508 us
# (profiles/r3_gemm_split_experiment.jsonl: bench_gemm8's "dgrad_*" hipBLASLt column vs
# bench_gemm_v2's, same session).
_DGRAD_NT = [os.environ.get("DTD_DGRAD_NT", "1") == "1"]


# A fresh transpose moves 4 bytes per weight element; the input-gradient GEMM does 2 * rows flops per
# element.  With few rows (a micro-batch of 512 tokens on a ZeRO-3-gathered weight, whose transpose
# cannot be prepared ahead) the transpose costs more than the NT form saves -- 11 ms of a 165 ms
# step on the 16 B-parameter ZeRO-3 model (profiles/r6_mp3_step_window.txt) -- so below this many
# rows an uncached weight keeps the NN form (dy @ W).
_DGRAD_NT_MIN_ROWS = int(os.environ.get("DTD_DGRAD_NT_MIN_ROWS", "8192"))


def transposed_for_dgrad(w: torch.Tensor, rows: int | None = None) -> torch.Tensor | None:
    """W^T contiguous for the NT input-gradient form, or None (keep dy @ W).  ``rows``: the
    gradient's row count, for the fresh-transpose cost rule above."""
    if not (_DGRAD_NT[0] and w.is_cuda and w.dtype == torch.bfloat16 and w.dim() == 2 and w.is_contiguous()):
        return None
    if w.shape[0] % 8:   # W^T rows (the GEMM's K) would not be 16-byte aligned (e.g. a 28996-row vocabulary)
        return None
    if rows is not None and rows < _DGRAD_NT_MIN_ROWS:
        e = _WT_CACHE.get(id(w))
        if not (e is not None and e[0] is w and e[1] == w.data_ptr()):
            return None
    return transposed(w)


# W^T of the weights of one backward, made by ONE batched launch at its start
# (prepare_transposes) instead of one small launch per weight as each layer's backward reaches it
# (49 launches of ~6 us at BERT-base).  Keyed by the parameter object and checked against its
# current storage address; cleared at the start of every forward (the weights change only at the
# optimizer step, which precedes the next forward).
_WT_CACHE: dict = {}
_WT_BATCH = [os.environ.get("DTD_WT_BATCH", "1") == "1"]


def clear_transposes() -> None:
    _WT_CACHE.clear()


def _batchable(w: torch.Tensor, dev) -> bool:
    return (w.is_cuda and w.device == dev and w.dtype == torch.bfloat16 and w.dim() == 2 and w.is_contiguous()
            and w.numel() > 0 and w.shape[0] % 8 == 0 and w.shape[1] % 8 == 0 and w.data_ptr() % 16 == 0)


def _batchable32(w: torch.Tensor, dev) -> bool:
    return (_F32_DG[0] and w.is_cuda and w.device == dev and w.dtype == torch.float32 and w.dim() == 2
            and w.is_contiguous() and w.numel() > 0 and w.shape[0] % 4 == 0 and w.shape[1] % 4 == 0
            and w.data_ptr() % 16 == 0)


def prepare_transposes(weights) -> None:
    """Transpose every eligible weight of ``weights`` (resident, on the current device) in batched
    launches of up to 64 -- bf16 weights, and fp32 ones when the hand-written fp32 GEMMs are on;
    transposed() / the fp32 input-gradient path then take the cached copies."""
    if not (_WT_BATCH[0] and _lib.has("dtd_transpose_many")):
        return
    if any(w.numel() == 0 for w in weights):
        return   # partitioned parameters (ZeRO-3 releases them between uses): per-call transposes
    dev = torch.device("cuda", torch.cuda.current_device())
    for fn, ok in (("dtd_transpose_many", _batchable), ("dtd_transpose_many_f32", _batchable32)):
        if not _lib.has(fn):
            continue
        todo = [w for w in weights if ok(w, dev) and id(w) not in _WT_CACHE]
        for k in range(0, len(todo), 64):
            chunk = todo[k:k + 64]
            outs = [torch.empty((w.shape[1], w.shape[0]), dtype=w.dtype, device=w.device) for w in chunk]
            n = len(chunk)
            ins_a = (ctypes.c_void_p * n)(*[w.data_ptr() for w in chunk])
            outs_a = (ctypes.c_void_p * n)(*[o.data_ptr() for o in outs])
            rows_a = (ctypes.c_int * n)(*[w.shape[0] for w in chunk])
            cols_a = (ctypes.c_int * n)(*[w.shape[1] for w in chunk])
            _lib.call(fn, ins_a, outs_a, rows_a, cols_a, n, _lib.stream())
            for w, o in zip(chunk, outs):
                _WT_CACHE[id(w)] = (w, w.data_ptr(), o)


def _t32(w: torch.Tensor) -> torch.Tensor | None:
    """W^T of an fp32 weight from this backward's batched transposes (handed out once), or None."""
    e = _WT_CACHE.pop(id(w), None)
    if e is not None and e[0] is w and e[1] == w.data_ptr():
        return e[2]
    return None


def transposed(w: torch.Tensor) -> torch.Tensor:
    """W^T: the copy prepare_transposes made for this backward (handed out once: the entry is
    dropped, so each copy is freed right after its layer's input-gradient GEMM instead of living
    until the next forward), else a fresh transpose."""
    e = _WT_CACHE.pop(id(w), None)
    if e is not None and e[0] is w and e[1] == w.data_ptr():
        return e[2]
    return transpose(w)


def dgrad_nt_enabled() -> bool:
    return _DGRAD_NT[0]


def _ok1d32(t: torch.Tensor) -> bool:
    return t.is_cuda and t.dtype == torch.float32 and t.dim() == 1 and t.is_contiguous() and t.data_ptr() % 16 == 0


def dgrad(dy: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """dy @ w for a Linear weight w [out, in], through the NT form when it applies (the
    hand-written kernel in the all-native mode; the fp32 kernel for fp32 operands)."""
    if (dy.dtype == torch.float32 and dy.dim() == 2 and _F32_DG[0]
            and f32_supported(dy.shape[0], w.shape[1], dy.shape[1], dy, w)):
        wt = _t32(w)
        return gemm_f32_nn(dy, w) if wt is None or _F32_DGRAD_NN else gemm_f32_nt(dy, wt)
    wt = transposed_for_dgrad(w, dy.shape[0] if dy.dim() == 2 else None)
    if wt is None:
        return dy @ w
    if dy.dim() == 2 and _w4_pick(dy.shape[0], wt.shape[0], dy.shape[1], dy, wt):
        return gemm_w4(dy, wt)
    if all_enabled() and dy.dim() == 2 and supported(dy.shape[0], wt.shape[0], dy.shape[1], dy, wt):
        return matmul_nt(dy, wt)
    return torch.nn.functional.linear(dy, wt)


def dgrad_add_(c: torch.Tensor, dy: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """c += dy @ w in place (residual-branch input gradient), NT form when it applies."""
    if (dy.dtype == torch.float32 and dy.dim() == 2 and _F32_DG[0]
            and f32_supported(dy.shape[0], w.shape[1], dy.shape[1], dy, w, c)):
        wt = _t32(w)
        return gemm_f32_nn(dy, w, out=c) if wt is None or _F32_DGRAD_NN else gemm_f32_nt(dy, wt, out=c)
    wt = transposed_for_dgrad(w, dy.shape[0] if dy.dim() == 2 else None)
    if wt is None:
        return c.addmm_(dy, w)
    if _W4_ADD[0] and dy.dim() == 2 and _w4_pick(dy.shape[0], wt.shape[0], dy.shape[1], dy, wt, c):
        return gemm_w4(dy, wt, out=c)
    if all_enabled() and dy.dim() == 2 and supported(dy.shape[0], wt.shape[0], dy.shape[1], dy, wt, c):
        return matmul_nt_add_(c, dy, wt)
    return c.addmm_(dy, wt.t())


def wgrad_supported(dy: torch.Tensor, x: torch.Tensor) -> bool:
    """Contract of the weight-gradient kernel (``ops/csrc/wgrad.hip``): dy [T, o], x [T, i] bf16
    row-major views on the GPU, o and i multiples of 256, T a multiple of 32."""
    if not (_ok(dy) and _ok(x)) or dy.shape[0] != x.shape[0] or not _lib.has("dtd_wgrad_tn"):
        return False
    T, o, i = dy.shape[0], dy.shape[1], x.shape[1]
    if not _lib.lib().dtd_wgrad_tn_supported(o, i, T):
        return False
    # a K-range's rows must fit the kernel's 32-bit buffer offsets
    splits = int(_lib.lib().dtd_wgrad_tn_splits(o, i, T))
    rows = -(-T // 32 // splits) * 32
    return rows * max(dy.stride(0), x.stride(0)) * 2 < 0x7FFFFFFF


def wgrad_tn(dy: torch.Tensor, x: torch.Tensor, splits: int | None = None, variant: int = 0) -> torch.Tensor:
    """fp32 partials [splits, o, i] of dy^T x over contiguous token ranges (``wgrad.hip``: LDS ring
    of 32-token stages; ``variant`` = ring depth 4 or 5, 0 = the default depth)."""
    T, o = dy.shape
    i = x.shape[1]
    if splits is None:
        splits = _lib.lib().dtd_wgrad_tn_splits(o, i, T)
    part = torch.empty((splits, o, i), dtype=torch.float32, device=dy.device)
    _lib.call("dtd_wgrad_tn", variant, dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), part.data_ptr(), o, i,
              T, splits, _lib.stream())
    return part


# Tall-K input gradient of a big-vocabulary LM head, dX = dLogits [M, V] . E [V, h] at small M
# (bloom-560m at micro-batch 1: M = 511, V = 250880): the library's one-pass GEMM has ~128 output
# tiles for a 250880-long reduction.  The K-split form runs it as ONE strided-batch GEMM over
# `s` contiguous vocabulary ranges with fp32 partials (hipBLASLt's bf16 x bf16 -> fp32 batched
# product) plus one sum.  Measured on one MI355X (profiles/r6_head_splitk.json): 511 x 250880 x
# 1024 868 -> 281 us (s = 16), 2047 rows 1744 -> 797 us (s = 8), 511 x 50304 x 768 180 -> 64 us
# (s = 16); the bloom-560m ZeRO-3 step 42.6-44.8 k -> 45.3-46.1 k tokens/s.
# DTD_HEAD_SPLITK: "auto" (default: 16 ranges up to 1024 rows, 8 up to 4096, off above), a fixed
# number of ranges, or 0 (off: the one-pass GEMM).
_HS = os.environ.get("DTD_HEAD_SPLITK", "auto")
_HEAD_SPLITK = [-1 if _HS == "auto" else int(_HS)]


def set_head_splitk(splits: int) -> None:
    """Number of vocabulary ranges of the LM-head input gradient; -1 = auto, 0 = off."""
    _HEAD_SPLITK[0] = int(splits)


def head_splits(M: int, V: int, h: int) -> int:
    s = _HEAD_SPLITK[0]
    if s < 0:
        s = 16 if M <= 1024 else 8 if M <= 4096 else 0
    while s > 1 and V % s:
        s //= 2
    return s if s > 1 and V // s >= 4 * h and M * h <= (1 << 22) else 0


def head_dgrad(dlogits: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """dlogits [M, V] @ w [V, h]; K-split when the output is small against the reduction."""
    M, V = dlogits.shape
    h = w.shape[1]
    s = head_splits(M, V, h)
    if (s and dlogits.is_cuda and dlogits.is_contiguous() and w.is_contiguous()
            and dlogits.dtype in (torch.bfloat16, torch.float16) and w.dtype == dlogits.dtype):
        part = torch.bmm(dlogits.view(M, s, V // s).transpose(0, 1), w.view(s, V // s, h), out_dtype=torch.float32)
        return part.sum(0).to(dlogits.dtype)
    return dlogits @ w
