"""Direct parameter-gradient emission for the fused (hand-written backward) modules.

The fused modules' backward passes write weight/bias gradients straight into their final
storage instead of returning them to autograd:

* if the parameter has ``main_grad`` (a view into a flat gradient buffer owned by the DDP /
  ZeRO engine, ``parallel/flat.py``), the wgrad GEMM writes into that view with
  beta = 0 on the first contribution of the step and beta = 1 afterwards (tied weights,
  gradient accumulation) -- no AccumulateGrad copy, no separate bucket-flatten pass;
* otherwise the gradient lands in ``param.grad`` (created on first use), so any stock
  ``torch.optim`` optimizer works with the fused modules too.

After each contribution ``grad_done`` calls the owner's ready hook (the reducer counts
contributions per parameter and launches a bucket's collective once the bucket is complete,
overlapping communication with the rest of backward -- the role of DDP's C++ Reducer,
SURVEY.md D3).
"""
from __future__ import annotations

import os

import torch


def grad_dst(p: torch.Tensor):
    """(destination tensor, accumulate?) for the next gradient contribution of ``p``."""
    pre = getattr(p, "_dtd_pre_write_hook", None)
    if pre is not None:  # ZeRO-2/3: materialise the landing bucket on first write
        pre(p)
    mg = getattr(p, "main_grad", None)
    if mg is not None:
        return mg, bool(getattr(p, "_dtd_touched", False))
    if p.grad is None:
        p.grad = torch.empty_like(p)
        return p.grad, False
    return p.grad, True


_COUNTING = [True]


class no_use_counting:
    """Context (activation recompute) in which forward passes do not register new
    gradient contributions with the reducer."""

    def __enter__(self):
        self._prev = _COUNTING[0]
        _COUNTING[0] = False

    def __exit__(self, *a):
        _COUNTING[0] = self._prev


def note_use(params) -> None:
    """Called by fused forwards: each use of a tracked parameter is one expected gradient
    contribution in the coming backward (tied weights are used twice)."""
    if not _COUNTING[0] or not torch.is_grad_enabled():
        return
    for p in params:
        exp = getattr(p, "_dtd_expect", None)
        if exp is not None:          # owner counts in the native tracker (runtime/)
            exp(p)
        elif getattr(p, "_dtd_ready_hook", None) is not None:
            p._dtd_pending = getattr(p, "_dtd_pending", 0) + 1


def grad_done(p: torch.Tensor) -> None:
    if getattr(p, "main_grad", None) is not None:
        p._dtd_touched = True
    hook = getattr(p, "_dtd_ready_hook", None)
    if hook is not None:
        hook(p)


def gemm_into(dst: torch.Tensor, a: torch.Tensor, b: torch.Tensor, acc: bool) -> None:
    """dst (+)= a @ b with fp32 accumulation (hipBLASLt on GPU).  Supports a bf16 product
    accumulated into an fp32 destination (fp32 main_grad) via ``out_dtype``."""
    if dst.dtype == a.dtype:
        dst.addmm_(a, b, beta=1.0 if acc else 0.0)
    elif dst.is_cuda:
        torch.addmm(dst, a, b, beta=1.0 if acc else 0.0, out_dtype=dst.dtype, out=dst)
    else:
        r = a.float() @ b.float()
        if acc:
            dst.add_(r)
        else:
            dst.copy_(r)


def emit_gemm_grad(p: torch.Tensor, a: torch.Tensor, b: torch.Tensor) -> None:
    dst, acc = grad_dst(p)
    gemm_into(dst, a, b, acc)
    grad_done(p)


def wgrad_splits(tokens: int, out_f: int, in_f: int) -> int:
    """K-split factor for dW = dY^T X.  The output of a weight-gradient GEMM is small (a
    768x3072 weight is 144 tiles of 128x128) while K = tokens is huge, so one GEMM leaves most
    of the 256 CUs idle.  Splitting K into s slices (one batched GEMM, then an fp32 sum) until
    there are >= 512 output tiles measured 1.6-2.6x faster on MI355X at 16k tokens
    (scripts/bench_gemm.py); at <= 4k tokens a single GEMM is best.  At 64k tokens (b128) slices
    of 4096 tokens (s = 16) beat the tile-count rule by 6-12 % per GEMM in isolation
    (scripts/wgrad_sweep.py: QKV 270 -> 253 us, FC1/FC2 333 -> 317 us with fp32 partials,
    235 / 294 us with bf16 partials)."""
    if tokens < 8192:
        return 1
    tiles = -(-out_f // 128) * -(-in_f // 128)
    s = 1
    while tiles * s < 512 and s < 16 and tokens % (2 * s) == 0 and tokens // (2 * s) >= 1024:
        s *= 2
    while s < 16 and tokens // (2 * s) >= 4096 and tokens % (2 * s) == 0:
        s *= 2
    return s


class _AsyncWgrad:
    """Side stream for weight-gradient GEMMs (opt-in, ``set_async_wgrad``).

    In a layer's backward the wgrad GEMMs (compute-bound MFMA work) depend only on tensors the
    dgrad chain has already produced, and nothing in the layer's backward reads their output.
    Issued on a second HIP stream they run concurrently with the memory- / latency-bound
    kernels of the dgrad chain (activation and LayerNorm backward, attention backward).  The
    reducer joins the side stream (``join_async_wgrad``) before it reads gradients: before a
    bucket's collective and before the optimizer."""

    def __init__(self):
        self.enabled = False
        self.defer_finalize = False
        self.streams: dict = {}
        self.pending = False
        self.hold: list = []      # inputs of side-stream GEMMs, freed once the side stream is joined

    def stream(self, device) -> torch.cuda.Stream:
        s = self.streams.get(device)
        if s is None:
            s = self.streams[device] = torch.cuda.Stream(device)
        return s


_ASYNC = _AsyncWgrad()


def set_async_wgrad(enabled: bool) -> None:
    _ASYNC.enabled = bool(enabled)


def async_wgrad_enabled() -> bool:
    return _ASYNC.enabled


def set_defer_finalize(enabled: bool) -> None:
    """While on (a DDP backward window: DDP.forward -> DDP.finish), gradient column-sum
    finalizes run on the async-gradient side stream (ops/functional.py::_finalize_stream)."""
    _ASYNC.defer_finalize = bool(enabled)


def finalize_side_stream(device):
    if not _ASYNC.defer_finalize:
        return None
    _ASYNC.pending = True
    return _ASYNC.stream(torch.device(device))


def hold_until_join(t: torch.Tensor) -> None:
    """Keep ``t`` (read by side-stream work) alive until ``join_async_wgrad``."""
    _ASYNC.hold.append(t)


def join_async_wgrad(device=None) -> None:
    """Make the current stream wait for every weight-gradient GEMM issued so far."""
    if not _ASYNC.pending:
        return
    for dev, s in _ASYNC.streams.items():
        if device is None or torch.device(device) == dev:
            torch.cuda.current_stream(dev).wait_stream(s)
    _ASYNC.pending = False
    _ASYNC.hold.clear()


def emit_wgrad(p: torch.Tensor, dy: torch.Tensor, x: torch.Tensor, async_ok: bool = False) -> None:
    """p.grad-slot (+)= dy^T @ x for a Linear weight [out, in]; dy [T, out], x [T, in].
    ``async_ok``: the caller guarantees that nothing else writes this parameter's gradient
    before the reducer joins the side stream (per-layer Linear weights), so the GEMM may run
    on the async-wgrad stream when that is enabled."""
    if async_ok and _ASYNC.enabled and dy.is_cuda:
        side = _ASYNC.stream(dy.device)
        side.wait_stream(torch.cuda.current_stream(dy.device))
        with torch.cuda.stream(side):
            _emit_wgrad(p, dy, x)
        # keep the inputs alive until the compute stream has joined the side stream (their memory
        # is then reused in stream order).  record_stream() instead left one allocator event per
        # freed block on the side stream, and the eager step slowed down step after step with the
        # host blocked inside kernel launches: 91 / 203 / 794 ms per step after 2 / 10 / 20 steps
        hold_until_join(dy)
        hold_until_join(x)
        _ASYNC.pending = True
        grad_done(p)
        return
    _emit_wgrad(p, dy, x)
    grad_done(p)


# Token count from which the weight gradients take wgrad.hip (below: hipBLASLt, split-K bmm from
# 8192, one GEMM under it); DTD_WGRAD_MIN_T.  At the reference's small batches the kernel loses:
# b4 graph 352-354 k vs 384-385 k tokens/s, bloom-560m b1 37.7 k vs 42.0 k with T >= 512
# (profiles/r6_wgrad_min_t.jsonl).
_WGRAD_MIN_T = [int(os.environ.get("DTD_WGRAD_MIN_T", "8192"))]


def _emit_wgrad(p: torch.Tensor, dy: torch.Tensor, x: torch.Tensor) -> None:
    dst, acc = grad_dst(p)
    T, o = dy.shape
    i = x.shape[1]
    if dy.is_cuda and dy.dtype == torch.float32:
        from . import gemm as G
        if G.f32_supported(o, i, T, dy, x, wgrad=True):
            # reference-precision path: the f32-MFMA TN kernel, fp32 split-K partials
            splitk_reduce(G.gemm_f32_tn(dy, x), dst, acc)
            return
    if dy.is_cuda and T >= _WGRAD_MIN_T[0]:
        from . import gemm as G
        if G.wgrad_enabled() and G.wgrad_supported(dy, x):
            # ring-pipelined TN MFMA kernel (ops/csrc/wgrad.hip): fp32 split-K partials, one wave
            # of workgroups, 1.2-1.29 PF/s on the BERT-base weights at 131k tokens against the
            # library's 0.89-1.05 (profiles/r5_s2_wgrad.jsonl)
            splitk_reduce(G.wgrad_tn(dy, x), dst, acc)
            return
    s = wgrad_splits(T, o, i) if dy.is_cuda else 1
    if s == 1:
        gemm_into(dst, dy.t(), x, acc)
    else:
        a, b = dy.view(s, T // s, o).transpose(1, 2), x.view(s, T // s, i)
        part = _bmm_partials(a, b, fp32=dst.dtype == torch.float32)
        splitk_reduce(part, dst, acc)


_F32_PARTIALS = [os.environ.get("DTD_WGRAD_F32_PARTIALS", "1") == "1"]


def _bmm_partials(a: torch.Tensor, b: torch.Tensor, fp32: bool = True) -> torch.Tensor:
    """Batched K-slice products.  The partials carry the destination's precision: fp32 (when
    hipBLASLt offers the bf16->fp32 batched GEMM) for an fp32 gradient buffer, the input dtype
    for a bf16 one -- there the final bf16 rounding dominates anyway (relative error 1.7e-3 with
    fp32 partials vs 2.4e-3 with bf16 ones at 16 x 1024-token slices), and half the partial
    traffic is +1.5 % BERT-base b128 throughput on MI355X (scripts/ab.py, same box)."""
    if fp32 and _F32_PARTIALS[0] and a.dtype != torch.float32:
        try:
            return torch.bmm(a, b, out_dtype=torch.float32)
        except (RuntimeError, TypeError):
            _F32_PARTIALS[0] = False
    return torch.bmm(a, b)


def splitk_reduce(part: torch.Tensor, dst: torch.Tensor, acc: bool) -> None:
    """dst (+)= part.sum(0) in fp32, one fused pass on GPU (ops/csrc/reduce.hip)."""
    if dst.is_cuda:
        from . import _lib
        assert part.is_contiguous() and dst.is_contiguous() and part[0].numel() == dst.numel()
        _lib.call("dtd_splitk_reduce", part.data_ptr(), _lib.dt(part), part.shape[0], dst.numel(),
                  dst.data_ptr(), _lib.dt(dst), int(acc), _lib.stream())
        return
    tot = part.sum(0, dtype=torch.float32)
    if acc:
        dst.add_(tot.view_as(dst))
    else:
        dst.copy_(tot.view_as(dst))


def emit_grad(p: torch.Tensor, g: torch.Tensor) -> None:
    dst, acc = grad_dst(p)
    if acc:
        dst.add_(g.to(dst.dtype))
    else:
        dst.copy_(g)
    grad_done(p)
