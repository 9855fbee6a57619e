"""Functional front-end of the fused ops.

Each function runs the gfx950 HIP kernel for CUDA(HIP) tensors and the PyTorch reference
(same semantics and dropout masks as the kernels) for CPU tensors.  Parameter-gradient outputs
are written into caller-provided destination tensors (``main_grad`` views of the flat
gradient buffers, see ``parallel/flat.py``) with overwrite-or-accumulate semantics,
which is how the framework avoids a separate gradient-accumulation pass.
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib
from .rng import RngState, keep_mask

ACT_CODES = {"none": 0, "gelu": 1, "gelu_tanh": 2, "relu": 3}
IGNORE_INDEX = -100


def _on_gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


def _c(t):
    return None if t is None else t.contiguous()


# --------------------------------------------------------------------------------------
# dropout
# --------------------------------------------------------------------------------------
def _ref_dropout(x: torch.Tensor, p: float, rng: RngState, sid: int) -> torch.Tensor:
    if p <= 0.0:
        return x
    seed, step = (int(v) for v in rng.state.tolist())
    keep = keep_mask(x.numel(), p, seed, step, sid, device=x.device).view_as(x)
    return (x.float() * keep / (1.0 - p)).to(x.dtype)


def dropout(x: torch.Tensor, p: float, rng: RngState, sid: int) -> torch.Tensor:
    if p <= 0.0:
        return x
    if not _on_gpu(x):
        return _ref_dropout(x, p, rng, sid)
    x = x.contiguous()
    y = torch.empty_like(x)
    _lib.call("dtd_dropout", _lib.dt(x), x.data_ptr(), None, y.data_ptr(), x.numel(), float(p),
              rng.state.data_ptr(), sid, _lib.stream())
    return y


def dropout_add(x: torch.Tensor, res: torch.Tensor, p: float, rng: RngState, sid: int) -> torch.Tensor:
    """res + dropout(x) in one pass (sum in fp32); same keep bits as ``dropout(x, p, rng, sid)``."""
    if not _on_gpu(x):
        return res + dropout(x, p, rng, sid)
    assert x.shape == res.shape and x.dtype == res.dtype
    x, res = x.contiguous(), res.contiguous()
    y = torch.empty_like(x)
    _lib.call("dtd_dropout", _lib.dt(x), x.data_ptr(), res.data_ptr(), y.data_ptr(), x.numel(), float(p),
              rng.state.data_ptr(), sid, _lib.stream())
    return y


# --------------------------------------------------------------------------------------
# residual + dropout + LayerNorm
# --------------------------------------------------------------------------------------
def ln_fwd(y, r, gamma, beta, eps: float, p: float, rng: RngState, sid: int, store_z: bool = True):
    """z = r + dropout(y); out = LN(z).  Returns (z, out, mean, rstd); z is None when it
    equals an input (no branch) or store_z is False."""
    ref = y if y is not None else r
    rows = ref.numel() // ref.shape[-1]
    h = ref.shape[-1]
    if not _on_gpu(ref):
        z = torch.zeros_like(ref, dtype=torch.float32)
        if y is not None:
            z = z + _ref_dropout(y, p, rng, sid).float()
        if r is not None:
            z = z + r.float()
        zf = z.view(rows, h)
        mean = zf.mean(-1)
        var = zf.var(-1, unbiased=False)
        rstd = torch.rsqrt(var + eps)
        out = ((zf - mean[:, None]) * rstd[:, None] * gamma.float() + beta.float()).to(ref.dtype).view_as(ref)
        zz = z.to(ref.dtype) if (store_z and y is not None) else None
        return zz, out, mean, rstd
    y, r = _c(y), _c(r)
    z = torch.empty_like(ref) if (store_z and y is not None) else None
    out = torch.empty_like(ref)
    mean = torch.empty(rows, dtype=torch.float32, device=ref.device)
    rstd = torch.empty_like(mean)
    _lib.call("dtd_ln_fwd", _lib.dt(ref), _lib.ptr(y), _lib.ptr(r), gamma.data_ptr(), beta.data_ptr(),
              _lib.ptr(z), out.data_ptr(), mean.data_ptr(), rstd.data_ptr(), rows, h, float(eps),
              float(p if y is not None else 0.0), rng.state.data_ptr(), sid, _lib.stream())
    return z, out, mean, rstd


def _unpack(dst, acc):
    """Gradient destinations are a tensor (with the call's ``acc``) or a (tensor, acc) pair."""
    if isinstance(dst, tuple):
        return dst
    return dst, acc


def _write_grad(dst, val: torch.Tensor, acc: bool) -> None:
    if dst is None:
        return
    dst, acc = _unpack(dst, acc)
    if acc:
        dst.add_(val.to(dst.dtype))
    else:
        dst.copy_(val)


def _finalize_stream(part: torch.Tensor, defer: bool = True) -> int:
    """Stream for a column-sum finalize of gradient partials.  Inside a DDP backward window
    (``grad.defer_finalize``) the ~10 us finalize launches go to the async-gradient side stream,
    off the dgrad chain: the side stream waits for the partials' producer, the partial buffer is
    held until the join, and the reducer joins it before any collective or the optimizer reads a
    gradient (``join_async_wgrad``)."""
    from .grad import finalize_side_stream
    side = finalize_side_stream(part.device) if defer and part.is_cuda else None
    if side is None:
        return _lib.stream()
    side.wait_stream(torch.cuda.current_stream(part.device))
    from .grad import hold_until_join
    hold_until_join(part)   # freed after the reducer's join (not record_stream: ops/grad.py emit_wgrad)
    return side.cuda_stream


# Batched finalizes.  Inside an autograd backward the column-sum finalizes (bias / LayerNorm
# gradients from fp32 partials) are queued and launched together -- one kernel per batch of up to 32
# (``dtd_colsum_finalize_batch``) -- when something is about to read a gradient: the DDP / ZeRO
# reducers flush before they launch a bucket's collective, and the end of the backward flushes the
# rest (an autograd-engine callback).  The queue holds the partial buffers, so the caching
# allocator cannot hand their memory to a later kernel first.  DTD_FINALIZE_BATCH=0: launch each
# finalize where it is issued (the round-5 behaviour).
_BATCH = [os.environ.get("DTD_FINALIZE_BATCH", "1") == "1"]
_PENDING: list = []        # (stream handle, job tuple, keep-alive tensors)
_PENDING_DST: set = set()
_CB_QUEUED = [False]


class _Job(ctypes.Structure):
    _fields_ = [("part", ctypes.c_void_p), ("out", ctypes.c_void_p), ("nparts", ctypes.c_int), ("cols", ctypes.c_int),
                ("dtype", ctypes.c_int), ("acc", ctypes.c_int), ("scale", ctypes.c_float), ("pad", ctypes.c_int)]


def set_finalize_batching(on: bool) -> None:
    flush_finalizes()
    _BATCH[0] = bool(on)


def _batching(part: torch.Tensor) -> bool:
    return (_BATCH[0] and part.is_cuda and _lib.has("dtd_colsum_finalize_batch")
            and torch._C._current_graph_task_id() != -1)


def _queue(stream: int, jobs, keep) -> None:
    """Queue finalize jobs (part_ptr, out_ptr, nparts, cols, dtype, acc, scale) on ``stream``."""
    dsts = {j[1] for j in jobs}
    if dsts & _PENDING_DST:      # a second finalize into the same gradient: keep them ordered
        flush_finalizes()
    for j in jobs:
        _PENDING.append((stream, j, keep))
        _PENDING_DST.add(j[1])
    if not _CB_QUEUED[0]:
        _CB_QUEUED[0] = True
        torch.autograd.Variable._execution_engine.queue_callback(_end_of_backward)


def _end_of_backward() -> None:
    _CB_QUEUED[0] = False
    flush_finalizes()


def flush_finalizes() -> None:
    """Launch every queued finalize (on the stream it was issued on, in issue order)."""
    if not _PENDING:
        return
    pending = list(_PENDING)
    _PENDING.clear()
    _PENDING_DST.clear()
    i = 0
    while i < len(pending):
        stream = pending[i][0]
        batch = []
        while i < len(pending) and pending[i][0] == stream and len(batch) < 32:
            batch.append(pending[i][1])
            i += 1
        arr = (_Job * len(batch))(*[_Job(*j, 0) for j in batch])
        _lib.call("dtd_colsum_finalize_batch", len(batch), ctypes.addressof(arr), stream)


def _finalize(part: torch.Tensor, n: int, cols: int, dst, acc: bool, scale: float = 1.0, defer: bool = True):
    if dst is None:
        return
    dst, acc = _unpack(dst, acc)
    stream = _finalize_stream(part, defer)
    if stream == _lib.stream() and _batching(part):
        _queue(stream, [(part.data_ptr(), dst.data_ptr(), n, cols, _lib.dt(dst), int(acc), float(scale))], (part, dst))
        return
    _lib.call("dtd_colsum_finalize", part.data_ptr(), n, cols, dst.data_ptr(), _lib.dt(dst), int(acc),
              float(scale), stream)


def ln_bwd(dout, dz_extra, z, mean, rstd, gamma, p: float, rng: RngState, sid: int,
           want_dz: bool = True, want_dy: bool = False,
           dgamma=None, dbeta=None, dbias=None, acc: bool = False, dout2=None, xout=None, beta=None):
    """Backward of ``ln_fwd``.  Returns (dz, dy); writes dgamma/dbeta/dbias (bias of the
    producer of y, i.e. column sums of dy) into the destination tensors.  ``dout2``: a second
    upstream gradient summed into ``dout`` inside the kernel (residual branches).

    Memory-efficient form (``z=None``, ``xout``/``beta`` given): x-hat is recomputed from the
    forward's output, x-hat = (xout - beta) / gamma, so the forward need not store z
    (``ln_fwd(store_z=False)``); ``mean`` is then unused."""
    rows = dout.numel() // dout.shape[-1]
    h = dout.shape[-1]
    fo = z is None
    if fo and (xout is None or beta is None):
        raise ValueError("ln_bwd: z=None needs the LayerNorm output (xout) and beta")
    if not _on_gpu(dout):
        if fo:
            g32 = gamma.float()
            g32 = torch.where(g32.abs() < 1e-12, torch.full_like(g32, 1e-12).copysign(g32), g32)
            xh = (xout.float().view(rows, h) - beta.float()) / g32
        else:
            zf = z.float().view(rows, h)
            xh = (zf - mean[:, None]) * rstd[:, None]
        d = dout.float().view(rows, h)
        if dout2 is not None:
            d = d + dout2.float().view(rows, h)
        g = d * gamma.float()
        m1 = g.mean(-1, keepdim=True)
        m2 = (g * xh).mean(-1, keepdim=True)
        dz = rstd[:, None] * (g - m1 - xh * m2)
        if dz_extra is not None:
            dz = dz + dz_extra.float().view(rows, h)
        dy = None
        if want_dy:
            dy = _ref_dropout(dz.to(dout.dtype), p, rng, sid) if p > 0 else dz.to(dout.dtype)
            _write_grad(dbias, dy.float().sum(0), acc)
            dy = dy.view_as(dout)
        _write_grad(dgamma, (d * xh).sum(0), acc)
        _write_grad(dbeta, d.sum(0), acc)
        return (dz.to(dout.dtype).view_as(dout) if want_dz else None), dy
    dout, dz_extra, dout2 = _c(dout), _c(dz_extra), _c(dout2)
    dz = torch.empty_like(dout) if want_dz else None
    dy = torch.empty_like(dout) if want_dy else None
    n = _lib.lib().dtd_ln_bwd_num_partials(rows, h)
    k = int(dgamma is not None) + int(dbeta is not None) + int(dbias is not None and want_dy)
    part = torch.empty((max(k, 1), n, h), dtype=torch.float32, device=dout.device)
    slots = iter(range(k))
    pg = part[next(slots)] if dgamma is not None else None
    pb = part[next(slots)] if dbeta is not None else None
    py = part[next(slots)] if (dbias is not None and want_dy) else None
    if fo:
        xout = xout.contiguous()
        assert xout.shape == dout.shape and xout.dtype == dout.dtype
        _lib.call("dtd_ln_bwd_fo", _lib.dt(dout), dout.data_ptr(), _lib.ptr(dout2), _lib.ptr(dz_extra),
                  xout.data_ptr(), beta.data_ptr(), rstd.data_ptr(), gamma.data_ptr(), _lib.ptr(dz), _lib.ptr(dy),
                  _lib.ptr(pg), _lib.ptr(pb), _lib.ptr(py), rows, h, float(p if want_dy else 0.0),
                  rng.state.data_ptr(), sid, _lib.stream())
    else:
        _lib.call("dtd_ln_bwd", _lib.dt(dout), dout.data_ptr(), _lib.ptr(dout2), _lib.ptr(dz_extra), z.data_ptr(),
                  mean.data_ptr(),
                  rstd.data_ptr(), gamma.data_ptr(), _lib.ptr(dz), _lib.ptr(dy), _lib.ptr(pg), _lib.ptr(pb),
                  _lib.ptr(py), rows, h, float(p if want_dy else 0.0), rng.state.data_ptr(), sid, _lib.stream())
    dsts = [d for d, on in ((dgamma, pg is not None), (dbeta, pb is not None), (dbias, py is not None)) if on]
    if dsts:
        args = []
        for d in dsts + [None] * (3 - len(dsts)):
            if d is None:
                args += [None, 0, 0]
            else:
                t, a = _unpack(d, acc)
                args += [t.data_ptr(), _lib.dt(t), int(a)]
        stream = _finalize_stream(part)
        if stream == _lib.stream() and _batching(part):
            jobs = []
            for i, d in enumerate(dsts):
                t, a = _unpack(d, acc)
                jobs.append((part.data_ptr() + i * n * h * 4, t.data_ptr(), n, h, _lib.dt(t), int(a), 1.0))
            _queue(stream, jobs, (part, [_unpack(d, acc)[0] for d in dsts]))
        else:
            _lib.call("dtd_colsum_finalize_multi", len(dsts), part.data_ptr(), n, h, *args, stream)
    return dz, dy


# --------------------------------------------------------------------------------------
# activations
# --------------------------------------------------------------------------------------
def _ref_act(u: torch.Tensor, act: str) -> torch.Tensor:
    x = u.float()
    if act == "gelu":
        y = 0.5 * x * (1.0 + torch.erf(x * 0.7071067811865476))
    elif act == "gelu_tanh":
        y = 0.5 * x * (1.0 + torch.tanh(0.7978845608028654 * (x + 0.044715 * x * x * x)))
    elif act == "relu":
        y = torch.clamp_min(x, 0.0)
    else:
        y = x
    return y.to(u.dtype)


def _ref_act_grad(u: torch.Tensor, act: str) -> torch.Tensor:
    x = u.float()
    if act == "gelu":
        cdf = 0.5 * (1.0 + torch.erf(x * 0.7071067811865476))
        return cdf + x * 0.3989422804014327 * torch.exp(-0.5 * x * x)
    if act == "gelu_tanh":
        k = 0.7978845608028654
        t = torch.tanh(k * (x + 0.044715 * x ** 3))
        return 0.5 * (1 + t) + 0.5 * x * (1 - t * t) * k * (1 + 3 * 0.044715 * x * x)
    if act == "relu":
        return (x > 0).float()
    return torch.ones_like(x)


def act_fwd(u: torch.Tensor, act: str) -> torch.Tensor:
    if act == "none":
        return u
    if not _on_gpu(u):
        return _ref_act(u, act)
    u = u.contiguous()
    y = torch.empty_like(u)
    _lib.call("dtd_act_fwd", _lib.dt(u), u.data_ptr(), y.data_ptr(), u.numel(), ACT_CODES[act], _lib.stream())
    return y


def act_bwd(dy: torch.Tensor, u: torch.Tensor | None, act: str, dbias=None, acc: bool = False,
            want_du: bool = True, want_act: bool = False):
    """du = dy * act'(u); writes column sums of du into ``dbias``.  act='none' is a plain
    bias-gradient column sum of dy (returns dy).  ``want_act``: also return act(u), recomputed
    in the same pass -> (du, a)."""
    cols = dy.shape[-1]
    rows = dy.numel() // cols
    if want_act and act == "none":
        raise ValueError("want_act needs an activation")
    if not _on_gpu(dy):
        du = dy.float() if act == "none" else dy.float() * _ref_act_grad(u, act)
        _write_grad(dbias, du.view(rows, cols).sum(0), acc)
        du = du.to(dy.dtype) if want_du else None
        return (du, act_fwd(u, act)) if want_act else du
    dy = dy.contiguous()
    du = torch.empty_like(dy) if (want_du and act != "none") else None
    a = torch.empty_like(u) if want_act else None
    n = _lib.lib().dtd_act_bwd_num_partials(rows, cols)
    part = torch.empty((n, cols), dtype=torch.float32, device=dy.device) if dbias is not None else None
    _lib.call("dtd_act_bwd", _lib.dt(dy), dy.data_ptr(), _lib.ptr(u), _lib.ptr(du), _lib.ptr(part), _lib.ptr(a),
              rows, cols, ACT_CODES[act], _lib.stream())
    if part is not None:
        _finalize(part, n, cols, dbias, acc)
    du = dy if act == "none" else du
    return (du, a) if want_act else du


def bias_grad(dy: torch.Tensor, dbias: torch.Tensor, acc: bool = False) -> None:
    act_bwd(dy, None, "none", dbias=dbias, acc=acc, want_du=False)


# --------------------------------------------------------------------------------------
# softmax cross-entropy
# --------------------------------------------------------------------------------------
def xent_fwd(logits: torch.Tensor, labels: torch.Tensor, ignore_index: int = IGNORE_INDEX):
    """Returns (mean loss [scalar fp32 tensor], lse [N], stats [2] = (mean, count))."""
    V = logits.shape[-1]
    rows = logits.numel() // V
    labels = labels.reshape(-1)
    if not _on_gpu(logits):
        z = logits.float().view(rows, V)
        lse = torch.logsumexp(z, -1)
        valid = labels != ignore_index
        tgt = z.gather(1, labels.clamp_min(0)[:, None])[:, 0]
        loss_row = torch.where(valid, lse - tgt, torch.zeros_like(lse))
        cnt = valid.sum().float()
        mean = loss_row.sum() / cnt
        return mean, lse, torch.stack([mean, cnt])
    logits = logits.contiguous()
    labels = labels.contiguous().to(torch.int64)
    loss_row = torch.empty(rows, dtype=torch.float32, device=logits.device)
    lse = torch.empty_like(loss_row)
    stats = torch.empty(2, dtype=torch.float32, device=logits.device)
    _lib.call("dtd_xent_fwd", _lib.dt(logits), logits.data_ptr(), labels.data_ptr(), loss_row.data_ptr(),
              lse.data_ptr(), stats.data_ptr(), rows, V, ignore_index, _lib.stream())
    return stats[0], lse, stats


def xent_fwd_train(logits, labels, ignore_index: int = IGNORE_INDEX):
    """Training forward of the mean cross-entropy in one pass over the logits: returns
    (loss, lse, stats, dlogits, dbias) with dlogits / dbias (fp32 column sums of dlogits) for a
    loss gradient of 1 -- ``xent_grad_scale`` applies the actual one in the backward -- or None
    when the fused kernel does not cover the case (CPU, not bf16, V % 4 != 0, V > 32768)."""
    V = logits.shape[-1]
    rows = logits.numel() // V
    if (not _on_gpu(logits) or logits.dtype != torch.bfloat16 or not logits.is_contiguous() or rows <= 0
            or logits.data_ptr() % 8 != 0 or not _lib.has("dtd_xent_fwd_train")
            or not _lib.lib().dtd_xent_bwd_colsum_supported(V)):
        return None
    labels = labels.reshape(-1).contiguous().to(torch.int64)
    loss_row = torch.empty(rows, dtype=torch.float32, device=logits.device)
    lse = torch.empty_like(loss_row)
    stats = torch.empty(2, dtype=torch.float32, device=logits.device)
    d = torch.empty_like(logits)
    n = _lib.lib().dtd_xent_bwd_colsum_parts(rows)
    part = torch.empty((n, V), dtype=torch.float32, device=logits.device)
    _lib.call("dtd_xent_fwd_train", logits.data_ptr(), labels.data_ptr(), loss_row.data_ptr(), lse.data_ptr(),
              stats.data_ptr(), d.data_ptr(), part.data_ptr(), rows, V, ignore_index, _lib.stream())
    dbias = torch.empty(V, dtype=torch.float32, device=logits.device)
    _finalize(part, n, V, dbias, False, defer=False)   # a forward result, read by the backward
    return stats[0], lse, stats, d, dbias


def xent_grad_scale_(d: torch.Tensor, grad_out: torch.Tensor) -> torch.Tensor:
    """d *= grad_out in place unless grad_out == 1 (checked on the device: no host sync)."""
    g = grad_out.reshape(1).to(torch.float32).contiguous()
    _lib.call("dtd_xent_grad_scale", d.data_ptr(), d.numel(), g.data_ptr(), _lib.stream())
    return d


def xent_bwd(logits, labels, lse, stats, grad_out, ignore_index: int = IGNORE_INDEX, dbias=None):
    """dlogits of the mean cross-entropy.  ``dbias`` = (dst, acc): also the column sums of dlogits
    (the bias gradient of the Linear that produced the logits) -- on the kernel path from the same
    pass (``dtd_xent_bwd_colsum``: no re-read of dlogits) when V % 4 == 0 and V <= 32768."""
    V = logits.shape[-1]
    rows = logits.numel() // V
    labels = labels.reshape(-1)
    if not _on_gpu(logits):
        z = logits.float().view(rows, V)
        p = torch.exp(z - lse[:, None])
        valid = labels != ignore_index
        p[torch.arange(rows), labels.clamp_min(0)] -= 1.0
        p = p * valid[:, None].float() * (grad_out.float() / stats[1])
        d = p.to(logits.dtype).view_as(logits)
        if dbias is not None:
            bias_grad(d, *dbias)
        return d
    if (dbias is not None and logits.dtype == torch.bfloat16 and logits.is_contiguous() and rows > 0
            and logits.data_ptr() % 8 == 0 and _lib.has("dtd_xent_bwd_colsum")
            and _lib.lib().dtd_xent_bwd_colsum_supported(V)):
        d = torch.empty_like(logits)
        n = _lib.lib().dtd_xent_bwd_colsum_parts(rows)
        part = torch.empty((n, V), dtype=torch.float32, device=logits.device)
        gout = grad_out.reshape(1).to(torch.float32).contiguous()
        _lib.call("dtd_xent_bwd_colsum", logits.data_ptr(), labels.contiguous().to(torch.int64).data_ptr(),
                  lse.data_ptr(), stats.data_ptr(), gout.data_ptr(), d.data_ptr(), part.data_ptr(), rows, V,
                  ignore_index, _lib.stream())
        _finalize(part, n, V, dbias, dbias[1] if isinstance(dbias, tuple) else False)
        return d
    phase = logits.data_ptr() % 16   # the kernel needs dlogits in the same 16-byte phase
    if phase:
        es = logits.element_size()
        buf = torch.empty(logits.numel() + 16 // es, dtype=logits.dtype, device=logits.device)
        d = buf[phase // es:phase // es + logits.numel()].view_as(logits)
    else:
        d = torch.empty_like(logits)
    gout = grad_out.reshape(1).to(torch.float32).contiguous()
    _lib.call("dtd_xent_bwd", _lib.dt(logits), logits.data_ptr(), labels.contiguous().to(torch.int64).data_ptr(),
              lse.data_ptr(), stats.data_ptr(), gout.data_ptr(), d.data_ptr(), rows, V, ignore_index,
              _lib.stream())
    if dbias is not None:
        bias_grad(d, *dbias)
    return d


class _CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, ignore_index):
        loss, lse, stats = xent_fwd(logits, labels, ignore_index)
        ctx.save_for_backward(logits, labels, lse, stats)
        ctx.ignore_index = ignore_index
        return loss

    @staticmethod
    def backward(ctx, gloss):
        logits, labels, lse, stats = ctx.saved_tensors
        return xent_bwd(logits, labels, lse, stats, gloss, ctx.ignore_index), None, None


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor, ignore_index: int = IGNORE_INDEX) -> torch.Tensor:
    """Mean softmax cross-entropy over rows of ``logits`` [..., V] straight from the logits' own
    dtype (bf16: no fp32 up-cast copy of the logits; the kernel accumulates in fp32) -- the
    drop-in for ``nn.CrossEntropyLoss()(logits.view(-1, V).float(), labels.view(-1))`` of
    /root/reference/model_parallel_training.py:51,73."""
    return _CrossEntropyFn.apply(logits.reshape(-1, logits.shape[-1]), labels.reshape(-1), ignore_index)


class CrossEntropyLoss(torch.nn.Module):
    def __init__(self, ignore_index: int = IGNORE_INDEX):
        super().__init__()
        self.ignore_index = ignore_index

    def forward(self, logits, labels):
        return cross_entropy(logits, labels, self.ignore_index)


# --------------------------------------------------------------------------------------
# embeddings
# --------------------------------------------------------------------------------------
def embed_fwd(ids: torch.Tensor, word: torch.Tensor, pos: torch.Tensor | None, type_: torch.Tensor | None,
              seq: int, pos_offset: int = 0, type_ids: torch.Tensor | None = None) -> torch.Tensor:
    rows = ids.numel()
    h = word.shape[1]
    if not _on_gpu(word):
        flat = ids.reshape(-1)
        out = word[flat].float()
        if pos is not None:
            pidx = torch.arange(rows, device=ids.device) % seq + pos_offset
            out = out + pos[pidx].float()
        if type_ is not None:
            tid = type_ids.reshape(-1) if type_ids is not None else torch.zeros_like(flat)
            out = out + type_[tid].float()
        return out.to(word.dtype)
    out = torch.empty((rows, h), dtype=word.dtype, device=word.device)
    ids_c = ids.reshape(-1).contiguous().to(torch.int64)
    tids = type_ids.reshape(-1).contiguous().to(torch.int64) if type_ids is not None else None
    _lib.call("dtd_embed_fwd", _lib.dt(word), ids_c.data_ptr(), _lib.ptr(tids), word.data_ptr(), _lib.ptr(pos),
              _lib.ptr(type_), out.data_ptr(), rows, h, seq, pos_offset, _lib.stream())
    return out


def embed_ln_fwd(ids, word, pos, type_, seq: int, pos_offset: int, gamma, beta, eps: float, p: float,
                 rng: RngState, sid: int, type_ids=None):
    """Embedding gather-sum + LayerNorm + dropout in one kernel: returns (out, z, mean, rstd), the
    same values as ``embed_fwd`` -> ``ln_fwd(None, z, ...)`` -> ``dropout`` (z = the LN input the
    backward needs), or None when the fused kernel does not cover the case (CPU, fp32, h other
    than 768 / 1024): the caller then runs the three passes."""
    h = word.shape[1]
    if (not _on_gpu(word) or word.dtype != torch.bfloat16 or h not in (768, 1024) or gamma is None
            or not _lib.has("dtd_embed_ln_fwd")
            or any(t is not None and (t.dtype != torch.bfloat16 or not t.is_contiguous())
                   for t in (word, pos, type_, gamma, beta))):
        return None
    rows = ids.numel()
    z = torch.empty((rows, h), dtype=word.dtype, device=word.device)
    out = torch.empty_like(z)
    mean = torch.empty(rows, dtype=torch.float32, device=word.device)
    rstd = torch.empty_like(mean)
    ids_c = ids.reshape(-1).contiguous().to(torch.int64)
    tids = type_ids.reshape(-1).contiguous().to(torch.int64) if type_ids is not None else None
    _lib.call("dtd_embed_ln_fwd", ids_c.data_ptr(), _lib.ptr(tids), word.data_ptr(), _lib.ptr(pos), _lib.ptr(type_),
              gamma.data_ptr(), beta.data_ptr(), z.data_ptr(), out.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
              rows, h, seq, pos_offset, float(eps), float(p), rng.state.data_ptr(), sid,
              _lib.stream())
    return out, z, mean, rstd


def scatter_rows_supported(g: torch.Tensor) -> bool:
    return (g.is_cuda and g.dtype == torch.bfloat16 and g.dim() == 2 and g.is_contiguous() and g.shape[1] % 8 == 0
            and g.data_ptr() % 16 == 0 and _lib.has("dtd_scatter_rows"))


def scatter_rows(g: torch.Tensor, idx: torch.Tensor, count: torch.Tensor | None, cap: int, rows: int) -> torch.Tensor:
    """[rows, h] with row idx[p] = g[p] for p < n and zeros elsewhere, n = min(count, cap) (count: a
    device scalar, None -> cap); idx[0:n) ascending and unique (the backward of a row gather)."""
    out = torch.empty((rows, g.shape[1]), dtype=g.dtype, device=g.device)
    assert idx.dtype == torch.int64 and idx.is_contiguous() and cap <= idx.numel() and cap <= g.shape[0]
    _lib.call("dtd_scatter_rows", g.data_ptr(), idx.data_ptr(), _lib.ptr(count), int(cap), out.data_ptr(), rows,
              g.shape[1], _lib.stream())
    return out


def embed_word_bwd(ids: torch.Tensor, dz: torch.Tensor, grad: torch.Tensor, acc: bool, padding_idx: int = -1):
    flat = ids.reshape(-1)
    h = grad.shape[1]
    dz = dz.reshape(-1, h)
    if not _on_gpu(grad):
        g = torch.zeros(grad.shape, dtype=torch.float32, device=grad.device)
        g.index_add_(0, flat, dz.float())
        if padding_idx >= 0:
            g[padding_idx] = 0
        if acc:
            grad.add_(g.to(grad.dtype))
        else:
            grad.copy_(g)
        return
    if not acc:
        grad.zero_()
    sorted_ids, perm = torch.sort(flat.to(torch.int64), stable=True)
    lo = torch.searchsorted(sorted_ids, sorted_ids, right=False)
    hi = torch.searchsorted(sorted_ids, sorted_ids, right=True)
    dz = dz.contiguous()
    scratch = torch.empty((flat.numel(), h), dtype=torch.float32, device=dz.device)
    _lib.call("dtd_embed_word_bwd_chunked", _lib.dt(dz), _lib.dt(grad), sorted_ids.data_ptr(), perm.data_ptr(),
              lo.data_ptr(), hi.data_ptr(), scratch.data_ptr(), dz.data_ptr(), grad.data_ptr(), flat.numel(), h, 1,
              padding_idx, _lib.stream())


def embed_pos_bwd(dz: torch.Tensor, grad: torch.Tensor, batch: int, seq: int, pos_offset: int, acc: bool):
    h = grad.shape[1]
    if not _on_gpu(grad):
        s = dz.reshape(batch, seq, h).float().sum(0)
        if not acc:
            grad.zero_()
        grad[pos_offset:pos_offset + seq].add_(s.to(grad.dtype))
        return
    if not acc:
        grad.zero_()
    dz = dz.contiguous()
    _lib.call("dtd_embed_pos_bwd", _lib.dt(dz), _lib.dt(grad), dz.data_ptr(), grad.data_ptr(), batch, seq, h,
              pos_offset, 1, _lib.stream())


# --------------------------------------------------------------------------------------
# flat-buffer utilities
# --------------------------------------------------------------------------------------
def scale_cast_(src: torch.Tensor, dst: torch.Tensor, scale: float = 1.0, dscale: torch.Tensor | None = None):
    """dst = src * scale * (dscale[0] if given), with dtype conversion (flat buffers)."""
    if not _on_gpu(src):
        v = src.float() * scale
        if dscale is not None:
            v = v * dscale[0]
        dst.copy_(v)
        return dst
    _lib.call("dtd_scale_cast", src.data_ptr(), _lib.dt(src), dst.data_ptr(), _lib.dt(dst), src.numel(),
              float(scale), _lib.ptr(dscale), _lib.stream())
    return dst


def sq_norm(x: torch.Tensor) -> torch.Tensor:
    """Sum of squares of a flat tensor as a 0-dim fp32 device tensor (no host sync)."""
    if not _on_gpu(x):
        return x.float().pow(2).sum()
    n = _lib.lib().dtd_sqnorm_num_partials(x.numel())
    part = torch.empty(n, dtype=torch.float32, device=x.device)
    _lib.call("dtd_sqnorm_partials", x.data_ptr(), _lib.dt(x), x.numel(), part.data_ptr(), _lib.stream())
    return part.sum()


# --------------------------------------------------------------------------------------
# row softmax (instrumented block)
# --------------------------------------------------------------------------------------
def softmax_fwd(x: torch.Tensor) -> torch.Tensor:
    if not _on_gpu(x) or x.dtype not in (torch.bfloat16, torch.float32):
        return torch.softmax(x.float(), dim=-1).to(x.dtype)
    x = x.contiguous()
    y = torch.empty_like(x)
    n = x.shape[-1]
    _lib.call("dtd_softmax_fwd", _lib.dt(x), x.data_ptr(), y.data_ptr(), x.numel() // n, n, _lib.stream())
    return y


def softmax_bwd(y: torch.Tensor, dy: torch.Tensor) -> torch.Tensor:
    if not _on_gpu(y) or y.dtype not in (torch.bfloat16, torch.float32):
        yf, df = y.float(), dy.float()
        return (yf * (df - (yf * df).sum(-1, keepdim=True))).to(y.dtype)
    dy = dy.contiguous().to(y.dtype)
    dx = torch.empty_like(y)
    n = y.shape[-1]
    _lib.call("dtd_softmax_bwd", _lib.dt(y), y.data_ptr(), dy.data_ptr(), dx.data_ptr(), y.numel() // n, n,
              _lib.stream())
    return dx


class _SoftmaxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y = softmax_fwd(x)
        ctx.save_for_backward(y)      # like ATen's softmax: the output is the saved activation
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        return softmax_bwd(y, dy)


class Softmax(torch.nn.Module):
    """Drop-in ``nn.Softmax(dim=-1)`` backed by the HIP row-softmax kernels on the GPU."""

    def __init__(self, dim: int = -1):
        super().__init__()
        if dim not in (-1,):
            raise ValueError("row softmax over the last dim only")
        self.dim = dim

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return _SoftmaxFn.apply(x)
