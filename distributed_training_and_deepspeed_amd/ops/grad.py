"""Direct parameter-gradient emission for the fused (hand-written backward) modules.

The fused modules' backward passes write weight/bias gradients straight into their final
storage instead of returning them to autograd:

* if the parameter has ``main_grad`` (a view into a flat gradient buffer owned by the DDP /
  ZeRO engine, ``parallel/grad_buffer.py``), the wgrad GEMM writes into that view with
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

import torch


def grad_dst(p: torch.Tensor):
    """(destination tensor, accumulate?) for the next gradient contribution of ``p``."""
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
        if getattr(p, "_dtd_ready_hook", None) is not None:
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


def emit_grad(p: torch.Tensor, g: torch.Tensor) -> None:
    dst, acc = grad_dst(p)
    if acc:
        dst.add_(g.to(dst.dtype))
    else:
        dst.copy_(g)
    grad_done(p)
