"""Flat parameter / gradient storage shared by DDP, ZeRO and the fused optimizer.

MI355X-first memory layout: every trainable parameter of a model lives as a view into ONE
contiguous buffer (``FlatLayout``), and its gradient as a view (``main_grad``) into a second
contiguous buffer in the same layout.  Consequences:
  * a DDP bucket or a ZeRO partition is a slice of the flat gradient buffer, so collectives run
    on it in place -- no flatten/unflatten copies (DDP Reducer copies into buckets, SURVEY.md D3;
    DeepSpeed flattens into IPG buckets, D10);
  * the optimizer step is a single fused kernel over the whole buffer (or the local shard);
  * the fused modules' backward passes write weight gradients into their final slot
    (``ops/grad.py``), with overwrite-on-first-contribution semantics that make a per-step
    zeroing pass unnecessary.
Offsets are aligned to 64 elements (128 B in bf16) so every view is 16-byte aligned for the
vectorised kernels and buckets/partitions can be cut on aligned boundaries.
"""
from __future__ import annotations

import torch

ALIGN = 64


def _align(n: int, a: int = ALIGN) -> int:
    return (n + a - 1) // a * a


def unique_params(params) -> list:
    seen, out = set(), []
    for p in params:
        if p.requires_grad and id(p) not in seen:
            seen.add(id(p))
            out.append(p)
    return out


class FlatLayout:
    """Ordered parameters with aligned offsets into a flat buffer."""

    def __init__(self, params, align: int = ALIGN):
        self.params = unique_params(params)
        self.offsets, off = [], 0
        for p in self.params:
            self.offsets.append(off)
            off += _align(p.numel(), align)
        self.numel = _align(off, align)
        self.index = {id(p): i for i, p in enumerate(self.params)}

    def view(self, flat: torch.Tensor, i: int) -> torch.Tensor:
        p = self.params[i]
        return flat[self.offsets[i]:self.offsets[i] + p.numel()].view_as(p)

    def range_of(self, i: int) -> tuple[int, int]:
        return self.offsets[i], self.offsets[i] + self.params[i].numel()

    def flatten_params_(self, device=None, dtype=None) -> torch.Tensor:
        """Move parameter storage into one flat buffer (``p.data`` becomes a view)."""
        p0 = self.params[0]
        device = device or p0.device
        dtype = dtype or p0.dtype
        flat = torch.zeros(self.numel, dtype=dtype, device=device)
        for i, p in enumerate(self.params):
            v = self.view(flat, i)
            v.copy_(p.data)
            p.data = v
        return flat


class GradBuffer:
    """Flat gradient storage in a layout; installs ``main_grad`` views and gradient hooks.

    ``on_ready(p)`` (optional) is called once per parameter per backward when all of its
    expected contributions have arrived (fused modules announce uses in forward via
    ``ops.grad.note_use``; autograd-path parameters contribute once, through a
    post-accumulate-grad hook that folds ``p.grad`` into ``main_grad``).
    ``on_contribution(p, autograd)`` (optional) replaces that counting: every contribution is
    handed to the owner (the DDP reducer counts them in the native tracker, runtime/)."""

    def __init__(self, layout: FlatLayout, dtype: torch.dtype, device, on_ready=None, on_contribution=None):
        self.layout = layout
        self.dtype = dtype
        self.buf = torch.zeros(layout.numel, dtype=dtype, device=device)
        self.on_ready = on_ready
        self.on_contribution = on_contribution
        self._hooks = []
        for i, p in enumerate(layout.params):
            p.main_grad = layout.view(self.buf, i)
            p._dtd_touched = False
            p._dtd_pending = 0
            p._dtd_ready_hook = self._ready
            self._hooks.append(p.register_post_accumulate_grad_hook(self._from_autograd))

    # autograd path: AccumulateGrad wrote p.grad; fold it into main_grad.
    def _from_autograd(self, p):
        g = p.grad
        if g is None:
            return
        if g.data_ptr() != p.main_grad.data_ptr():
            if p._dtd_touched:
                p.main_grad.add_(g.to(self.dtype))
            else:
                p.main_grad.copy_(g)
            p.grad = None
        p._dtd_touched = True
        self._ready(p, autograd=True)

    def _ready(self, p, autograd: bool = False):
        if self.on_contribution is not None:
            self.on_contribution(p, autograd)
            return
        pend = getattr(p, "_dtd_pending", 0)
        if pend > 0 and not autograd:
            pend -= 1
            p._dtd_pending = pend
            if pend > 0:
                return
        if self.on_ready is not None:
            self.on_ready(p)

    def reset(self) -> None:
        """Start of a new accumulation window: next contribution overwrites."""
        for p in self.layout.params:
            p._dtd_touched = False
            p._dtd_pending = 0
            p.grad = None

    def zero_untouched_(self) -> None:
        for i, p in enumerate(self.layout.params):
            if not p._dtd_touched:
                p.main_grad.zero_()
                p._dtd_touched = True

    def expose_as_grad(self) -> None:
        """Point ``p.grad`` at ``main_grad`` (same dtype only) for stock torch optimizers."""
        for p in self.layout.params:
            if p.main_grad.dtype == p.dtype:
                p.grad = p.main_grad

    def remove(self) -> None:
        for h in self._hooks:
            h.remove()
        for p in self.layout.params:
            for a in ("main_grad", "_dtd_ready_hook", "_dtd_touched", "_dtd_pending", "_dtd_expect"):
                if hasattr(p, a):
                    delattr(p, a)
