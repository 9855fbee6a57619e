"""Point-to-point activation transfer between pipeline stages.

Reference: ``hidden_states.to(device)`` at every device-group boundary of BertModelWithMP
(model/bert_mp.py:93-97) and torch Pipe's copy streams.

Single process, several GPUs: the copy is issued on a dedicated *copy stream* of the
destination device (peer DMA over xGMI on MI355X, ``hipMemcpyPeerAsync`` underneath), fenced
by events: the destination compute stream waits only for the copy, and the source stream
is not blocked -- the previous stage can start its next micro-batch while the activation
is in flight.  Backward sends the gradient the opposite way on the source device's copy
stream.  Same-device "stages" (1-GPU testing of the schedule) pass tensors through.
"""
from __future__ import annotations

import torch

_COPY_STREAMS: dict = {}


def copy_stream(device: torch.device):
    device = torch.device(device)
    if device.type != "cuda":
        return None
    key = device.index if device.index is not None else torch.cuda.current_device()
    if key not in _COPY_STREAMS:
        _COPY_STREAMS[key] = torch.cuda.Stream(device=key)
    return _COPY_STREAMS[key]


def _transfer(x: torch.Tensor, dst: torch.device) -> torch.Tensor:
    src = x.device
    if src == dst:
        return x
    if dst.type != "cuda" or src.type != "cuda":
        return x.to(dst)
    cs = copy_stream(dst)
    src_stream = torch.cuda.current_stream(src)
    ready = torch.cuda.Event()
    ready.record(src_stream)          # x is produced on the source compute stream
    # y is allocated on the destination's compute stream -- its consumer -- so the allocator
    # recycles it in that stream's order and it needs no record_stream; that stream waits for
    # the copy below before anything reads y
    with torch.cuda.device(dst):
        y = torch.empty(x.shape, dtype=x.dtype, device=dst)
    with torch.cuda.device(dst), torch.cuda.stream(cs):
        cs.wait_event(ready)
        y.copy_(x, non_blocking=True)
    # x belongs to the source stream's pool; the copy stream's read must finish before the
    # allocator hands x's block out again: one record_stream per transfer (two per micro-batch
    # and stage boundary, not per kernel -- not the per-tensor pattern that slowed --async-wgrad)
    x.record_stream(cs)
    done = torch.cuda.Event()
    done.record(cs)
    torch.cuda.current_stream(dst).wait_event(done)
    return y


class _SendRecv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dst):
        ctx.src = x.device
        return _transfer(x, dst)

    @staticmethod
    def backward(ctx, g):
        return _transfer(g, ctx.src), None


def send_to(x: torch.Tensor, device) -> torch.Tensor:
    """Differentiable stage-to-stage transfer of an activation."""
    device = torch.device(device)
    if x.device == device:
        return x
    if x.requires_grad:
        return _SendRecv.apply(x, device)
    return _transfer(x, device)
