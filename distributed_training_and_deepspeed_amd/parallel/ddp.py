"""Data parallelism: bucketed gradient all-reduce overlapped with backward (RCCL over xGMI).

Replaces ``torch.nn.parallel.DistributedDataParallel(model, device_ids=[rank],
bucket_cap_mb=N)`` (data_parallel_training.py:44) with an MI355X-first
reducer:

* Parameters and gradients live in flat buffers (``parallel/flat.py``), ordered in reverse
  registration order (~ the order gradients become ready in backward).  A bucket is a
  contiguous slice of the flat gradient buffer, so the all-reduce runs in place: no
  copy-into-bucket, no copy-back (the C++ Reducer's two copies per step disappear).
* The fused modules write weight gradients straight into their bucket slot; each parameter
  reports readiness once all its contributions (tied weights: two) have arrived.  A complete
  bucket is all-reduced immediately (``async_op``: RCCL runs on its own stream and waits on
  the compute stream's event), in bucket-index order on every rank, so communication overlaps
  the remaining backward.  ``finish`` makes the compute stream wait for all buckets.
* The bookkeeping -- bucket assignment, per-parameter expected-contribution counts, bucket
  completeness and the in-order launch decisions -- runs in the native C++ tracker
  (``runtime/csrc/reducer.cpp``, the counterpart of torch's C++ Reducer); Python issues the
  collectives it asks for.
* RCCL averages in the collective (``ReduceOp.AVG``); gloo (CPU tests) sums then scales.
* Gradients can be kept/communicated in bf16 (``grad_dtype``): half the xGMI bytes of the
  reference's fp32 buckets.  Bucket size defaults to the reference's 25 MiB; on an 8-GPU
  MI355X node larger buckets (fewer, bigger RCCL calls saturating the 7 xGMI links) are
  selected with ``bucket_cap_mb`` (see ``bench/`` sweep).
* Optional native path for small buckets (``small_bucket_allreduce="xgmi"``): buckets of at
  most ``xgmi_max_mb`` go through the peer-mapped one-shot/two-shot kernel of
  ``comm/xgmi.py`` on a side stream instead of an RCCL ring (latency-bound sizes).
* ``force_collectives`` (or env ``DTD_FORCE_COLLECTIVES=1``) issues the bucket all-reduces even
  on a one-rank process group, so the N > 1 data path -- RCCL kernels on RCCL's stream, launched
  from the autograd thread while backward runs, waited for by the compute stream, and captured
  in a hipGraph with the rest of the step -- runs and is measured on a single GPU.
* The constructor broadcasts parameters from rank 0 (C3).  Per-step buffer broadcast (C4) is
  elided: the only module buffers of the reference models are constant index tensors.
"""
from __future__ import annotations

import contextlib
import os

import torch
import torch.distributed as dist
from torch import nn

from ..comm import logger as comm_log
from ..ops.functional import flush_finalizes
from ..ops.grad import join_async_wgrad, set_async_wgrad, set_defer_finalize
from ..ops.grad import _ASYNC as _ASYNC_WGRAD
from ..runtime import ReadyTracker, assign_buckets
from .flat import FlatLayout, GradBuffer


def wgrad_stream(device) -> torch.cuda.Stream:
    return _ASYNC_WGRAD.stream(device)


class _Bucket:
    __slots__ = ("index", "start", "end", "params", "work")

    def __init__(self, index, start, end, params):
        self.index, self.start, self.end, self.params = index, start, end, params
        self.work = None


class _StreamWork:
    """Work handle of a collective issued on a side stream: wait() fences the current stream."""

    def __init__(self, stream, device):
        self.stream, self.device = stream, device

    def wait(self):
        torch.cuda.current_stream(self.device).wait_stream(self.stream)


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, device_ids=None, bucket_cap_mb: float = 25.0,
                 grad_dtype: torch.dtype | None = None, process_group=None, broadcast_parameters: bool = True,
                 overlap: bool = True, flatten_params: bool = True, small_bucket_allreduce: str = "rccl",
                 xgmi_max_mb: float = 4.0, async_wgrad: bool = False, xgmi_check_every: int = 100,
                 force_collectives: bool | None = None):
        super().__init__()
        self.module = module
        self.process_group = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        if force_collectives is None:
            force_collectives = os.environ.get("DTD_FORCE_COLLECTIVES", "0") == "1"
        if force_collectives and not dist.is_initialized():
            raise RuntimeError("force_collectives needs an initialised process group (comm.init())")
        # collectives run whenever there is a peer -- or always, when forced (one-GPU rehearsal of
        # the multi-GPU data path)
        self.collectives = self.world > 1 or bool(force_collectives)
        self.overlap = overlap
        params = [p for p in module.parameters() if p.requires_grad]
        # reverse registration order ~ gradient-ready order in backward (torch DDP does the same)
        self.layout = FlatLayout(list(reversed(params)))
        p0 = self.layout.params[0]
        self.device = p0.device
        self.param_flat = self.layout.flatten_params_() if flatten_params else None
        self.grad_dtype = grad_dtype or p0.dtype
        self.grads = GradBuffer(self.layout, self.grad_dtype, self.device, on_contribution=self._on_contribution)
        self._build_buckets(bucket_cap_mb)
        for p in self.layout.params:
            p._dtd_expect = self._expect
        self._sync_enabled = True
        self._need_reset = True
        self._window_open = False
        self._callback_queued = False
        self.backend = dist.get_backend(process_group) if dist.is_initialized() else "none"
        self._xgmi = None
        # a timed-out xGMI barrier (a peer never arrived) leaves the bucket holding a sum over
        # stale peer data; the kernel only raises a device flag.  finish() polls it every synced
        # step without a host sync (an async copy into pinned memory, read one step later), so
        # at most one optimizer step applies corrupt gradients before the run raises; every
        # ``xgmi_check_every`` steps it also does a blocking read
        self._xgmi_check_every = max(1, int(xgmi_check_every))
        self._xgmi_steps = 0
        if small_bucket_allreduce == "xgmi" and self.world > 1 and self.backend == "nccl":
            from ..comm.xgmi import XgmiAllReduce
            self._xgmi = XgmiAllReduce(process_group, max_bytes=int(xgmi_max_mb * 2 ** 20))
            self._xgmi_stream = torch.cuda.Stream(self.device)
        elif small_bucket_allreduce not in ("rccl", "xgmi"):
            raise ValueError(f"small_bucket_allreduce must be 'rccl' or 'xgmi', got {small_bucket_allreduce!r}")
        # weight-gradient GEMMs of the fused layers on a side stream (ops/grad.py _AsyncWgrad):
        # bucket collectives are issued from that stream after it joins the compute stream, so
        # neither stream blocks the other; finish() joins it before the optimizer reads grads
        self.async_wgrad = bool(async_wgrad) and self.device.type == "cuda"
        # gradient column-sum finalizes (bias / LN parameters) on the side stream during backward:
        # opt-in (DTD_DEFER_FINALIZE=1) and world 1 only.  It measured +0.15 % at b256
        # (profiles/r2_ab_defer_finalize.jsonl); off by default so the 1-GPU bench runs the same
        # stream schedule as the N > 1 path, where every bucket launch would have to join the
        # side stream on the compute stream
        self._defer_finalize = (self.device.type == "cuda" and os.environ.get("DTD_DEFER_FINALIZE", "0") == "1"
                                and self.world == 1)
        if self.async_wgrad:
            set_async_wgrad(True)
        if broadcast_parameters and self.world > 1:
            self._broadcast_params()

    # ------------------------------------------------------------------ setup
    def _trailing_start(self) -> int:
        """Layout index from which every parameter belongs to the model's first unit (the
        embeddings, incl. a tied decoder weight): their gradients are complete only when the whole
        backward is, so they form the trailing bucket(s) of the step.  len(params) if none."""
        units = self.module.zero3_units() if hasattr(self.module, "zero3_units") else []
        if not units:
            return len(self.layout.params)
        first = {id(p) for p in units[0].parameters()}
        i = len(self.layout.params)
        while i > 0 and id(self.layout.params[i - 1]) in first:
            i -= 1
        return i

    def _build_buckets(self, cap_mb: float) -> None:
        """Consecutive buckets of <= cap over the layout (reverse registration ~ backward order),
        with a shaped tail for the multi-GPU critical path: the trailing group (embeddings: ready
        only when backward ends) gets bucket(s) of its own, and the parameters just before it (the
        first layer) a small bucket of <= tail_bucket_mb, launched as soon as that layer's
        backward ends so its all-reduce finishes under the embedding backward.  What is exposed
        after backward is then the embedding all-reduce alone, not a full bucket of layer
        gradients queued in front of it.  DTD_DDP_TAIL_BUCKET_MB=0 disables the shaping."""
        es = self.grads.buf.element_size()
        cap = int(cap_mb * 1024 * 1024 / es)
        tail_cap = int(float(os.environ.get("DTD_DDP_TAIL_BUCKET_MB", "16")) * 1024 * 1024 / es)
        L = self.layout
        n = len(L.params)
        numels = [p.numel() for p in L.params]
        cuts = [0, n]
        t = self._trailing_start() if tail_cap > 0 else n
        if 0 < t < n:
            cuts = [0, t, n]
            # the small pre-trailing bucket: the parameters before t that fit in tail_cap
            j, size = t, 0
            while j > 0 and size + numels[j - 1] <= tail_cap:
                size += numels[j - 1]
                j -= 1
            if 0 < j < t:
                cuts = [0, j, t, n]
        bucket_of, ranges = [], []
        for a, b in zip(cuts[:-1], cuts[1:]):
            lo = L.offsets[a]
            hi = L.offsets[b] if b < n else L.numel
            bo, rg = assign_buckets([o - lo for o in L.offsets[a:b]], numels[a:b], hi - lo, cap)
            base = len(ranges)
            bucket_of += [base + k for k in bo]
            ranges += [(lo + s0, lo + e0) for s0, e0 in rg]
        members = [[] for _ in ranges]
        for i, b in enumerate(bucket_of):
            members[b].append(L.params[i])
        self.buckets = [_Bucket(k, s, e, members[k]) for k, (s, e) in enumerate(ranges)]
        self.tracker = ReadyTracker(bucket_of, len(self.buckets))

    @torch.no_grad()
    def _broadcast_params(self) -> None:
        if self.param_flat is not None:
            comm_log.broadcast(self.param_flat, src=0, group=self.process_group)
        else:
            for p in self.layout.params:
                comm_log.broadcast(p.data, src=0, group=self.process_group)

    # ------------------------------------------------------------------ step lifecycle
    def _reset(self) -> None:
        self.grads.reset()
        for b in self.buckets:
            b.work = None
        self._callback_queued = False
        self._need_reset = False

    def forward(self, *args, **kwargs):
        if self._need_reset:
            self._reset()
        if not self._window_open:   # a new backward window: fresh readiness / launch state
            self.tracker.reset()
            self._window_open = True
        if self._defer_finalize and torch.is_grad_enabled():
            # bias / LN-parameter finalizes off the dgrad chain until the end of this backward
            # (_finish_backward joins them, synced or not)
            set_defer_finalize(True)
        return self.module(*args, **kwargs)

    @contextlib.contextmanager
    def no_sync(self):
        """Gradient accumulation: backward passes inside accumulate without communication."""
        prev = self._sync_enabled
        self._sync_enabled = False
        try:
            yield
        finally:
            self._sync_enabled = prev

    def _expect(self, p) -> None:
        self.tracker.expect(self.layout.index[id(p)])

    def _on_contribution(self, p, autograd: bool) -> None:
        if not self._callback_queued:
            self._callback_queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finish_backward)
        # the tracker launches complete buckets in bucket order only (identical collective
        # sequence on every rank); inside no_sync it just counts
        _, launch = self.tracker.contribute(self.layout.index[id(p)], autograd,
                                            allow_launch=self._sync_enabled and self.overlap)
        for k in launch:
            self._launch(self.buckets[k])

    def _launch(self, b: _Bucket) -> None:
        if not self.collectives:
            return
        flush_finalizes()   # queued bias / LayerNorm finalizes write into this bucket
        view = self.grads.buf[b.start:b.end]
        if self._xgmi is not None and self._xgmi.supports(view):
            join_async_wgrad(self.device)
            side = self._xgmi_stream
            side.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(side):
                self._xgmi.all_reduce(view, average=True)
            b.work = _StreamWork(side, self.device)
        elif self.backend == "nccl" and self.async_wgrad:
            side = wgrad_stream(self.device)
            side.wait_stream(torch.cuda.current_stream(self.device))   # bias / LN grads of the bucket
            with torch.cuda.stream(side):
                b.work = comm_log.all_reduce(view, op=dist.ReduceOp.AVG, group=self.process_group, async_op=True)
        elif self.backend == "nccl":
            b.work = comm_log.all_reduce(view, op=dist.ReduceOp.AVG, group=self.process_group, async_op=True)
        else:
            b.work = comm_log.all_reduce(view, op=dist.ReduceOp.SUM, group=self.process_group, async_op=True)

    def _finish_backward(self) -> None:
        # one end-of-backward callback per backward pass, synced or not: the next backward
        # (e.g. the synced micro-step after a no_sync one) must queue its own
        self._callback_queued = False
        self._window_open = False
        if not self._sync_enabled:
            # a no_sync micro-step: its side-stream finalizes wrote main_grad; join them before
            # anything else (logging, the next micro-step's autograd-path adds) touches it
            flush_finalizes()
            join_async_wgrad(self.device)
            set_defer_finalize(False)
            return
        self.finish()

    def finish(self) -> None:
        """Launch any bucket not yet launched (unused parameters get zero gradients) and make
        the current stream wait for every all-reduce."""
        flush_finalizes()               # batched finalizes still queued by this backward
        join_async_wgrad(self.device)   # async wgrad GEMMs / deferred finalizes
        set_defer_finalize(False)
        self.grads.zero_untouched_()
        for k in self.tracker.drain():
            self._launch(self.buckets[k])
        self._window_open = False
        for b in self.buckets:
            if b.work is not None:
                b.work.wait()
                if self.backend != "nccl" and not isinstance(b.work, _StreamWork):
                    self.grads.buf[b.start:b.end].div_(self.world)
                b.work = None
        self.grads.expose_as_grad()
        self._need_reset = True
        if self._xgmi is not None:
            self._xgmi_steps += 1
            if self._xgmi.error_poll() or self._xgmi_steps % self._xgmi_check_every == 0:
                self.check_xgmi()

    def check_xgmi(self) -> None:
        """Raise if any native xGMI all-reduce barrier timed out since creation (its results
        were computed from peer buffers that may be stale: the gradients are corrupt)."""
        if self._xgmi is not None and self._xgmi.error():
            raise RuntimeError("xGMI all-reduce barrier timed out (a peer rank never arrived): "
                               "the small-bucket gradients of this run are corrupt")

    # ------------------------------------------------------------------ conveniences
    def zero_grad(self, set_to_none: bool = True) -> None:
        self._need_reset = True

    @property
    def grad_buffer(self) -> GradBuffer:
        return self.grads

    def bucket_sizes_bytes(self) -> list[int]:
        es = self.grads.buf.element_size()
        return [(b.end - b.start) * es for b in self.buckets]

    def state_dict(self, *a, **k):
        return self.module.state_dict(*a, **k)

    def load_state_dict(self, *a, **k):
        return self.module.load_state_dict(*a, **k)
