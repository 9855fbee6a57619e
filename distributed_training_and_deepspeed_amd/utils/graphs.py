"""Whole-training-step HIP graphs (the MI355X alternative to a tracing compiler).

At small per-GPU batches (the reference's 4 x 512 tokens) a BERT-base step is ~300 kernel
launches of a few microseconds each and the host becomes the bottleneck.  ``CapturedStep``
records one complete step -- forward, backward with the DDP bucket reductions, fused optimizer,
dropout-RNG advance -- into a ``torch.cuda.CUDAGraph`` (hipGraph) once, then replays it with one
launch per step after copying the new batch into static input buffers.

What makes the step capturable (and is kept that way by the framework):
* every kernel goes onto torch's current stream (ops/_lib.py), side streams fork from and join
  back into it (attention-mask generation);
* no host synchronisation inside the step: optimizer hyper-parameters, the Adam step count and
  the dropout RNG step live in device memory and are updated by kernels; the sparse MLM head
  uses a static row capacity (``rt.mlm_capacity``) with a device-side overflow flag;
* gradient buffers, buckets and the optimizer state are persistent (flat buffers), so replays
  write the same addresses.
``check()`` reads the overflow flag (one sync; call it occasionally, e.g. at the end).
"""
from __future__ import annotations

import gc
import math
import weakref

import torch

# captured steps recorded while a process group existed (their graphs may hold RCCL work)
_WITH_GROUP: "weakref.WeakSet[CapturedStep]" = weakref.WeakSet()


def mlm_capacity(tokens: int, p: float = 0.15, sigmas: float = 8.0) -> int:
    """Static labelled-row capacity: mean + 8 sigma of Binomial(tokens, p) (+64), capped."""
    mean, sd = tokens * p, math.sqrt(tokens * p * (1 - p))
    return min(tokens, int(math.ceil(mean + sigmas * sd)) + 64)


# Captures run with capture_error_mode="thread_local": only the capturing thread is barred from
# capture-unsafe HIP calls.  ProcessGroupNCCL's watchdog thread polls the end events of enqueued
# collectives (hipEventQuery) every 100 ms; under the default global mode one of those polls landing
# inside the capture aborted the process ("operation not permitted when stream is capturing",
# profiles/r5_capture_results.jsonl).  Work that other threads put on the capturing stream (the
# autograd engine's backward, DDP's bucket all-reduces) is still captured: capture is per stream.
CAPTURE_ERROR_MODE = "thread_local"


class CapturedStep:
    def __init__(self, step_fn, static_inputs: dict, warmup: int = 3, runtime=None, warmup_batches=None):
        """``step_fn(**inputs)`` runs one full training step and returns a tensor (the loss).
        ``warmup`` real steps run eagerly on a side stream first (library handles, GEMM
        solution lookup and allocator pools must exist before capture).  ``warmup_batches``
        (list of input dicts): run those batches as the warm-up steps instead of repeating
        ``static_inputs``, so a trainer can count them as its first training steps (the
        capture itself computes nothing: only replays do); their losses are in
        ``self.warmup_losses``."""
        self.rt = runtime
        if runtime is not None and runtime.mlm_overflow is None:
            runtime.mlm_overflow = torch.zeros((), dtype=torch.bool, device="cuda")
        self.static = {k: v.detach().clone() for k, v in static_inputs.items()}
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        batches = list(warmup_batches) if warmup_batches is not None else [self.static] * warmup
        self.warmup_losses = []
        with torch.cuda.stream(side):
            for b in batches:
                self.warmup_losses.append(step_fn(**b))
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, capture_error_mode=CAPTURE_ERROR_MODE):
            self.out = step_fn(**self.static)
        self.warmup = len(batches)
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            _WITH_GROUP.add(self)

    def release(self) -> None:
        """Destroy the graph (and its memory pool) now rather than whenever the garbage collector
        reaches this object."""
        if self.graph is not None:
            torch.cuda.synchronize()
            self.graph.reset()
        self.graph, self.out = None, None

    def __call__(self, **inputs):
        if self.graph is None:
            raise RuntimeError("CapturedStep: the graph was released (comm.destroy() releases the graphs "
                               "captured with its process group)")
        for k, v in inputs.items():
            self.static[k].copy_(v, non_blocking=True)
        self.graph.replay()
        return self.out

    def check(self) -> None:
        if self.rt is not None and self.rt.mlm_overflow is not None and bool(self.rt.mlm_overflow):
            raise RuntimeError("a batch had more labelled rows than rt.mlm_capacity: raise the capacity")


def release_group_graphs() -> None:
    """Reset every live captured step recorded while a process group existed.  ``comm.destroy()``
    calls this before destroying the group, so a hipGraph holding RCCL collectives never outlives
    its communicator (a step object kept alive by a reference cycle would otherwise be destroyed at
    some later garbage collection, after the communicator is gone)."""
    gc.collect()
    for cs in list(_WITH_GROUP):
        cs.release()
    _WITH_GROUP.clear()
