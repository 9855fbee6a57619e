"""Process-group bootstrap and communication helpers.

Replaces the reference's ``create_process_group`` (data_parallel_training.py:15-23,
pytorch_allreduce.py:7-15: env MASTER_ADDR=localhost / MASTER_PORT=12355 +
init_process_group('nccl')) and DeepSpeed's ``init_distributed``.

On MI355X the torch backend name ``"nccl"`` is RCCL: collectives run over the xGMI full mesh
(7 point-to-point links per GPU inside a node).  ``init`` pins the HIP device of the local
rank *before* creating the group and passes ``device_id`` so the RCCL communicator is created
eagerly (no lazy first-collective stall inside the timed loop).  gloo is used for CPU runs
and the multi-process CPU tests.
"""
from __future__ import annotations

import datetime
import os
import sys

import torch
import torch.distributed as dist

from . import logger  # noqa: F401
from .logger import (all_gather_into_tensor, all_reduce, all_to_all_single, barrier, broadcast,  # noqa: F401
                     comms_logger, log_summary, reduce, reduce_scatter_tensor)


def env_rank() -> int:
    return int(os.environ.get("RANK", os.environ.get("LOCAL_RANK", "0")))


def env_local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", "0"))


def env_world_size() -> int:
    return int(os.environ.get("WORLD_SIZE", "1"))


def default_backend() -> str:
    return "nccl" if torch.cuda.is_available() else "gloo"


def init(rank: int | None = None, world_size: int | None = None, backend: str | None = None,
         master_addr: str | None = None, master_port: int | str | None = None, local_rank: int | None = None,
         timeout_s: float = 1800.0, init_method: str | None = None,
         high_priority: bool | None = None) -> tuple[int, int]:
    """Initialise the default process group (idempotent).  Returns (rank, world_size).
    ``init_method`` (e.g. ``file:///tmp/x/rdzv``) replaces the TCP rendezvous on MASTER_ADDR /
    MASTER_PORT -- single-host jobs that must not race for a port (tests).

    ``high_priority`` (default: env ``DTD_RCCL_HIGH_PRIORITY``, on): RCCL's internal streams are
    created with high priority, so the dispatcher hands freed CUs to the all-reduce /
    reduce-scatter kernels that DDP and ZeRO launch during backward before the next compute
    workgroups -- the collectives overlap the backward instead of queueing behind it.  The
    persistent GEMMs tolerate the CUs they lose (dynamic tile queue, ops/gemm.py).

    Kernels first launched after the communicator exists run 5-25 % slower for the rest of the
    process: run the step's kernels once before calling this (utils/prewarm.py; the entry
    scripts do)."""
    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    rank = env_rank() if rank is None else rank
    world_size = env_world_size() if world_size is None else world_size
    local_rank = env_local_rank() if local_rank is None else local_rank
    if master_addr is not None or "MASTER_ADDR" not in os.environ:
        os.environ["MASTER_ADDR"] = master_addr or "127.0.0.1"
    if master_port is not None or "MASTER_PORT" not in os.environ:
        os.environ["MASTER_PORT"] = str(master_port or 12355)
    backend = backend or default_backend()
    if backend in ("rccl", "nccl"):
        backend = "nccl"
    kw = {}
    if backend == "nccl":
        torch.cuda.set_device(local_rank)
        kw["device_id"] = torch.device("cuda", local_rank)
        if high_priority is None:
            high_priority = os.environ.get("DTD_RCCL_HIGH_PRIORITY", "1") == "1"
        if high_priority:
            opts = dist.ProcessGroupNCCL.Options()
            opts.is_high_priority_stream = True
            kw["pg_options"] = opts
    if init_method is not None:
        kw["init_method"] = init_method
    dist.init_process_group(backend=backend, rank=rank, world_size=world_size,
                            timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return rank, world_size


def destroy(barrier: bool | None = None) -> None:
    """Orderly teardown: every rank reaches the barrier before any rank closes its transport.
    (Without it a fast rank's exit can close gloo pairs under a peer that is still finishing
    its last collective; that peer's transport thread then aborts the process.)

    ``barrier=None`` skips the barrier when called while an exception is propagating (a
    ``finally`` block on an error path): a dead or stuck peer would otherwise hold every
    surviving rank for the whole process-group timeout."""
    if not dist.is_initialized():
        return
    if barrier is None:
        barrier = sys.exc_info()[0] is None
    try:
        if barrier:
            dist.barrier()
    finally:
        from ..utils.graphs import release_group_graphs
        release_group_graphs()   # graphs holding this group's RCCL work go before the communicator
        dist.destroy_process_group()


def rank() -> int:
    return dist.get_rank() if dist.is_initialized() else 0


def world_size() -> int:
    return dist.get_world_size() if dist.is_initialized() else 1


def is_initialized() -> bool:
    return dist.is_initialized()
