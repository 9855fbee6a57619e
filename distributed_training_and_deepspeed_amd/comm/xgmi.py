"""Native peer-mapped all-reduce over xGMI (``comm/csrc/xgmi_allreduce.hip``).

SURVEY.md D2 / 2.6: besides RCCL (torch's ``nccl`` backend), the framework ships its own
latency-optimised all-reduce for the small messages of a training step -- the last DDP
buckets, ZeRO bookkeeping scalars, gradient-norm reductions -- where a ring's per-hop latency
dominates.  Each rank allocates a staging buffer + a fine-grained signal array, the IPC handles
are exchanged once through the process group, and every call is ONE kernel launch on the
caller's stream that reads the peers' buffers directly over the xGMI full mesh:

* ``one-shot`` (messages <= ``one_shot_max``): copy in, barrier, sum all n peers' copies;
* ``two-shot`` (larger, ``numel % (8 world) == 0``): reduce-scatter + all-gather through the
  peers' result buffers -- 2(n-1)/n of the bytes per GPU, all 7 links busy at once.

Results are bitwise identical on every rank (fixed summation order).  Every barrier spin is
bounded: when a peer never arrives the kernel sets a device error flag and still finishes, so
that call's result is summed over possibly stale peer data (CORRUPT) -- callers must poll
``error()`` (DDP does every ``xgmi_check_every`` steps and raises).  Messages above
``max_bytes`` or with odd sizes fall back to RCCL.  ``XgmiAllReduce.local(world)`` builds the
single-process variant (``world`` virtual ranks on one GPU) used by the tests on a 1-GPU box.

Status: the kernel logic, the barrier protocol and the epoch double-buffering are tested in
local mode on one MI355X, and the IPC path (handle exchange, ``hipIpcOpenMemHandle`` mapping,
cross-process release/acquire barrier) with 2 and 4 processes sharing one MI355X
(``tests/test_xgmi_gpu.py::test_ipc_mode_processes_share_one_gpu``).  Cross-GPU xGMI traffic
needs a multi-GPU node; the path is opt-in (``DistributedDataParallel(small_bucket_allreduce="xgmi")``).
"""
from __future__ import annotations

import ctypes

import torch
import torch.distributed as dist

from ..ops import _lib

P = ctypes.c_void_p
_SIGS = {
    "dtd_xgmi_max_ranks": (ctypes.c_int, []),
    "dtd_xgmi_handle_bytes": (ctypes.c_int, []),
    "dtd_xgmi_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_longlong, ctypes.POINTER(P), P]),
    "dtd_xgmi_create_local": (ctypes.c_int, [ctypes.c_int, ctypes.c_longlong, ctypes.POINTER(P)]),
    "dtd_xgmi_open": (ctypes.c_int, [P, P]),
    "dtd_xgmi_destroy": (ctypes.c_int, [P]),
    "dtd_xgmi_error": (ctypes.c_int, [P, P]),
    "dtd_xgmi_error_poll": (ctypes.c_int, [P, P, P]),
    "dtd_xgmi_allreduce": (ctypes.c_int, [P, P, P, ctypes.c_longlong, ctypes.c_int, ctypes.c_int, ctypes.c_uint,
                                          ctypes.c_float, ctypes.c_int, P]),
}


def _L():
    lib = _lib.lib()
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        if fn.argtypes is None or list(fn.argtypes) != args:
            fn.restype, fn.argtypes = res, args
    return lib


class XgmiAllReduce:
    """In-place ``all_reduce(SUM)`` of bf16/fp32 CUDA tensors through peer-mapped buffers."""

    def __init__(self, group=None, max_bytes: int = 8 << 20, one_shot_max: int = 256 << 10, blocks: int = 32,
                 _local_world: int = 0):
        self.lib = _L()
        self.max_bytes = int(max_bytes)
        self.one_shot_max = int(one_shot_max)
        self.blocks = blocks
        self.epoch = 0
        self.ctx = P()
        if _local_world:
            self.world, self.rank, self.local = _local_world, 0, _local_world
            rc = self.lib.dtd_xgmi_create_local(_local_world, self.max_bytes, ctypes.byref(self.ctx))
            if rc:
                raise RuntimeError(f"dtd_xgmi_create_local failed ({rc})")
            return
        self.group = group
        self.world, self.rank, self.local = dist.get_world_size(group), dist.get_rank(group), 0
        if self.world > self.lib.dtd_xgmi_max_ranks():
            raise ValueError(f"xGMI all-reduce supports <= {self.lib.dtd_xgmi_max_ranks()} ranks (one node)")
        nb = self.lib.dtd_xgmi_handle_bytes()
        buf = ctypes.create_string_buffer(nb)
        rc = self.lib.dtd_xgmi_create(self.rank, self.world, self.max_bytes, ctypes.byref(self.ctx), buf)
        if rc:
            raise RuntimeError(f"dtd_xgmi_create failed ({rc})")
        handles: list = [None] * self.world
        dist.all_gather_object(handles, buf.raw, group=group)
        allh = ctypes.create_string_buffer(b"".join(handles), nb * self.world)
        rc = self.lib.dtd_xgmi_open(self.ctx, allh)
        if rc:
            raise RuntimeError(f"dtd_xgmi_open failed ({rc}): peers not IPC-mappable (not one node?)")
        dist.barrier(group=group)

    @classmethod
    def local(cls, world: int, max_bytes: int = 8 << 20, **kw) -> "XgmiAllReduce":
        return cls(max_bytes=max_bytes, _local_world=world, **kw)

    def supports(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.is_contiguous() and t.dtype in (torch.bfloat16, torch.float32)
                and t.numel() % 8 == 0 and t.numel() * t.element_size() <= self.max_bytes)

    def _mode(self, numel: int, nbytes: int) -> int:
        if nbytes <= self.one_shot_max or numel % (8 * self.world):
            return 0
        return 1

    def all_reduce_local(self, tensors: list[torch.Tensor], mode: int | None = None, scale: float = 1.0) -> None:
        """Local mode: ``tensors[r]`` is virtual rank r's buffer; all are reduced in place."""
        assert self.local and len(tensors) == self.local
        t0 = tensors[0]
        assert all(self.supports(t) and t.shape == t0.shape and t.dtype == t0.dtype for t in tensors)
        self._launch([t.data_ptr() for t in tensors], [t.data_ptr() for t in tensors], t0, mode, scale)

    def all_reduce(self, t: torch.Tensor, mode: int | None = None, average: bool = False) -> torch.Tensor:
        """In-place sum (or mean) over the group; falls back to RCCL when the message does not fit."""
        if self.local:
            raise RuntimeError("local-mode instance: use all_reduce_local")
        if not self.supports(t):
            dist.all_reduce(t, op=dist.ReduceOp.AVG if average else dist.ReduceOp.SUM, group=self.group)
            return t
        self._launch([t.data_ptr()], [t.data_ptr()], t, mode, 1.0 / self.world if average else 1.0)
        return t

    def _launch(self, ins, outs, t, mode, scale=1.0):
        n = len(ins)
        mode = self._mode(t.numel(), t.numel() * t.element_size()) if mode is None else mode
        self.epoch = (self.epoch + 1) & 0xFFFFFFFF or 1
        ia = (P * n)(*ins)
        oa = (P * n)(*outs)
        rc = self.lib.dtd_xgmi_allreduce(self.ctx, ia, oa, t.numel(), _lib.dt(t), mode, self.epoch, scale, self.blocks,
                                         _lib.stream())
        if rc:
            raise RuntimeError(f"dtd_xgmi_allreduce failed ({rc})")

    def error(self) -> bool:
        """True if a barrier timed out (a peer never arrived) since creation."""
        return bool(self.lib.dtd_xgmi_error(self.ctx, _lib.stream()))

    def error_poll(self) -> bool:
        """Non-blocking check: True if a barrier timeout was seen by an EARLIER poll.  Each call
        reads the pinned host word that the previous call's async copy filled, then queues a new
        copy on the current stream -- the exposure window is the one step between polls."""
        if getattr(self, "_herr", None) is None:
            self._herr = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        seen = bool(int(self._herr[0]))
        self.lib.dtd_xgmi_error_poll(self.ctx, self._herr.data_ptr(), _lib.stream())
        return seen

    def close(self) -> None:
        if self.ctx:
            self.lib.dtd_xgmi_destroy(self.ctx)
            self.ctx = P()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
