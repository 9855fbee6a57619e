"""Logged collectives (the ``deepspeed.comm`` comms-logger equivalent).

Reference: zero_dp_training.py:34-39 enables DeepSpeed's comms logger with ``prof_all``, resets
``dist.comms_logger.comms_dict`` before the loop (:74), sums ``comms_dict[op][size][1]`` and
calls ``dist.log_summary()`` (:102-112).  SURVEY.md D13.  Same record layout here:
``comms_dict[op_name][msg_bytes] = [count, [latency_ms...], [algbw_Gbps...], [busbw_Gbps...]]``.

MI355X-first timing: DeepSpeed synchronises the device around every logged op, which
serialises communication with compute (reference quirk 13).  Here each GPU collective is
bracketed by HIP events -- the start event on the issuing stream, the end event on a side
stream that waits on the collective's work handle -- and the events are resolved lazily when
the summary is requested, so logging never blocks the host or breaks comm/compute overlap.
(``sync_timing=True`` reproduces DeepSpeed's synchronous measurements.)  Latency is from
issue to completion as seen by the stream, i.e. it includes queueing behind earlier
collectives.  Bus bandwidth uses the nccl-tests convention: all_reduce x 2(n-1)/n,
all_gather / reduce_scatter x (n-1)/n.
"""
from __future__ import annotations

import time

import torch
import torch.distributed as dist


def _busbw_factor(op: str, n: int) -> float:
    if n <= 1:
        return 0.0 if op == "barrier" else 1.0
    if op == "all_reduce":
        return 2.0 * (n - 1) / n
    if op in ("all_gather", "all_gather_into_tensor", "reduce_scatter", "reduce_scatter_tensor", "all_to_all_single"):
        return (n - 1) / n
    if op == "barrier":
        return 0.0
    return 1.0


def _fmt_size(b: int) -> str:
    for unit in ("B", "KB", "MB", "GB"):
        if b < 1024 or unit == "GB":
            return f"{b:.2f} {unit}" if unit != "B" else f"{b} B"
        b /= 1024.0
    return str(b)


class CommsLogger:
    def __init__(self):
        self.enabled = False
        self.prof_all = True
        self.prof_ops: list[str] = []
        self.verbose = False
        self.debug = False
        self.sync_timing = False
        self.comms_dict: dict = {}
        self._pending: list = []
        self._side: dict = {}

    def configure(self, cfg: dict | None = None, **kw) -> None:
        cfg = dict(cfg or {})
        cfg.update(kw)
        self.enabled = bool(cfg.get("enabled", self.enabled))
        self.prof_all = bool(cfg.get("prof_all", self.prof_all))
        self.prof_ops = list(cfg.get("prof_ops", self.prof_ops))
        self.verbose = bool(cfg.get("verbose", self.verbose))
        self.debug = bool(cfg.get("debug", self.debug))
        self.sync_timing = bool(cfg.get("sync_timing", self.sync_timing))

    def reset(self) -> None:
        self._resolve()
        self.comms_dict = {}

    def should_log(self, op: str) -> bool:
        return self.enabled and (self.prof_all or op in self.prof_ops)

    # -- recording
    def _record(self, op: str, nbytes: int, ms: float, world: int) -> None:
        algbw = (nbytes * 8 / 1e9) / (ms / 1e3) if ms > 0 else 0.0  # Gbps
        busbw = algbw * _busbw_factor(op, world)
        rec = self.comms_dict.setdefault(op, {}).setdefault(nbytes, [0, [], [], []])
        rec[0] += 1
        rec[1].append(ms)
        rec[2].append(algbw)
        rec[3].append(busbw)
        if self.verbose:
            print(f"comm op: {op} | time (ms): {ms:.3f} | msg size: {_fmt_size(nbytes)} | "
                  f"algbw (Gbps): {algbw:.2f} | busbw (Gbps): {busbw:.2f}")

    def _resolve(self) -> None:
        still = []
        for op, nbytes, start, end, world in self._pending:
            if end.query():
                self._record(op, nbytes, start.elapsed_time(end), world)
            else:
                still.append((op, nbytes, start, end, world))
        if still:
            torch.cuda.synchronize()
            for op, nbytes, start, end, world in still:
                self._record(op, nbytes, start.elapsed_time(end), world)
        self._pending = []

    def _side_stream(self, device):
        k = str(device)
        if k not in self._side:
            self._side[k] = torch.cuda.Stream(device)
        return self._side[k]

    def run(self, op: str, fn, tensor: torch.Tensor | None, nbytes: int, group, async_op: bool):
        """Execute collective ``fn(async_op=...)`` with timing; returns its work/None."""
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        if not self.should_log(op) or (tensor is not None and tensor.is_cuda and torch.cuda.is_current_stream_capturing()):
            # (inside a hipGraph capture the timing side stream would be left un-joined and the
            # synchronising form is illegal: captured collectives are not logged)
            return fn(async_op)
        gpu = tensor is not None and tensor.is_cuda
        if gpu and not self.sync_timing:
            start = torch.cuda.Event(enable_timing=True)
            end = torch.cuda.Event(enable_timing=True)
            start.record()
            work = fn(True)
            side = self._side_stream(tensor.device)
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                if work is not None:
                    work.wait()
                end.record()
            self._pending.append((op, nbytes, start, end, world))
            if len(self._pending) > 4096:
                self._resolve()
            if async_op:
                return work
            if work is not None:
                work.wait()
            return None
        if gpu:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        work = fn(True)
        if work is not None:
            work.wait()
        if gpu:
            torch.cuda.synchronize()
        self._record(op, nbytes, (time.perf_counter() - t0) * 1e3, world)
        return _DoneWork() if async_op else None

    # -- summary
    def total_latency_ms(self, skip=("log_summary_barrier",)) -> float:
        self._resolve()
        return sum(sum(v[1]) for op, d in self.comms_dict.items() if op not in skip for v in d.values())

    def summary(self) -> str:
        self._resolve()
        hdr = f"{'Comm. Op':<22}{'Message Size':<16}{'Count':<8}{'Total Latency(ms)':<20}{'Avg Latency(ms)':<18}{'tput_avg (Gbps)':<18}{'busbw_avg (Gbps)':<18}"
        lines = [hdr]
        for op in sorted(self.comms_dict):
            lines.append(op)
            for size in sorted(self.comms_dict[op]):
                cnt, lat, alg, bus = self.comms_dict[op][size]
                tot = sum(lat)
                lines.append(f"{'':<22}{_fmt_size(size):<16}{cnt:<8}{tot:<20.2f}{tot / cnt:<18.3f}"
                             f"{sum(alg) / cnt:<18.2f}{sum(bus) / cnt:<18.2f}")
        return "\n".join(lines)


class _DoneWork:
    def wait(self):
        return True

    def is_completed(self):
        return True


comms_logger = CommsLogger()


# ---------------------------------------------------------------------- logged collectives
def _nbytes(t: torch.Tensor) -> int:
    return t.numel() * t.element_size()


def all_reduce(tensor, op=dist.ReduceOp.SUM, group=None, async_op=False):
    return comms_logger.run("all_reduce", lambda a: dist.all_reduce(tensor, op=op, group=group, async_op=a),
                            tensor, _nbytes(tensor), group, async_op)


def broadcast(tensor, src=0, group=None, async_op=False):
    return comms_logger.run("broadcast", lambda a: dist.broadcast(tensor, src=src, group=group, async_op=a),
                            tensor, _nbytes(tensor), group, async_op)


def _gloo_cuda(t: torch.Tensor, group) -> bool:
    """gloo on GPU tensors (several ranks sharing one GPU in tests): gloo implements all_reduce /
    all_gather for device tensors but not the fused-buffer reduce-scatter / all-gather forms."""
    return t.is_cuda and dist.is_initialized() and dist.get_backend(group) == "gloo"


def reduce_scatter_tensor(output, input, op=dist.ReduceOp.SUM, group=None, async_op=False):
    def fn(a):
        if _gloo_cuda(input, group):   # all-reduce a copy, keep this rank's chunk
            tmp = input.clone()
            dist.all_reduce(tmp, op=op, group=group)
            output.copy_(tmp.view(dist.get_world_size(group), -1)[dist.get_rank(group)].view_as(output))
            return _DoneWork() if a else None
        return dist.reduce_scatter_tensor(output, input, op=op, group=group, async_op=a)
    return comms_logger.run("reduce_scatter_tensor", fn, input, _nbytes(input), group, async_op)


def all_gather_into_tensor(output, input, group=None, async_op=False):
    def fn(a):
        if _gloo_cuda(output, group):   # list form into row views of the output
            dist.all_gather(list(output.view(dist.get_world_size(group), -1).unbind(0)), input.reshape(-1),
                            group=group)
            return _DoneWork() if a else None
        return dist.all_gather_into_tensor(output, input, group=group, async_op=a)
    return comms_logger.run("all_gather_into_tensor", fn, output, _nbytes(output), group, async_op)


class _MultiWork:
    """Work handle over several collectives (the gloo fallback of the coalesced calls)."""

    def __init__(self, works):
        self.works = [w for w in works if w is not None]

    def wait(self):
        for w in self.works:
            w.wait()
        return True

    def is_completed(self):
        return all(w.is_completed() for w in self.works)


def all_gather_coalesced(outputs, inputs, group=None, async_op=False):
    """Several ``all_gather_into_tensor`` calls as ONE RCCL group launch (ncclGroupStart/End via
    torch's coalescing manager) on the nccl backend; one call each elsewhere.  Logged as one
    all_gather_into_tensor of the summed size (DeepSpeed's ``allgather_bucket_size`` unit)."""
    outputs, inputs = list(outputs), list(inputs)
    nccl = dist.is_initialized() and dist.get_backend(group) == "nccl"

    def fn(a):
        # one RCCL group launch -- except inside a hipGraph capture, where torch's coalescing
        # manager is not capturable (the capture's end-of-capture crashed in it): there each
        # gather is its own captured RCCL call
        capturing = outputs and outputs[0].is_cuda and torch.cuda.is_current_stream_capturing()
        if nccl and len(outputs) > 1 and not capturing:
            with dist._coalescing_manager(group=group, device=outputs[0].device, async_ops=True) as cm:
                for o, i in zip(outputs, inputs):
                    dist.all_gather_into_tensor(o, i, group=group)
            if a:
                return cm
            cm.wait()
            return None
        if outputs and _gloo_cuda(outputs[0], group):
            for o, i in zip(outputs, inputs):
                all_gather_into_tensor(o, i, group=group)
            return _DoneWork() if a else None
        works = [dist.all_gather_into_tensor(o, i, group=group, async_op=a) for o, i in zip(outputs, inputs)]
        return _MultiWork(works) if a else None

    return comms_logger.run("all_gather_into_tensor", fn, outputs[0] if outputs else None,
                            sum(_nbytes(o) for o in outputs), group, async_op)


def all_to_all_single(output, input, group=None, async_op=False):
    return comms_logger.run("all_to_all_single",
                            lambda a: dist.all_to_all_single(output, input, group=group, async_op=a),
                            input, _nbytes(input), group, async_op)


def reduce(tensor, dst, op=dist.ReduceOp.SUM, group=None, async_op=False):
    return comms_logger.run("reduce", lambda a: dist.reduce(tensor, dst=dst, op=op, group=group, async_op=a),
                            tensor, _nbytes(tensor), group, async_op)


def send(tensor, dst, group=None):
    return comms_logger.run("send", lambda a: dist.isend(tensor, dst=dst, group=group) if a else dist.send(tensor, dst=dst, group=group),
                            tensor, _nbytes(tensor), group, False)


def recv(tensor, src, group=None):
    return comms_logger.run("recv", lambda a: dist.irecv(tensor, src=src, group=group) if a else dist.recv(tensor, src=src, group=group),
                            tensor, _nbytes(tensor), group, False)


def isend(tensor, dst, group=None):
    """Non-blocking point-to-point send (logged as "send"); returns the work handle."""
    return comms_logger.run("send", lambda a: dist.isend(tensor, dst=dst, group=group) if a else dist.send(tensor, dst=dst, group=group),
                            tensor, _nbytes(tensor), group, True)


def irecv(tensor, src, group=None):
    """Non-blocking point-to-point receive into ``tensor`` (logged as "recv"); returns the work handle."""
    return comms_logger.run("recv", lambda a: dist.irecv(tensor, src=src, group=group) if a else dist.recv(tensor, src=src, group=group),
                            tensor, _nbytes(tensor), group, True)


def barrier(group=None, name: str = "barrier"):
    if not dist.is_initialized():
        return
    t0 = time.perf_counter()
    dist.barrier(group=group)
    if comms_logger.should_log(name):
        comms_logger._record(name, 0, (time.perf_counter() - t0) * 1e3, dist.get_world_size(group))


def log_summary(show_straggler: bool = False) -> None:
    """Barrier then rank-0 print of the per-op/size table (deepspeed.comm.log_summary)."""
    barrier(name="log_summary_barrier")
    rank = dist.get_rank() if dist.is_initialized() else 0
    if rank == 0:
        print(comms_logger.summary())
