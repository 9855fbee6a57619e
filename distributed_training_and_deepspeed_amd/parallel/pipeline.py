"""Layer-wise model parallelism and GPipe pipelining across the GPUs of one process.

Reference (model/bert_mp.py, model_parallel_training.py):
* naive placement: the flat module list is split into contiguous groups with the
  ``np.array_split`` law (first ``n % d`` groups one longer) and group i lives on device i;
* forward moves activations between groups; only one device works at a time, which the
  per-device idle-time table makes visible;
* ``to_pipeline(chunks)`` wraps the stages in torch's GPipe ``Pipe`` (removed from torch >= 2.4):
  fill-drain schedule over ``chunks`` micro-batches, activation checkpointing of every
  micro-batch except the last, copy streams between devices.

Here: ``GPipe`` issues micro-batch m of stage s at clock t = m + s from one Python thread;
kernel launches are asynchronous per device, so stage s computes micro-batch m while stage
s-1 already runs m+1 (the same overlap torch Pipe gets from per-device worker threads), and
activations move on side copy streams (``parallel/p2p.py``).  Checkpointed micro-batches are
recomputed in backward with *identical* dropout masks, because masks come from the counter
RNG keyed on the micro-batch index (``RngState.micro``) rather than from a saved RNG state.
``IdleTimeTracker`` measures per-device idle gaps with HIP events on each device's stream
(device-accurate) or, like the reference, with host timestamps.
"""
from __future__ import annotations

import time
from datetime import datetime

import torch
from torch import nn
from torch.utils.checkpoint import checkpoint

from .p2p import send_to


def array_split_sizes(n: int, parts: int) -> list[int]:
    """Group sizes of ``np.array_split(range(n), parts)``."""
    q, r = divmod(n, parts)
    return [q + 1 if i < r else q for i in range(parts)]


def partition(modules: list, parts: int) -> list[list]:
    out, i = [], 0
    for sz in array_split_sizes(len(modules), parts):
        out.append(modules[i:i + sz])
        i += sz
    return out


class IdleTimeTracker:
    """Per-device idle time between consecutive forward/backward activities.

    ``timing='device'``: HIP events recorded on the device's current stream at group entry and
    exit; idle = event gap from a device's previous exit to its next entry (resolved at
    ``collect()``).  ``timing='host'``: ``time.time()`` like the reference hooks
    (model/bert_mp.py:106-130).  ``device_idle_time[d] = (sum_ms, count)``."""

    def __init__(self, devices, timing: str = "device", verbose: bool = False):
        self.devices = list(devices)
        self.timing = timing if any(torch.device(d).type == "cuda" for d in self.devices) else "host"
        self.verbose = verbose
        self.device_idle_time = {i: (0.0, 0) for i in range(len(self.devices))}
        self._last = {}
        self._pending = []
        # off while a step is captured into / replayed from a hipGraph: an event recorded during
        # capture is only a dependency marker, not a timestamp
        self.enabled = True

    def _stamp(self, idx: int):
        if self.timing == "host":
            return time.time()
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(torch.device(self.devices[idx])))
        return ev

    def mark(self, idx: int, forward: bool, entering: bool) -> None:
        if not self.enabled:
            return
        now = self._stamp(idx)
        last = self._last.get(idx)
        msg = f"{'Entering' if entering else 'Finished'} {'forward' if forward else 'backward'} pass on device {idx}"
        if entering and last is not None:
            if self.timing == "host":
                ms = (now - last) * 1000.0
                self._add(idx, ms)
                msg += f". Idle time: {ms:.2f}ms"
            else:
                self._pending.append((idx, last, now))
        self._last[idx] = now
        if self.verbose:
            print(f"{datetime.now()} - {msg}")

    def _add(self, idx: int, ms: float) -> None:
        s, c = self.device_idle_time[idx]
        self.device_idle_time[idx] = (s + ms, c + 1)

    def collect(self) -> None:
        if not self._pending:
            return
        torch.cuda.synchronize()
        for idx, a, b in self._pending:
            self._add(idx, max(0.0, a.elapsed_time(b)))
        self._pending = []

    def _collect_ready(self) -> None:
        """Resolve the event pairs that have already completed, without blocking: a per-step
        synchronize would stop the host from queueing the next step while the GPU runs this
        one (2-stage BERT-base b16 on one GPU: 36 ms host-serialised vs 14 ms of kernels)."""
        still = []
        for idx, a, b in self._pending:
            if b.query():
                self._add(idx, max(0.0, a.elapsed_time(b)))
            else:
                still.append((idx, a, b))
        self._pending = still
        if len(self._pending) > 4096:   # bound the number of live events
            self.collect()

    def step_boundary(self) -> None:
        """Idle time is accumulated within a training step (not across optimizer steps)."""
        if self.timing == "host":
            self.collect()
        else:
            self._collect_ready()
        self._last = {}

    def table(self, steps: int) -> list[list]:
        self.collect()
        rows = [["Device", "Average Idle Time (ms)"]]
        for k, (s, _) in self.device_idle_time.items():
            rows.append([k, s / max(steps, 1)])
        return rows


def attach_idle_hooks(groups: list[list[nn.Module]], tracker: IdleTimeTracker) -> None:
    """Forward pre/post hooks and full-backward pre/post hooks on each group's boundary modules.
    (The reference registers its 'entering forward' hook as a post-hook on the group's first
    module -- quirk 6; the pre-hook here measures from the true group entry.)"""
    for idx, g in enumerate(groups):
        first, last = g[0], g[-1]
        first.register_forward_pre_hook(lambda m, a, i=idx: tracker.mark(i, True, True))
        last.register_forward_hook(lambda m, a, o, i=idx: tracker.mark(i, True, False))
        if getattr(last, "token_input", False):   # a group of the embeddings alone
            def _bwd_start(m, a, o, i=idx):
                if torch.is_tensor(o) and o.requires_grad:
                    o.register_hook(lambda g: tracker.mark(i, False, True))
            last.register_forward_hook(_bwd_start)
        else:
            last.register_full_backward_pre_hook(lambda m, go, i=idx: tracker.mark(i, False, True))
        if getattr(first, "token_input", False):
            # the group starts at the embeddings, whose inputs (token ids) take no gradient: a full
            # backward hook there would fire when the gradient of its OUTPUT arrives -- the START
            # of its backward.  The embeddings' backward is the last work of the whole backward
            # pass, so the group's backward ends when the autograd engine finishes: mark it from
            # an engine callback queued when that backward starts.
            # (A tensor hook on the embeddings' output, not a module backward hook: torch warns
            # and misfires module backward hooks on a module whose inputs take no gradient.)
            def _queue_end(g, i=idx):
                torch.autograd.Variable._execution_engine.queue_callback(lambda: tracker.mark(i, False, False))

            def _watch_output(m, a, o, cb=_queue_end):
                if torch.is_tensor(o) and o.requires_grad:
                    o.register_hook(cb)
            first.register_forward_hook(_watch_output)
        else:
            first.register_full_backward_hook(lambda m, gi, go, i=idx: tracker.mark(i, False, False))


class GPipe(nn.Module):
    """Synchronous pipeline (fill-drain) over per-device stages.

    stages[i] is an nn.Module (usually nn.Sequential) resident on devices[i].  ``chunks``
    micro-batches are split along dim 0.  ``checkpoint``: 'except_last' (torch Pipe default),
    'always' or 'never'.  ``set_micro(m)`` (optional) is called before each micro-batch's
    forward and recompute so dropout masks are keyed on the micro-batch."""

    def __init__(self, stages, devices, chunks: int = 1, checkpoint: str = "except_last", set_micro=None,
                 owner: nn.Module | None = None):
        super().__init__()
        self.stages = nn.ModuleList(stages)
        self.owner = owner  # the full model: makes .parameters() / .train() cover every stage
        self.devices = [torch.device(d) for d in devices]
        self.chunks = chunks
        self.checkpoint = checkpoint
        self.set_micro = set_micro

    def _run(self, s: int, m: int, x):
        def fn(inp, _s=s, _m=m):
            if self.set_micro is not None:
                self.set_micro(_m)
            return self.stages[_s](inp)
        ck = (self.checkpoint == "always") or (self.checkpoint == "except_last" and m < self.chunks - 1)
        if ck and torch.is_grad_enabled() and self.training:
            return checkpoint(fn, x, use_reentrant=False, preserve_rng_state=False)
        return fn(x)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        micro = list(torch.chunk(x, self.chunks, dim=0))
        n, S = len(micro), len(self.stages)
        acts = [[None] * n for _ in range(S)]
        for clock in range(n + S - 1):
            for s in range(S):
                m = clock - s
                if not 0 <= m < n:
                    continue
                inp = micro[m] if s == 0 else acts[s - 1][m]
                inp = send_to(inp, self.devices[s]) if torch.is_tensor(inp) else inp
                with torch.cuda.device(self.devices[s]) if self.devices[s].type == "cuda" else _null():
                    acts[s][m] = self._run(s, m, inp)
                if s > 0:
                    acts[s - 1][m] = None
        if self.set_micro is not None:
            self.set_micro(0)
        return torch.cat(acts[S - 1], dim=0)

    def local_value(self):  # torch Pipe returned an RRef; kept for script-level parity
        return self

    def train_step(self, x: torch.Tensor, target: torch.Tensor, loss_fn, schedule: str = "1f1b",
                   loss_weighting: str = "tokens", ignore_index: int = -100) -> torch.Tensor:
        """Forward + backward of one mini-batch; returns the mini-batch loss.

        ``1f1b``: after S-1 warm-up forwards, every new micro-batch forward is followed by the
        backward of the oldest one, so at most S micro-batches hold activations at a time
        (GPipe fill-drain keeps all ``chunks``, which is why torch Pipe checkpoints them).
        Backward of micro-batch m on stage s and forward of m+S-1 on stage 0 run on different
        devices and overlap.  ``gpipe``: all forwards, then all backwards.  The loss of each
        micro-batch is ``loss_fn(out, target_chunk)`` weighted by its share of the batch's labelled
        tokens (``loss_weighting="tokens"``: the loss of the concatenated batch, as ``forward`` +
        one loss gives -- stage_pipeline.micro_loss_weights) or by 1 / chunks ("mean")."""
        from .stage_pipeline import micro_loss_weights
        if schedule not in ("1f1b", "gpipe"):
            raise ValueError(schedule)
        mx = list(torch.chunk(x, self.chunks, dim=0))
        mt = list(torch.chunk(target, self.chunks, dim=0))
        n, S = len(mx), len(self.stages)
        pending, total = [], None
        weights = (micro_loss_weights(target.to(self.devices[-1]), n, ignore_index) if loss_weighting == "tokens"
                   else None)

        def fwd(m):
            h = mx[m]
            for s in range(S):
                h = send_to(h, self.devices[s]) if torch.is_tensor(h) else h
                with torch.cuda.device(self.devices[s]) if self.devices[s].type == "cuda" else _null():
                    h = self._run(s, m, h)
            loss = loss_fn(h, mt[m].to(h.device))
            loss = loss * weights[m].to(loss.device) if weights is not None else loss / n
            pending.append(loss)
            return loss.detach()

        def bwd():
            pending.pop(0).backward()

        warm = n if schedule == "gpipe" else min(S - 1, n)
        for m in range(n):
            ls = fwd(m)
            total = ls if total is None else total + ls.to(total.device)
            if m >= warm:
                bwd()
        while pending:
            bwd()
        if self.set_micro is not None:
            self.set_micro(0)
        return total


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
