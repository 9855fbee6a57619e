"""Phase markers and step metrics.

* ``marker(name)``: a roctx range (``torch.cuda.nvtx`` maps to roctx on ROCm) around a training
  phase -- forward / backward / comm / optimizer -- so ``rocprofv3 --marker-trace`` timelines
  show where each kernel belongs.  Enabled by ``DTD_MARKERS=1`` or ``enable_markers()``; free
  when disabled.
* ``StepTimer``: HIP-event step timing without per-step host syncs (events are resolved at the
  end), producing the ``--metrics-json`` record: tokens/s, step-time percentiles, peak HBM.
"""
from __future__ import annotations

import contextlib
import json
import os

import torch

_ON = [os.environ.get("DTD_MARKERS", "0") == "1"]


def enable_markers(on: bool = True) -> None:
    _ON[0] = on


@contextlib.contextmanager
def marker(name: str):
    if not (_ON[0] and torch.cuda.is_available()):
        yield
        return
    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()


class StepTimer:
    """Per-step device time from HIP events recorded on the current stream."""

    def __init__(self, tokens_per_step: int, world_size: int = 1):
        self.tokens, self.world = tokens_per_step, world_size
        self.events: list = []
        self.cuda = torch.cuda.is_available()
        self._t0 = None

    def start(self):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._t0 = e
        else:
            import time
            self._t0 = time.perf_counter()

    def stop(self):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.events.append((self._t0, e))
        else:
            import time
            self.events.append(time.perf_counter() - self._t0)

    def step_ms(self) -> list[float]:
        if self.cuda:
            if self.events:
                self.events[-1][1].synchronize()
            return [a.elapsed_time(b) for a, b in self.events]
        return [t * 1e3 for t in self.events]

    def summary(self) -> dict:
        ms = sorted(self.step_ms())
        if not ms:
            return {}

        def pct(q):
            return ms[min(len(ms) - 1, int(round(q * (len(ms) - 1))))]
        mean = sum(ms) / len(ms)
        out = {"steps": len(ms), "step_ms_mean": mean, "step_ms_p50": pct(0.5), "step_ms_p90": pct(0.9),
               "step_ms_max": ms[-1], "tokens_per_s": self.tokens * self.world / (mean / 1e3)}
        if self.cuda:
            out["peak_hbm_gb"] = torch.cuda.max_memory_allocated() / 1e9
        return out

    def write(self, path: str, extra: dict | None = None) -> dict:
        rec = {**self.summary(), **(extra or {})}
        with open(path, "w") as f:
            json.dump(rec, f, indent=1)
        return rec
