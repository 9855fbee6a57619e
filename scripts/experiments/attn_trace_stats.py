#!/usr/bin/env python
"""Summarise attn_trace CSVs (s_memrealtime ticks, 100 MHz): per-phase workgroup times and
in-flight workgroup counts over the kernel's span."""
import csv
import statistics as st
import sys

for path in sys.argv[1:]:
    rows = [[int(x) for x in r.values()] for r in csv.DictReader(open(path))]
    t0 = min(r[1] for r in rows)
    us = lambda a, b: [(r[b] - r[a]) / 100.0 for r in rows]  # noqa: E731
    span = (max(r[7] for r in rows) - t0) / 100.0
    def q(v):
        v = sorted(v)
        return f"p10 {v[len(v) // 10]:.2f} med {st.median(v):.2f} p90 {v[9 * len(v) // 10]:.2f} mean {st.mean(v):.2f}"
    print(path, f"workgroups {len(rows)} span {span:.1f} us")
    for name, a, b in [("prologue", 1, 2), ("tile0", 2, 3), ("mid tiles", 3, 4), ("last tile", 4, 5),
                       ("pre-epi", 5, 6), ("epilogue", 6, 7), ("total", 1, 7)]:
        print(f"  {name:10s} {q(us(a, b))}")
    starts = sorted((r[1] - t0) / 100.0 for r in rows)
    ends = sorted((r[7] - t0) / 100.0 for r in rows)
    for frac in (0.0, 0.25, 0.5, 0.75, 0.95):
        t = frac * span
        inflight = sum(1 for s in starts if s <= t) - sum(1 for e in ends if e <= t)
        print(f"  t={t:6.1f} us in flight {inflight}")
    print("  first-wave start spread (first 768 starts): "
          f"{starts[min(767, len(starts) - 1)] - starts[0]:.2f} us; last start {starts[-1]:.1f} us")
