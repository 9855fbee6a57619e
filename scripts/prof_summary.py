#!/usr/bin/env python
"""Summarise a rocprofv3 --stats kernel_stats.csv: top kernels by total time, per-step ms."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.2f} ms  ({tot/1e6/steps:.2f} ms/step over {steps:g} steps)")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[: int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    t = float(r["TotalDurationNs"]) / 1e6
    print(f"{t/steps:8.3f} ms/step {float(r['Percentage']):6.2f}%  n={int(r['Calls'])/steps:7.1f}/step "
          f"avg={float(r['AverageNs'])/1e3:8.1f}us  {r['Name'][:100]}")
