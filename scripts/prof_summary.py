#!/usr/bin/env python
"""Summarise a rocprofv3 kernel trace: top kernels by total time, per-step ms.

Input: the --stats kernel_stats.csv, or the rocpd SQLite database (``*_results.db``, the default
output of rocprofv3 without --output-format csv) -- its ``kernels`` view is grouped by name here.
Usage: prof_summary.py FILE [steps] [top]"""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
if path.endswith(".db"):
    import sqlite3
    con = sqlite3.connect(path)
    q = "select name, count(*), sum(duration), avg(duration) from kernels group by name"
    agg = con.execute(q).fetchall()
    total = sum(r[2] for r in agg) or 1
    rows = [{"Name": n, "Calls": c, "TotalDurationNs": t, "AverageNs": a, "Percentage": 100.0 * t / total}
            for n, c, t, a in agg]
else:
    rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.2f} ms  ({tot/1e6/steps:.2f} ms/step over {steps:g} steps)")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[: int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    t = float(r["TotalDurationNs"]) / 1e6
    print(f"{t/steps:8.3f} ms/step {float(r['Percentage']):6.2f}%  n={int(r['Calls'])/steps:7.1f}/step "
          f"avg={float(r['AverageNs'])/1e3:8.1f}us  {r['Name'][:100]}")
