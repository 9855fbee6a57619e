#!/usr/bin/env python
"""Per-kernel time inside ONE training step of a rocprofv3 --kernel-trace database: the window
between the ends of the last two launches of a marker kernel (default: the Adam kernel, one per
step), plus the window's wall span and the GPU-idle time inside it.

  python scripts/diag/step_window.py gpurun_out/r6_mp3/run_results.db [marker-substring]
"""
import collections
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    marker = sys.argv[2] if len(sys.argv) > 2 else "adam_kernel"
    rows = list(db.execute("select name, start, end from kernels order by start"))
    ends = [e for n, s, e in rows if marker in n]
    if len(ends) < 2:
        sys.exit(f"fewer than 2 '{marker}' launches")
    lo, hi = ends[-2], ends[-1]
    win = [(n, s, e) for n, s, e in rows if s >= lo and e <= hi]
    busy, cur_s, cur_e = 0, None, None
    for _, s, e in win:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    span = hi - lo
    print(f"step window {span / 1e6:.2f} ms, GPU busy {busy / 1e6:.2f} ms, idle {(span - busy) / 1e6:.2f} ms, "
          f"{len(win)} kernels")
    agg = collections.defaultdict(lambda: [0, 0])
    for n, s, e in win:
        agg[n][0] += e - s
        agg[n][1] += 1
    for n, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:25]:
        print(f"{t / 1e6:9.3f} ms  n={c:5d}  {n[:110]}")


if __name__ == "__main__":
    main()
