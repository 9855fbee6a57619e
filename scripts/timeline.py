#!/usr/bin/env python
"""Kernel-timeline analysis of a rocprofv3 --kernel-trace CSV: for the last N training steps
(delimited by the fused Adam kernel, one per step), the busy union of all kernels vs the step's
wall span (GPU idle gaps), time per kernel class, and how much of the side-stream dropout-mask
generation overlaps other work."""
import csv
import sys
from collections import defaultdict


def classify(name):
    n = name
    if "attn_mask" in n:
        return "attn_mask"
    if "attn_" in n:
        return "attention"
    if "Cijk" in n or "gemm" in n.lower():
        return "gemm"
    if "ln_" in n:
        return "layernorm"
    if "act_" in n:
        return "activation"
    if "adam" in n:
        return "adam"
    if "nccl" in n.lower() or "rccl" in n.lower():
        return "collective"
    return "other"


def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot


def per_sum(win, cls):
    return sum(e - s for s, e, n in win if classify(n) == cls)


def main(path, nsteps=3):
    rows = list(csv.DictReader(open(path)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    ks.sort()
    adam = [(s, e) for s, e, n in ks if "adam_kernel" in n]
    # one step boundary per optimizer step: the last Adam kernel of a burst (the staged optimizer,
    # FusedAdam.overlap_with_forward, launches one per model stage)
    adam_ends = [e for i, (s, e) in enumerate(adam) if i + 1 == len(adam) or adam[i + 1][0] - e > 5_000_000]
    if len(adam_ends) < nsteps + 1:
        print("not enough steps")
        return
    t0, t1 = adam_ends[-nsteps - 1], adam_ends[-1]
    win = [(max(s, t0), min(e, t1), n) for s, e, n in ks if e > t0 and s < t1]
    span = t1 - t0
    busy = union([(s, e) for s, e, _ in win])
    nomask = union([(s, e) for s, e, n in win if classify(n) != "attn_mask"])
    mask = [(s, e) for s, e, n in win if classify(n) == "attn_mask"]
    mask_t = sum(e - s for s, e in mask)
    per = defaultdict(float)
    for s, e, n in win:
        per[classify(n)] += e - s
    ms = lambda x: round(x / 1e6 / nsteps, 3)
    print(f"per step: wall {ms(span)} ms, busy(all) {ms(busy)} ms, busy(without mask kernels) {ms(nomask)} ms, "
          f"idle {ms(span - busy)} ms")
    print(f"mask kernels {ms(mask_t)} ms/step; exposed (busy - busy_without_mask) {ms(busy - nomask)} ms/step")
    noadam = union([(s, e) for s, e, n in win if classify(n) != "adam"])
    print(f"adam kernels {ms(per_sum(win, 'adam'))} ms/step; exposed (busy - busy_without_adam) "
          f"{ms(busy - noadam)} ms/step")
    for k, v in sorted(per.items(), key=lambda x: -x[1]):
        print(f"  {k:12s} {ms(v):8.3f} ms/step")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3)
