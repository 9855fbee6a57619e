#!/usr/bin/env python
"""ZeRO parameter refresh vs the next forward, from a rocprofv3 --kernel-trace CSV of
`bench.py --zero-stage 2` (or zero_dp_training.py): after each step's fused-Adam kernel the
engine all-gathers (world 1: copies) the updated shards on its comm stream, one event per
`allgather_bucket_size` group, and each layer's forward pre-hook waits only for its own buckets.
For every step: the refresh kernels (RCCL all-gather / copy kernels issued after the Adam kernel
and before the next Adam) and how much of their time overlaps compute kernels of other streams.
Prints one JSON line."""
import csv
import json
import sys


def is_refresh(n):
    n = n.lower()
    return "copybuffer" in n or "allgather" in n or "all_gather" in n or ("nccl" in n and "gather" in n)


def main(path):
    rows = list(csv.DictReader(open(path)))
    sid = "Stream_Id" if rows and "Stream_Id" in rows[0] else ("Queue_Id" if rows and "Queue_Id" in rows[0] else None)
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get(sid, "?") if sid else "?")
                for r in rows)
    adam = [e for s, e, n, q in ks if "adam_kernel" in n]
    steps = []
    for a0, a1 in zip(adam, adam[1:]):
        win = [k for k in ks if a0 <= k[0] < a1]
        # the refresh precedes the backward; the backward's reduce-scatters (copies at world 1)
        # start after its first kernel (the loss / LayerNorm backward)
        bwd0 = min((k[0] for k in win if "xent_bwd" in k[2] or "ln_bwd" in k[2]), default=a1)
        ref = [k for k in win if is_refresh(k[2]) and k[0] < bwd0]
        comp = [k for k in win if not is_refresh(k[2]) and k[0] < bwd0]
        if not ref:
            continue
        tot = sum(e - s for s, e, _, _ in ref)
        ov = 0
        for s, e, _, q in ref:
            for cs, ce, _, cq in comp:
                if cq != q and cs < e and s < ce:
                    ov += min(e, ce) - max(s, cs)
        first_comp = min((k[0] for k in comp if k[0] > ref[0][0]), default=None)
        steps.append({"refresh_kernels": len(ref), "refresh_us": round(tot / 1e3, 1),
                      "overlapped_us": round(min(ov, tot) / 1e3, 1),
                      "forward_started_before_refresh_end": first_comp is not None and first_comp < max(e for _, e, _, _ in ref)})
    print(json.dumps({"stream_column": sid, "steps": steps}))


if __name__ == "__main__":
    main(sys.argv[1])
