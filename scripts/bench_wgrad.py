#!/usr/bin/env python
"""Weight-gradient GEMMs of a BERT-base layer at bench.py's token count: the production library
path (hipBLASLt split-K bmm, TunableOp-tuned, + splitk_reduce) and the ring-pipelined TN kernel
(ops/csrc/wgrad.hip) at each ring depth (profiles/r5_s2_wgrad.jsonl also has the round-2/3
TN kernel, since removed, as "tn_r3").  Interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24); one JSON
line per shape with median us, TF/s and the error of each path against an fp32 reference.

    T=131072 ROUNDS=5 python scripts/bench_wgrad.py
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_and_deepspeed_amd.ops import gemm as G  # noqa: E402
from distributed_training_and_deepspeed_amd.ops import grad as GR  # noqa: E402


def timed(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def main():
    from distributed_training_and_deepspeed_amd.utils.tuning import use_tuned_gemms
    use_tuned_gemms()
    T = int(os.environ.get("T", 131072))
    rounds = int(os.environ.get("ROUNDS", 5))
    variants = [int(v) for v in os.environ.get("VARIANTS", "4,5").split(",")]
    H, F = 768, 3072
    bf = torch.bfloat16
    torch.manual_seed(0)
    x = torch.randn(T, H, device="cuda", dtype=bf)
    xf = torch.randn(T, F, device="cuda", dtype=bf)
    dy3 = torch.randn(T, 3 * H, device="cuda", dtype=bf)
    shapes = {"qkv": (dy3, x), "o": (x, x), "fc1": (xf, x), "fc2": (x, xf)}
    out = {}
    for name, (dy, xx) in shapes.items():
        o, i = dy.shape[1], xx.shape[1]
        dst = torch.empty((o, i), device="cuda", dtype=bf)
        s = GR.wgrad_splits(T, o, i)

        def lib():
            a, b = dy.view(s, T // s, o).transpose(1, 2), xx.view(s, T // s, i)
            GR.splitk_reduce(GR._bmm_partials(a, b, fp32=False), dst, False)

        paths = {"hipblaslt": lib}
        for v in variants:
            if v < 100:
                paths[f"ring{v}"] = lambda v=v: GR.splitk_reduce(G.wgrad_tn(dy, xx, variant=v), dst, False)
            paths[f"ring{v}_kernel"] = lambda v=v: G.wgrad_tn(dy, xx, variant=v)   # >= 100: timing-only diag
        ref = dy.float().t() @ xx.float()
        err = {}
        for k, f in paths.items():
            if k.endswith("_kernel"):
                continue
            dst.zero_()
            f()
            torch.cuda.synchronize()
            err[k] = round(rel(dst, ref), 6)
        del ref
        times = {k: [] for k in paths}
        for f in paths.values():
            f()
        torch.cuda.synchronize()
        for _ in range(rounds):
            for k, f in paths.items():
                times[k].append(timed(f, 10))
        fl = 2 * T * o * i
        row = {"shape": [T, o, i], "lib_splits": s, "ring_splits": int(G._lib.lib().dtd_wgrad_tn_splits(o, i, T)),
               "err_vs_fp32": err}
        for k, ts in times.items():
            med = statistics.median(ts)
            row[k] = {"us": round(med, 1), "min_us": round(min(ts), 1), "TF": round(fl / med / 1e6, 1)}
        out[name] = row
        print(json.dumps({name: row}), flush=True)
    tot = {k: round(sum(out[n][k]["us"] for n in out), 1) for k in out["qkv"] if isinstance(out["qkv"][k], dict)
           and "us" in out["qkv"][k]}
    print(json.dumps({"T": T, "rounds": rounds, "layer_total_us": tot}), flush=True)


if __name__ == "__main__":
    main()
