#!/usr/bin/env python
"""Four-wave GEMM (ops/csrc/gemm4.hip) vs the eight-wave kernel (gemm.hip) vs hipBLASLt on the
plain BERT-base b256 projections (T = 131072 tokens): forward x W^T + b and the NT input gradients
dy (W^T)^T.  Correctness first (fp32 reference on a 1024-row slice and on the full output's first
and last tiles), then interleaved timing rounds in one process (cdna_hip_programming.md §5.4 rule 24).
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_and_deepspeed_amd.ops import gemm as G  # noqa: E402


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
    H, F = 768, 3072
    bf = torch.bfloat16
    torch.manual_seed(0)
    x = torch.randn(T, H, device="cuda", dtype=bf)
    xf = torch.randn(T, F, device="cuda", dtype=bf)
    dy3 = torch.randn(T, 3 * H, device="cuda", dtype=bf)
    w = {n: (torch.randn(o, i, device="cuda") * 0.03).to(bf)
         for n, (o, i) in {"qkv": (3 * H, H), "o": (H, H), "fc1": (F, H), "fc2": (H, F)}.items()}
    b = {n: torch.randn(t.shape[0], device="cuda", dtype=bf) * 0.1 for n, t in w.items()}
    wt = {n: t.t().contiguous() for n, t in w.items()}
    L = torch.nn.functional.linear
    cases = {
        "fwd_qkv": (x, w["qkv"], b["qkv"]),
        "fwd_o": (x, w["o"], b["o"]),
        "fwd_fc1": (x, w["fc1"], b["fc1"]),
        "fwd_fc2": (xf, w["fc2"], b["fc2"]),
        "dgrad_qkv": (dy3, wt["qkv"], None),
        "dgrad_o": (x, wt["o"], None),
        "dgrad_fc1": (xf, wt["fc1"], None),
        "dgrad_fc2": (x, wt["fc2"], None),
    }
    chk = {}
    for k, (a, bb, bias) in cases.items():
        out = G.gemm4_bt(a, bb, bias)
        torch.cuda.synchronize()
        for name, sl in (("head", slice(0, 1024)), ("tail", slice(T - 1024, T))):
            ref = a[sl].float() @ bb.float().t() + (bias.float() if bias is not None else 0)
            chk[f"{k}_{name}"] = round(rel(out[sl], ref), 6)
        chk[f"{k}_vs_hipblaslt"] = round(rel(out, L(a, bb, bias)), 6)
    print(json.dumps({"check": chk}), flush=True)
    bad = {k: v for k, v in chk.items() if v > 1e-2}
    if bad:
        print(json.dumps({"FAILED": bad}), flush=True)
        sys.exit(1)
    fns = {}
    for k, (a, bb, bias) in cases.items():
        fl = 2 * a.shape[0] * a.shape[1] * bb.shape[0]
        fns[k] = (fl, {"hipblaslt": lambda a=a, bb=bb, bias=bias: L(a, bb, bias),
                       "gemm8": lambda a=a, bb=bb, bias=bias: G.gemm_bt(a, bb, bias),
                       "gemm4": lambda a=a, bb=bb, bias=bias: G.gemm4_bt(a, bb, bias)})
    for _, (_, d) in fns.items():
        for f in d.values():
            f()
    torch.cuda.synchronize()
    times = {k: {n: [] for n in d} for k, (_, d) in fns.items()}
    for _ in range(rounds):
        for k, (_, d) in fns.items():
            for n, f in d.items():
                times[k][n].append(timed(f, 10))
    res = {}
    for k, (fl, d) in fns.items():
        row = {}
        for n in d:
            t = statistics.median(times[k][n])
            row[n + "_us"] = round(t, 1)
            row[n + "_TF"] = round(fl / t / 1e6, 1)
        row["gemm4_vs_hipblaslt"] = round(row["hipblaslt_us"] / row["gemm4_us"], 3)
        res[k] = row
        print(json.dumps({k: row}), flush=True)
    print(json.dumps({"T": T, "rounds": rounds, "results": res}), flush=True)


if __name__ == "__main__":
    main()
