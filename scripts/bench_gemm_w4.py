#!/usr/bin/env python
"""gemm_w4.hip (one wave per SIMD) vs hipBLASLt (TunableOp table) vs gemm.hip's 8-wave kernel on the
plain BERT-base products of the training step, interleaved rounds in one process.

T tokens (default 524288 = bench.py's b1024 x 512).  Prints one JSON line per product (median us,
TF/s, speed-up over hipBLASLt, relative error against fp32 on a 2048-row slice) and a summary line.
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
    if "--untuned" not in sys.argv:
        from distributed_training_and_deepspeed_amd.utils.tuning import use_tuned_gemms
        use_tuned_gemms()
    T = int(os.environ.get("T", 524288))
    rounds = int(os.environ.get("ROUNDS", 5))
    reps = int(os.environ.get("REPS", 5))
    only = os.environ.get("ONLY")
    H, F = 768, 3072
    bf = torch.bfloat16
    torch.manual_seed(0)
    x = torch.randn(T, H, device="cuda", dtype=bf)
    xf = torch.randn(T, F, device="cuda", dtype=bf)
    dy3 = torch.randn(T, 3 * H, device="cuda", dtype=bf)
    res = torch.randn(T, H, device="cuda", dtype=bf)
    w = {n: (torch.randn(o, i, device="cuda") * 0.03).to(bf)
         for n, (o, i) in {"qkv": (3 * H, H), "o": (H, H), "fc1": (F, H), "fc2": (H, F)}.items()}
    b = {n: torch.randn(t.shape[0], device="cuda", dtype=bf) * 0.1 for n, t in w.items()}
    wt = {n: t.t().contiguous() for n, t in w.items()}
    L = torch.nn.functional.linear
    # name: (flops, A, B, bias, add-target)
    cases = {
        "fwd_qkv": (x, w["qkv"], b["qkv"], None),
        "fwd_o": (x, w["o"], b["o"], None),
        "fwd_fc2": (xf, w["fc2"], b["fc2"], None),
        "fwd_fc1_plain": (x, w["fc1"], b["fc1"], None),
        "dgrad_qkv_add": (dy3, wt["qkv"], None, res),
        "dgrad_o": (x, wt["o"], None, None),
        "dgrad_fc1": (xf, wt["fc1"], None, None),
    }
    if only:
        cases = {k: v for k, v in cases.items() if k in only.split(",")}
    # SCHEDS="0,1,2": time gemm_w4.hip's K-step schedule variants (dtd_gemm_w4_set_sched) as extra columns
    scheds = [int(x) for x in os.environ.get("SCHEDS", "").split(",") if x]
    lib = __import__("distributed_training_and_deepspeed_amd.ops._lib", fromlist=["_lib"])

    def sched(i, fn):
        def run():
            lib.call("dtd_gemm_w4_set_sched", i)
            fn()
            lib.call("dtd_gemm_w4_set_sched", 0)
        return run
    fns = {}
    S = 2048
    for k, (a, bb, bias, add) in cases.items():
        fl = 2 * T * a.shape[1] * bb.shape[0]
        if add is None:
            lib_fn = (lambda a=a, bb=bb, bias=bias: L(a, bb, bias))
            w4 = (lambda a=a, bb=bb, bias=bias: G.gemm_w4(a, bb, bias))
            w8 = (lambda a=a, bb=bb, bias=bias: G.gemm_bt(a, bb, bias))
            ref = a[:S].float() @ bb.float().t() + (bias.float() if bias is not None else 0)
            err = {"lib": rel(L(a[:S], bb, bias), ref), "w4": rel(G.gemm_w4(a[:S], bb, bias), ref)}
        else:
            lib_fn = (lambda a=a, bb=bb, add=add: add.addmm_(a, bb.t()))
            w4 = (lambda a=a, bb=bb, add=add: G.gemm_w4(a, bb, out=add))
            w8 = (lambda a=a, bb=bb, add=add: G.matmul_nt_add_(add, a, bb))
            c0 = add[:S].clone()
            ref = c0.float() + a[:S].float() @ bb.float().t()
            c1 = c0.clone()
            G.gemm_w4(a[:S], bb, out=c1)
            err = {"lib": rel(c0.clone().addmm_(a[:S], bb.t()), ref), "w4": rel(c1, ref)}
        row = {"lib": lib_fn, "w4": w4, "w8": w8}
        for i in scheds:
            row[f"w4s{i}"] = sched(i, w4)
        fns[k] = (fl, row, err)
    for _, f, _ in fns.values():
        for fn in f.values():
            fn()
    torch.cuda.synchronize()
    times = {k: {n: [] for n in f} for k, (_, f, _) in fns.items()}
    for r in range(rounds):
        for k, (_, f, _) in fns.items():
            for n, fn in f.items():
                times[k][n].append(timed(fn, reps))
        print(json.dumps({"round": r}), flush=True)
    out = {}
    tot = {n: 0.0 for n in next(iter(fns.values()))[1]}
    for k, (fl, f, err) in fns.items():
        row = {n: round(statistics.median(v), 1) for n, v in times[k].items()}
        for n in row:
            tot[n] += row[n]
        row.update({f"{n}_TF": round(fl / row[n] / 1e6, 1) for n in f})
        row["w4_vs_lib"] = round(row["lib"] / row["w4"], 3)
        row["err"] = {n: round(e, 5) for n, e in err.items()}
        out[k] = row
        print(json.dumps({k: row}), flush=True)
    print(json.dumps({"T": T, "rounds": rounds, "total_us": {n: round(v, 1) for n, v in tot.items()},
                      "w4_vs_lib_total": round(tot["lib"] / tot["w4"], 3), "results": out}), flush=True)


if __name__ == "__main__":
    main()
