#!/usr/bin/env python
"""EXPERIMENT record (round 5): needs scripts/experiments/proj_fragB_r5.hip built into the library
and its ops/gemm.py wrappers (proj_pack / proj_nt, removed with the kernel); results in
profiles/r5_s37_proj_fragB.jsonl.

Projection products of a BERT-base layer at bench.py's token count: hipBLASLt (TunableOp table,
the production path: F.linear, NT input gradients against W^T) vs ops/csrc/proj.hip (B packed in
fragment order).  Interleaved rounds; per product the median us, TF/s and each path's error
against an fp32 reference.

    T=131072 ROUNDS=5 python scripts/bench_proj.py
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
    d = "cuda"
    x = torch.randn(T, H, device=d, dtype=bf)
    xf = torch.randn(T, F, device=d, dtype=bf)
    dy3 = torch.randn(T, 3 * H, device=d, dtype=bf)
    wqkv = torch.randn(3 * H, H, device=d, dtype=bf) * 0.03
    wo = torch.randn(H, H, device=d, dtype=bf) * 0.03
    w1 = torch.randn(F, H, device=d, dtype=bf) * 0.03
    w2 = torch.randn(H, F, device=d, dtype=bf) * 0.03
    b3 = torch.randn(3 * H, device=d, dtype=bf)
    bh = torch.randn(H, device=d, dtype=bf)
    # (name, A, W, trans, bias, add)  -- C = A . B^T, B = W (forward) or W^T (input gradient)
    cases = [("fwd_qkv", x, wqkv, False, b3, False), ("fwd_o", x, wo, False, bh, False),
             ("fwd_fc2", xf, w2, False, bh, False), ("dgrad_qkv_add", dy3, wqkv, True, None, True),
             ("dgrad_o", x, wo, True, None, False), ("dgrad_fc1", xf, w1, True, None, False)]
    tot = {"hipblaslt": 0.0, "proj": 0.0, "pack": 0.0}
    for name, a, w, trans, bias, add in cases:
        wt = w.t().contiguous() if trans else w
        N = wt.shape[0]
        bp = G.proj_pack(w, trans)
        c0 = torch.randn(T, N, device=d, dtype=bf) if add else None
        c = torch.empty(T, N, device=d, dtype=bf)
        ref = a.float() @ wt.float().t()
        if bias is not None:
            ref += bias.float()
        if add:
            ref += c0.float()

        def lib():
            if add:
                c.copy_(c0)
                c.addmm_(a, wt.t())
            else:
                c.copy_(torch.nn.functional.linear(a, wt, bias))

        def lib_t():   # timing form: the product only (addmm in place / linear into a fresh tensor)
            if add:
                c.addmm_(a, wt.t())
            else:
                torch.nn.functional.linear(a, wt, bias)

        def pj():
            if add:
                c.copy_(c0)
            G.proj_nt(a, bp, N, bias, out=c, add=add)

        def pj_t():
            G.proj_nt(a, bp, N, bias, out=c, add=add)

        err = {}
        for k, f in (("hipblaslt", lib), ("proj", pj)):
            f()
            torch.cuda.synchronize()
            err[k] = round(rel(c, ref), 6)
        del ref
        times = {"hipblaslt": [], "proj": [], "pack": []}
        for _ in range(rounds):
            times["hipblaslt"].append(timed(lib_t, 10))
            times["proj"].append(timed(pj_t, 10))
            times["pack"].append(timed(lambda: G.proj_pack(w, trans), 10))
        fl = 2 * T * N * a.shape[1]
        row = {"shape": [T, N, a.shape[1]], "err_vs_fp32": err}
        for k, ts in times.items():
            med = statistics.median(ts)
            row[k] = {"us": round(med, 1), "TF": round(fl / med / 1e6, 1)}
            tot[k] += med
        row["speedup"] = round(row["hipblaslt"]["us"] / row["proj"]["us"], 3)
        print(json.dumps({name: row}), flush=True)
    print(json.dumps({"T": T, "rounds": rounds, "layer_total_us": {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
