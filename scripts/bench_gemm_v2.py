#!/usr/bin/env python
"""A GEMM kernel form (DTD_GEMM_VARIANT = VNEW, default 4) vs the production persistent form v1 vs
hipBLASLt, C = A B^T (+ bias), bf16, at the BERT-base b256 plain projection shapes.  The round-3
experimental forms live in scripts/experiments/gemm_variants_r3.hip (paste into gemm.hip to rerun).

1. correctness: v2 against an fp32 reference on several shapes (1 tile per workgroup, several,
   uneven XCD groups, with / without bias);
2. timing: interleaved rounds in one process (cdna_hip_programming.md 5.4 rule 24), median us.
Prints one JSON line per shape and a summary line."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_and_deepspeed_amd.ops import _lib  # noqa: E402
from distributed_training_and_deepspeed_amd.ops import gemm as G  # noqa: E402


VNEW = int(os.environ.get("VNEW", "4"))   # the variant compared against v1 (the "v2" columns)


def setv(v):
    return _lib.lib().dtd_gemm_set_variant(v)


def run(a, b, c, bias, v):
    setv(v)
    G._call(G.EPI_STORE, a, b, c, bias=bias)


def check():
    torch.manual_seed(0)
    bad = 0
    for (M, N, K) in [(256, 256, 128), (2048, 768, 768), (4096, 2304, 768), (1024 * 9, 768, 3072),
                      (256 * 300, 768, 256), (512, 3072, 192)]:
        for with_bias in (False, True):
            a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
            bias = torch.randn(N, device="cuda", dtype=torch.bfloat16) if with_bias else None
            ref = a.float() @ b.float().t()
            if bias is not None:
                ref += bias.float()
            c = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
            run(a, b, c, bias, VNEW)
            torch.cuda.synchronize()
            err = ((c.float() - ref).norm() / ref.norm()).item()
            nan = bool(torch.isnan(c).any())
            ok = err < 1e-2 and not nan
            bad += not ok
            print(json.dumps({"check": [M, N, K], "bias": with_bias, "rel_err": round(err, 6), "nan": nan, "ok": ok}),
                  flush=True)
    return bad


def timed(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    from distributed_training_and_deepspeed_amd.utils.tuning import use_tuned_gemms
    use_tuned_gemms()
    bad = check()
    T = int(os.environ.get("T", 131072))
    rounds = int(os.environ.get("ROUNDS", 5))
    shapes = {"fwd_qkv": (2304, 768, True), "fwd_o": (768, 768, True), "fwd_fc2": (768, 3072, True),
              "dgrad_qkv": (768, 2304, False), "dgrad_o": (768, 768, False), "dgrad_fc1": (768, 3072, False),
              "fwd_fc1_plain": (3072, 768, True), "dgrad_fc2_plain": (3072, 768, False)}
    res = {}
    for name, (N, K, with_bias) in shapes.items():
        a = torch.rand(T, K, device="cuda", dtype=torch.bfloat16) * 2 - 1
        b = torch.rand(N, K, device="cuda", dtype=torch.bfloat16) * 2 - 1
        bias = torch.rand(N, device="cuda", dtype=torch.bfloat16) if with_bias else None
        c = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
        fns = {"hipblaslt": (lambda: torch.nn.functional.linear(a, b, bias)),
               "v1": (lambda: run(a, b, c, bias, 1)), "v2": (lambda: run(a, b, c, bias, VNEW))}
        for f in fns.values():
            f()
        torch.cuda.synchronize()
        t = {k: [] for k in fns}
        for _ in range(rounds):
            for k, f in fns.items():
                t[k].append(timed(f, 10))
        med = {k: statistics.median(v) for k, v in t.items()}
        fl = 2.0 * T * N * K
        r = {k + "_us": round(v, 1) for k, v in med.items()}
        r.update({k + "_TF": round(fl / v / 1e6, 1) for k, v in med.items()})
        r["v2_vs_hipblaslt"] = round(med["hipblaslt"] / med["v2"], 3)
        r["v2_vs_v1"] = round(med["v1"] / med["v2"], 3)
        res[name] = r
        print(json.dumps({name: r}), flush=True)
    setv(1)
    print(json.dumps({"T": T, "rounds": rounds, "check_failures": bad, "results": res}))


if __name__ == "__main__":
    main()
