#!/usr/bin/env python
"""Start stagger of the persistent 8-phase GEMM (ops/csrc/gemm.hip, DTD_GEMM_STAGGER_US): the odd
members of each XCD group start `us` later, so the CUs' epilogue store bursts stop coinciding.
Times hipBLASLt (F.linear) and the hand kernel at several staggers in interleaved rounds in one
process (cdna_hip_programming.md §5.4 rule 24), at the BERT-base projection shapes (T = 131072
tokens), and checks the staggered output against the unstaggered one (must be bitwise equal)."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_and_deepspeed_amd.ops import _lib  # noqa: E402
from distributed_training_and_deepspeed_amd.ops import gemm as G  # noqa: E402


def timed(fn, reps=5):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    T = int(os.environ.get("T", 131072))
    staggers = [float(v) for v in os.environ.get("STAGGERS", "0,2,4,8").split(",")]
    H, F = 768, 3072
    bf = torch.bfloat16
    torch.manual_seed(0)
    x = torch.randn(T, H, device="cuda", dtype=bf)
    xf = torch.randn(T, F, device="cuda", dtype=bf)
    w = {n: (torch.randn(o, i, device="cuda") * 0.03).to(bf)
         for n, (o, i) in {"qkv": (3 * H, H), "o": (H, H), "fc1": (F, H), "fc2": (H, F)}.items()}
    cases = {"qkv": (x, w["qkv"]), "o": (x, w["o"]), "fc1": (x, w["fc1"]), "fc2": (xf, w["fc2"])}
    lib = _lib.lib()
    res = {k: {"hipblaslt": []} | {f"s{s}": [] for s in staggers} for k in cases}
    ok = {}
    for k, (a, b) in cases.items():
        lib.dtd_gemm_set_stagger(0.0)
        ref = G.gemm_bt(a, b)
        for s in staggers:
            lib.dtd_gemm_set_stagger(s)
            ok[f"{k}_s{s}"] = bool(torch.equal(G.gemm_bt(a, b), ref))
    for _ in range(int(os.environ.get("ROUNDS", 5))):
        for k, (a, b) in cases.items():
            res[k]["hipblaslt"].append(timed(lambda: torch.nn.functional.linear(a, b)))
            for s in staggers:
                lib.dtd_gemm_set_stagger(s)
                res[k][f"s{s}"].append(timed(lambda: G.gemm_bt(a, b)))
    lib.dtd_gemm_set_stagger(0.0)
    out = {}
    for k, (a, b) in cases.items():
        fl = 2 * a.shape[0] * a.shape[1] * b.shape[0]
        out[k] = {v: {"us": round(statistics.median(ts), 1), "TF": round(fl / statistics.median(ts) / 1e6, 1)}
                  for v, ts in res[k].items()}
        print(json.dumps({k: out[k]}), flush=True)
    print(json.dumps({"T": T, "bitwise_equal": ok, "results": out}), flush=True)


if __name__ == "__main__":
    main()
