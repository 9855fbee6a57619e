#!/usr/bin/env python
"""Per-K-step cost and per-tile overhead of the hand-written GEMM (ops/csrc/gemm.hip).

Times C = A B^T at M = 131072, N = 768 for K = 768 .. 6144 (one process, interleaved rounds) and
fits t = tiles_per_CU * (overhead + K/64 * t_kstep): the slope is the main loop's rate, the
intercept the per-tile prologue + epilogue.  ``--once K`` runs a single shape (for rocprofv3 PMC
passes).  Env DTD_GEMM_VARIANT selects the kernel form as in the library.
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


def main():
    M, N = int(os.environ.get("M", 131072)), int(os.environ.get("N", 768))
    Ks = [768, 1536, 3072, 6144]
    if "--once" in sys.argv:
        Ks = [int(sys.argv[sys.argv.index("--once") + 1])]
    torch.manual_seed(0)
    a = {K: torch.rand(M, K, device="cuda", dtype=torch.bfloat16) * 2 - 1 for K in Ks}
    b = {K: torch.rand(N, K, device="cuda", dtype=torch.bfloat16) * 2 - 1 for K in Ks}
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    run = {K: (lambda K=K: G._call(G.EPI_STORE, a[K], b[K], c)) for K in Ks}
    hip = {K: (lambda K=K: torch.matmul(a[K], b[K].t())) for K in Ks}
    for K in Ks:
        run[K](), hip[K]()
    torch.cuda.synchronize()
    if "--once" in sys.argv:
        for _ in range(20):
            run[Ks[0]]()
        torch.cuda.synchronize()
        return
    t = {K: ([], []) for K in Ks}
    for _ in range(5):
        for K in Ks:
            t[K][0].append(timed(run[K], 10))
            t[K][1].append(timed(hip[K], 10))
    tiles = (M // 256) * (N // 256) / 256.0   # tiles per CU
    xs = [K / 64 for K in Ks]
    ys = [statistics.median(t[K][0]) / tiles for K in Ks]
    n = len(xs)
    mx, my = sum(xs) / n, sum(ys) / n
    slope = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
    icpt = my - slope * mx
    out = {"M": M, "N": N, "variant": os.environ.get("DTD_GEMM_VARIANT", "1"),
           "rows": {K: {"ours_us": round(statistics.median(t[K][0]), 1), "hipblaslt_us": round(statistics.median(t[K][1]), 1),
                        "ours_TF": round(2 * M * N * K / statistics.median(t[K][0]) / 1e6, 1),
                        "hipblaslt_TF": round(2 * M * N * K / statistics.median(t[K][1]) / 1e6, 1)} for K in Ks},
           "us_per_kstep_per_tile": round(slope, 3), "us_overhead_per_tile": round(icpt, 3),
           "mainloop_TF": round(256 * 256 * 64 * 2 / slope / 1e6 * 256, 1)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
