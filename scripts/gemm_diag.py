#!/usr/bin/env python
"""Main-loop limiter probe for the persistent NT GEMM: time the plain product at two BERT shapes
with the kernel library named by DTD_KERNELS_SO (the diagnostic builds of ops/csrc/gemm.hip with
-DDTD_GEMM_DIAG=1 no main-loop LDS-DMA, 2 no fragment reads, 4 no main-loop barriers, 7 none of
them -- timing only, their outputs are wrong).  One JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_and_deepspeed_amd.ops import gemm as G  # noqa: E402


def main():
    T = 131072
    out = {"so": os.path.basename(os.environ.get("DTD_KERNELS_SO", "default"))}
    for name, (N, K) in {"qkv_N2304_K768": (2304, 768), "fc2_N768_K3072": (768, 3072)}.items():
        a = torch.rand(T, K, device="cuda", dtype=torch.bfloat16) - 0.5
        b = torch.rand(N, K, device="cuda", dtype=torch.bfloat16) - 0.5
        c = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
        for _ in range(3):
            G._call(G.EPI_STORE, a, b, c)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(5):
            e0.record()
            for _ in range(10):
                G._call(G.EPI_STORE, a, b, c)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) / 10 * 1e3)
        us = sorted(ts)[2]
        out[name] = {"us": round(us, 1), "TF": round(2 * T * N * K / us / 1e6, 1)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
