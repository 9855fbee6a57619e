#!/usr/bin/env python
"""PMC probe: the TN weight-gradient kernel (fc1 shape, T = 131072) and the NT kernel on the
same FLOPs (C[3072 x 768] over K = 131072 is not an NT shape, so NT runs M = 131072, N = 768,
K = 3072 -- the fc2-forward-like product), 3 launches each, for rocprofv3 --pmc passes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_and_deepspeed_amd.ops import gemm as G  # noqa: E402


def main():
    T, O, I = 131072, 3072, 768
    dy = torch.randn(T, O, device="cuda").bfloat16()
    x = torch.randn(T, I, device="cuda").bfloat16()
    w = (torch.randn(I, O, device="cuda") * 0.03).bfloat16()
    for _ in range(3):
        G.wgrad_tn(dy, x)
        G.matmul_nt(dy, w)
    torch.cuda.synchronize()
    print("ok", flush=True)


if __name__ == "__main__":
    main()
