#!/usr/bin/env python
"""PMC probe: the persistent NT GEMM (ops/csrc/gemm.hip) vs hipBLASLt on the same products, for
rocprofv3 --pmc passes (scripts/sessions/gpu_session_r3_gemm_pmc.sh).  Shapes (T = 131072): fc2
forward (N 768, K 3072: long main loop) and qkv forward (N 2304, K 768: short).  Three launches each;
`summarize` folds a counter CSV into per-kernel-family means (ours vs hipBLASLt)."""
import csv
import json
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run():
    from distributed_training_and_deepspeed_amd.ops import gemm as G
    from distributed_training_and_deepspeed_amd.utils.tuning import use_tuned_gemms
    use_tuned_gemms()
    T = 131072
    for N, K in ((768, 3072), (2304, 768)):
        a = torch.rand(T, K, device="cuda", dtype=torch.bfloat16) * 2 - 1
        b = torch.rand(N, K, device="cuda", dtype=torch.bfloat16) * 2 - 1
        c = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
        for _ in range(3):
            G._call(G.EPI_STORE, a, b, c)
            torch.nn.functional.linear(a, b)
    torch.cuda.synchronize()
    print("ok", flush=True)


def run_wgrad():
    """fc1 weight gradient (dW [3072, 768] = dU^T X over T = 131072 tokens): the TN kernel's fp32
    split-K partials (ops/csrc/wgrad.hip) vs hipBLASLt's 16-slice bmm, three launches each."""
    from distributed_training_and_deepspeed_amd.ops import gemm as G
    from distributed_training_and_deepspeed_amd.utils.tuning import use_tuned_gemms
    use_tuned_gemms()
    T, o, i = 131072, 3072, 768
    dy = torch.rand(T, o, device="cuda", dtype=torch.bfloat16) * 2 - 1
    x = torch.rand(T, i, device="cuda", dtype=torch.bfloat16) * 2 - 1
    for _ in range(3):
        G.wgrad_tn(dy, x)
        torch.bmm(dy.view(16, T // 16, o).transpose(1, 2), x.view(16, T // 16, i))
    torch.cuda.synchronize()
    print("ok", flush=True)


def run_w4():
    """gemm_w4.hip (one wave per SIMD) vs hipBLASLt on fc2 forward (N 768, K 3072) and o forward
    (N 768, K 768) at T = 131072, three launches each."""
    from distributed_training_and_deepspeed_amd.ops import gemm as G
    from distributed_training_and_deepspeed_amd.utils.tuning import use_tuned_gemms
    use_tuned_gemms()
    T = 131072
    for N, K in ((768, 3072), (768, 768)):
        a = torch.rand(T, K, device="cuda", dtype=torch.bfloat16) * 2 - 1
        b = torch.rand(N, K, device="cuda", dtype=torch.bfloat16) * 2 - 1
        bias = torch.rand(N, device="cuda", dtype=torch.bfloat16)
        for _ in range(3):
            G.gemm_w4(a, b, bias)
            torch.nn.functional.linear(a, b, bias)
    torch.cuda.synchronize()
    print("ok", flush=True)


def summarize(paths):
    acc = defaultdict(lambda: defaultdict(list))
    for path in paths:
        for r in csv.DictReader(open(path)):
            name = r.get("Kernel_Name", "")
            fam = ("ours" if ("gemm_bt" in name or "gemm_tn" in name or "wgrad_tn" in name or "gemm_w4" in name)
                   else ("hipblaslt" if "Cijk" in name else None))
            if fam is None:
                continue
            grid = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
            key = f"{fam}:{r.get('Kernel_Name')[:60]}:grid{grid}"
            acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in acc.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "summarize":
        summarize(sys.argv[2:])
    elif len(sys.argv) > 1 and sys.argv[1] == "wgrad":
        run_wgrad()
    elif len(sys.argv) > 1 and sys.argv[1] == "w4":
        run_w4()
    else:
        run()
