#!/usr/bin/env python
"""Weight-gradient GEMM dW[o,i] = dY^T X at T = 65536 tokens (BERT-base b128): split-K factor
sweep (fp32 / bf16 partials + the framework's reduce kernel) and, with --tune, TunableOp's
exhaustive hipBLASLt/rocBLAS search over the un-split GEMM."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_and_deepspeed_amd.ops.grad import splitk_reduce  # noqa: E402


def t_us(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    T = int(os.environ.get("T", 65536))
    bf = torch.bfloat16
    if "--tune" in sys.argv:
        import torch.cuda.tunable as tunable
        tunable.enable(True)
        tunable.tuning_enable(True)
        tunable.set_filename("gpurun_out/wgrad_tuned%d.csv")
        tunable.set_max_tuning_duration(400)
    for (o, i) in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
        dy = torch.randn(T, o, device="cuda", dtype=bf)
        x = torch.randn(T, i, device="cuda", dtype=bf)
        g = torch.empty(o, i, device="cuda", dtype=bf)
        fl = 2.0 * T * o * i
        row = {"T": T, "o": o, "i": i}
        row["mm"] = round(t_us(lambda: torch.mm(dy.t(), x, out=g)), 1)
        if "--tune" not in sys.argv:
            for s in (2, 4, 8, 16, 32):
                a3, b3 = dy.view(s, T // s, o).transpose(1, 2), x.view(s, T // s, i)
                row[f"sk{s}_f32"] = round(t_us(lambda: splitk_reduce(torch.bmm(a3, b3, out_dtype=torch.float32), g, False)), 1)
                row[f"sk{s}_bf16"] = round(t_us(lambda: splitk_reduce(torch.bmm(a3, b3), g, False)), 1)
        best = min((v, k) for k, v in row.items() if k not in ("T", "o", "i"))
        row["best"] = best[1]
        row["best_TF"] = round(fl / best[0] / 1e6, 1)
        print(json.dumps(row), flush=True)
    if "--tune" in sys.argv:
        tunable.write_file()


if __name__ == "__main__":
    main()
