#!/usr/bin/env python
"""hipBLASLt bf16 GEMM throughput on MI355X: large square shapes (practical peak) vs the
BERT-base b128 training shapes (T = 65536 tokens), with the framework's tuned table loaded."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def t_ms(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    from distributed_training_and_deepspeed_amd.utils.tuning import use_tuned_gemms
    tuned = use_tuned_gemms() if "--tuned" in sys.argv else False
    bf = torch.bfloat16
    for n in (4096, 8192, 16384):
        a = torch.randn(n, n, device="cuda", dtype=bf)
        b = torch.randn(n, n, device="cuda", dtype=bf)
        ms = t_ms(lambda: a @ b, reps=10)
        print(json.dumps({"shape": f"{n}^3", "ms": round(ms, 3), "TF": round(2 * n ** 3 / ms / 1e9, 1)}), flush=True)
    T = 65536
    for (o, i) in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
        x = torch.randn(T, i, device="cuda", dtype=bf)
        w = torch.randn(o, i, device="cuda", dtype=bf)
        bias = torch.randn(o, device="cuda", dtype=bf)
        dy = torch.randn(T, o, device="cuda", dtype=bf)
        g = torch.empty(o, i, device="cuda", dtype=bf)
        fl = 2.0 * T * o * i
        r = {"T": T, "out": o, "in": i, "tuned": tuned}
        for k, f in (("fwd", lambda: torch.nn.functional.linear(x, w, bias)), ("dgrad", lambda: dy @ w),
                     ("wgrad", lambda: torch.mm(dy.t(), x, out=g))):
            ms = t_ms(f)
            r[k + "_us"] = round(ms * 1e3, 1)
            r[k + "_TF"] = round(fl / ms / 1e9, 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
