#!/usr/bin/env python
"""TunableOp rows for the NT-form input-gradient GEMMs at bench.py's b256 (T = 131072 tokens):
F.linear(dY, W^T) and the residual-accumulating addmm_ (ops/gemm.py::dgrad / dgrad_add_) for
the qkv, o and fc1 weights.  The repo table is loaded, the shapes it lacks are tuned, and each
product is timed with the tuned solution and with the hipBLASLt heuristic (TunableOp off).
Writes the merged table (validator rows + every result) to gpurun_out/tunableop_dgrad.csv."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_and_deepspeed_amd.utils.tuning import DEFAULT_TABLE  # noqa: E402


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
    return round(s.elapsed_time(e) / reps * 1e3, 1)


def main():
    import torch.cuda.tunable as tunable
    T = int(os.environ.get("T", 131072))
    bf = torch.bfloat16
    tunable.enable(True)
    tunable.read_file(str(DEFAULT_TABLE))
    tunable.tuning_enable(True)
    tunable.record_untuned_enable(False)
    tunable.set_max_tuning_duration(int(os.environ.get("TUNE_MS", "300")))
    data = {}
    for (o, i) in ((2304, 768), (768, 768), (3072, 768)):
        dy = torch.randn(T, o, device="cuda", dtype=bf)
        wt = torch.randn(i, o, device="cuda", dtype=bf)
        c = torch.randn(T, i, device="cuda", dtype=bf)
        F.linear(dy, wt)
        c.addmm_(dy, wt.t())
        torch.cuda.synchronize()
        data[(o, i)] = (dy, wt, c)
        print(json.dumps({"tuned": [o, i]}), flush=True)
    tunable.tuning_enable(False)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/tunableop_dgrad.csv", "w") as f:
        for line in open(DEFAULT_TABLE):
            if line.startswith("Validator"):
                f.write(line)
        for r in tunable.get_results():
            f.write(",".join(str(v) for v in r) + "\n")
    for (o, i), (dy, wt, c) in data.items():
        row = {"T": T, "out": o, "in": i}
        row["linear_tuned_us"] = t_us(lambda: F.linear(dy, wt))
        row["addmm_tuned_us"] = t_us(lambda: c.addmm_(dy, wt.t()))
        tunable.enable(False)
        row["linear_default_us"] = t_us(lambda: F.linear(dy, wt))
        row["addmm_default_us"] = t_us(lambda: c.addmm_(dy, wt.t()))
        tunable.enable(True)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
