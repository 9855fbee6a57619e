#!/usr/bin/env python
"""Split-K factor of the weight-gradient GEMMs at bench.py's b256 (T = 131072 tokens) with
TunableOp-tuned hipBLASLt / rocBLAS solutions for every candidate shape: the existing table is
loaded, new batched shapes are tuned on first use, then every variant (bmm into bf16 partials +
the framework's reduce) is timed with tuning off.  Writes the merged table to gpurun_out/."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_and_deepspeed_amd.ops.grad import splitk_reduce  # noqa: E402
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
    return s.elapsed_time(e) / reps * 1e3


def main():
    import torch.cuda.tunable as tunable
    T = int(os.environ.get("T", 131072))
    splits = [int(v) for v in os.environ.get("SPLITS", "8,16,32,64").split(",")]
    bf = torch.bfloat16
    tunable.enable(True)
    tunable.read_file(str(DEFAULT_TABLE))
    tunable.tuning_enable(True)
    tunable.record_untuned_enable(False)
    tunable.set_max_tuning_duration(int(os.environ.get("TUNE_MS", "300")))
    shapes = tuple(tuple(int(v) for v in sh.split("x")) for sh in
                   os.environ.get("SHAPES", "2304x768,768x768,3072x768,768x3072").split(","))
    data = {}
    for (o, i) in shapes:
        dy = torch.randn(T, o, device="cuda", dtype=bf)
        x = torch.randn(T, i, device="cuda", dtype=bf)
        data[(o, i)] = (dy, x)
        for s in splits:   # tune (first call of each new shape)
            torch.bmm(dy.view(s, T // s, o).transpose(1, 2), x.view(s, T // s, i))
        torch.cuda.synchronize()
        print(json.dumps({"tuned": [o, i]}), flush=True)
    tunable.tuning_enable(False)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/tunableop_results.csv", "w") as f:   # every result, table rows included
        for r in tunable.get_results():
            f.write(",".join(str(v) for v in r) + "\n")
    for (o, i), (dy, x) in data.items():
        g = torch.empty(o, i, device="cuda", dtype=bf)
        row = {"T": T, "o": o, "i": i}
        for s in splits:
            a3, b3 = dy.view(s, T // s, o).transpose(1, 2), x.view(s, T // s, i)
            row[f"sk{s}"] = round(t_us(lambda: splitk_reduce(torch.bmm(a3, b3), g, False)), 1)
        best = min((v, k) for k, v in row.items() if k.startswith("sk"))
        row["best"] = best[1]
        row["best_TF"] = round(2.0 * T * o * i / best[0] / 1e6, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
