#!/usr/bin/env python
"""Fused Adam bandwidth at a max-params-sized partition: the kernel forms of DTD_ADAM_FORM
(1 / 2 groups per thread, non-temporal / cached loads) interleaved, median ms and TB/s at
28 B per element (fp32 p, m, v read + written, bf16 gradient read, bf16 copy written).
Env N (elements, default 2^30)."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_and_deepspeed_amd.optim.fused_adam import FusedAdam  # noqa: E402


def main():
    n = int(os.environ.get("N", 1 << 30))
    master = torch.randn(n, device="cuda") * 0.02
    grad = (torch.randn(n, device="cuda") * 1e-3).bfloat16()
    lowp = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    opt = FusedAdam.from_flat(master, grad, lowp, lr=1e-4)
    forms = sys.argv[1:] or ["1", "2", "1c", "2c"]
    times = {f: [] for f in forms}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for f in forms:
        os.environ["DTD_ADAM_FORM"] = f
        opt.step()
    torch.cuda.synchronize()
    for _ in range(5):
        for f in forms:
            os.environ["DTD_ADAM_FORM"] = f
            e0.record()
            for _ in range(3):
                opt.step()
            e1.record()
            e1.synchronize()
            times[f].append(e0.elapsed_time(e1) / 3)
    for f in forms:
        ms = statistics.median(times[f])
        print(json.dumps({"form": f, "n": n, "ms": round(ms, 3), "TBps": round(28 * n / ms / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
