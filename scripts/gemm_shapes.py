#!/usr/bin/env python
"""Every GEMM of one BERT-base training step (b = DTD_BENCH_BATCH, seq 512): op, shapes, strides,
GPU time -- torch.profiler with record_shapes, grouped by (op, shapes).  Shows which products
run on hipBLASLt and at what rate."""
import json
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_and_deepspeed_amd.data import SyntheticLMDataset  # noqa: E402
from distributed_training_and_deepspeed_amd.models import build_model  # noqa: E402
from distributed_training_and_deepspeed_amd.optim import hf_adamw  # noqa: E402
from distributed_training_and_deepspeed_amd.parallel import DistributedDataParallel  # noqa: E402
from distributed_training_and_deepspeed_amd.utils.tuning import use_tuned_gemms  # noqa: E402


def main():
    use_tuned_gemms()
    B = int(os.environ.get("DTD_BENCH_BATCH", 256))
    model = build_model("base", dtype=torch.bfloat16, device="cuda", seed=0)
    model.train()
    ddp = DistributedDataParallel(model, bucket_cap_mb=64)
    opt = hf_adamw(ddp.parameters())
    ds = SyntheticLMDataset(model.cfg, B, seq_len=512, seed=0)
    ids, lab = ds.input_ids.cuda(), ds.labels.cuda()

    def step():
        out = ddp(ids, labels=lab)
        out.loss.backward()
        opt.step()
        model.rt.rng.advance()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    agg = defaultdict(lambda: [0, 0.0])
    for e in prof.key_averages(group_by_input_shape=True):
        if e.key in ("aten::mm", "aten::addmm", "aten::bmm", "aten::linear", "aten::matmul", "aten::baddbmm"):
            dev_us = getattr(e, "device_time_total", getattr(e, "cuda_time_total", 0.0))
            agg[(e.key, str(e.input_shapes))][0] += e.count
            agg[(e.key, str(e.input_shapes))][1] += dev_us
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    for (k, shp), (n, us) in rows:
        print(json.dumps({"op": k, "shapes": shp, "count": n, "device_us": round(us, 1)}), flush=True)


if __name__ == "__main__":
    main()
