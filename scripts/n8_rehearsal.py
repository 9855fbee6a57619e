#!/usr/bin/env python
"""Rehearse the N > 1 DDP step on ONE GPU (not a scaling measurement).

bench.py at world 1 runs no collective: DDP._launch returns at once.  On an 8-GPU node every
gradient bucket is all-reduced by RCCL on a high-priority comm stream while backward continues;
RCCL's kernels hold CUs that the persistent GEMMs and attention kernels would otherwise use.  This
script runs bench.py's exact training step (BERT-base MLM, b256 x 512, bf16, fused kernels,
staged Adam, 64 MiB buckets) and, in place of each bucket's all-reduce, launches at the same point
in backward the stand-in `dtd_spin_occupy` on a high-priority side stream: OCC workgroups (each
holds a CU against the 128 KiB-LDS GEMM workgroups) for the time a ring all-reduce of that bucket
would take at world 8 (2 * 7/8 * bytes / BUSBW + LAT_US).  finish() makes the compute stream wait
for the stand-ins exactly as for RCCL work.  Rows sweep OCC (CUs RCCL occupies) x BUSBW (GB/s).

Output: one JSON line per row with ms/step, the projected per-GPU tokens/s and the projected
8-GPU whole-node tokens/s (8 x per-GPU), plus the exposed communication (step - quiet step).
"""
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_training_and_deepspeed_amd.data import SyntheticLMDataset  # noqa: E402
from distributed_training_and_deepspeed_amd.models import build_model  # noqa: E402
from distributed_training_and_deepspeed_amd.ops import _lib  # noqa: E402
from distributed_training_and_deepspeed_amd.optim import hf_adamw  # noqa: E402
from distributed_training_and_deepspeed_amd.parallel import DistributedDataParallel  # noqa: E402
from distributed_training_and_deepspeed_amd.parallel import ddp as ddp_mod  # noqa: E402
from distributed_training_and_deepspeed_amd.utils.graphs import mlm_capacity  # noqa: E402
from distributed_training_and_deepspeed_amd.utils.tuning import use_tuned_gemms  # noqa: E402


def ring_allreduce_us(nbytes, world, busbw_gbs, lat_us):
    return 2.0 * (world - 1) / world * nbytes / (busbw_gbs * 1e3) + lat_us


def main():
    B, S = int(os.environ.get("B", 256)), 512
    steps, warm = int(os.environ.get("STEPS", 10)), int(os.environ.get("WARM", 4))
    world = 8
    occs = [int(v) for v in os.environ.get("OCC", "0,16,32,64").split(",")]
    busbws = [float(v) for v in os.environ.get("BUSBW", "150,300").split(",")]
    lat = float(os.environ.get("LAT_US", "30"))
    bucket_mb = float(os.environ.get("BUCKET_MB", "64"))
    use_tuned_gemms()
    dev = torch.device("cuda", 0)
    model = build_model("base", dtype=torch.bfloat16, device=dev, seed=1234, sparse_mlm_head=True)
    model.train()
    model.rt.mlm_capacity = -(-mlm_capacity(B * S) // 256) * 256
    model.rt.mlm_overflow = torch.zeros((), dtype=torch.bool, device=dev)
    ddp = DistributedDataParallel(model, bucket_cap_mb=bucket_mb)
    opt = hf_adamw(ddp.parameters(), lr=5e-5)
    opt.overlap_with_forward(model.zero3_units(), root=model)
    ds = SyntheticLMDataset(model.cfg, num_samples=B * 4, seq_len=S, seed=100)
    ids = ds.input_ids.view(-1, B, S).to(dev)
    labels = ds.labels.view(-1, B, S).to(dev)
    side = torch.cuda.Stream(dev, priority=-1)   # high priority, like the RCCL streams (comm.init)
    es = ddp.grads.buf.element_size()
    cfg = {"occ": 0, "busbw": 0.0}
    launched = []

    def fake_launch(self, b):   # the bucket's all-reduce -> CU-holding stand-in of its duration
        if cfg["occ"] <= 0:
            return
        us = ring_allreduce_us((b.end - b.start) * es, world, cfg["busbw"], lat)
        side.wait_stream(torch.cuda.current_stream(dev))
        _lib.call("dtd_spin_occupy", cfg["occ"], us, side.cuda_stream)
        b.work = ddp_mod._StreamWork(side, dev)
        launched.append(us)

    ddp_mod.DistributedDataParallel._launch = fake_launch

    def step(i):
        out = ddp(ids[i % ids.shape[0]], labels=labels[i % labels.shape[0]])
        out.loss.backward()
        opt.step()
        model.rt.rng.advance()

    rows = []
    quiet = None
    for busbw in busbws:
        for occ in occs:
            if occ == 0 and quiet is not None:
                continue
            cfg.update(occ=occ, busbw=busbw)
            for i in range(warm):
                step(i)
            torch.cuda.synchronize()
            launched.clear()
            t0 = time.perf_counter()
            for i in range(steps):
                step(i)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / steps * 1e3
            comm_us = sum(launched) / steps
            if occ == 0:
                quiet = ms
            tok = B * S / (ms / 1e3)
            r = {"occ_cus": occ, "busbw_GBps": busbw if occ else None, "buckets": len(ddp.buckets),
                 "bucket_mb": bucket_mb, "ms_per_step": round(ms, 3),
                 "allreduce_ms_per_step": round(comm_us / 1e3, 3),
                 "exposed_ms": round(ms - quiet, 3) if quiet is not None else None,
                 "proj_tokens_per_s_per_gpu": round(tok, 1), "proj_tokens_per_s_8gpu": round(8 * tok, 1),
                 "note": "one-GPU rehearsal with CU-holding stand-ins for RCCL; NOT a scaling measurement"}
            rows.append(r)
            print(json.dumps(r), flush=True)
    print(json.dumps({"summary": rows}))


if __name__ == "__main__":
    main()
