#!/usr/bin/env python
"""Run-to-run determinism of the fused BERT-base training step (tests/test_model_gpu.py
test_staged_adam_overlapped_with_forward_is_bit_identical's setup: B 2 x S 128, 4 steps, DDP at
world 1, hf AdamW).  The same training runs REPEAT times in this process; per step it records a
checksum of the loss, the flat gradient buffer and the fp32 master weights, and prints the first
step / quantity where two runs differ.  Environment switches select the variant (DTD_GEMM=0,
DTD_KERNELS_SO=..., OVERLAP=1 for the staged optimizer)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_training_and_deepspeed_amd.data import SyntheticLMDataset  # noqa: E402
from distributed_training_and_deepspeed_amd.models import build_model  # noqa: E402
from distributed_training_and_deepspeed_amd.optim import hf_adamw  # noqa: E402
from distributed_training_and_deepspeed_amd.parallel import DistributedDataParallel  # noqa: E402


def chk(t):
    v = t.detach().float().view(-1)
    w = torch.arange(1, v.numel() + 1, device=v.device, dtype=torch.float64) % 9973
    return float((v.double() * w).sum().item())


def run(overlap, steps, B, S):
    model = build_model("base", dtype=torch.bfloat16, device="cuda:0", seed=0)
    ddp = DistributedDataParallel(model)
    opt = hf_adamw(ddp.parameters(), lr=1e-3)
    if overlap:
        opt.overlap_with_forward(model.zero3_units(), root=model)
    ds = SyntheticLMDataset(model.cfg, steps * B, seq_len=S, seed=0)
    ids, lab = ds.input_ids.view(steps, B, S).cuda(), ds.labels.view(steps, B, S).cuda()
    rec = []
    for i in range(steps):
        out = ddp(ids[i], labels=lab[i])
        out.loss.backward()
        torch.cuda.synchronize()
        g = chk(ddp.grads.buf)
        opt.step()
        model.rt.rng.advance()
        if overlap:
            opt.synchronize()
        torch.cuda.synchronize()
        rec.append({"loss": float(out.loss.detach().float()), "grad": g, "master": chk(opt.master)})
    return rec


def main():
    reps = int(os.environ.get("REPEAT", 3))
    steps = int(os.environ.get("STEPS", 4))
    B, S = int(os.environ.get("B", 2)), int(os.environ.get("S", 128))
    overlap = os.environ.get("OVERLAP", "0") == "1"
    runs = [run(overlap, steps, B, S) for _ in range(reps)]
    first = None
    for r in range(1, reps):
        for i in range(steps):
            for k in ("loss", "grad", "master"):
                if runs[r][i][k] != runs[0][i][k] and first is None:
                    first = {"run": r, "step": i, "what": k}
    print(json.dumps({"variant": os.environ.get("VARIANT", "base"), "overlap": overlap, "reps": reps,
                      "deterministic": first is None, "first_diff": first,
                      "grad_chk": [[x["grad"] for x in rr] for rr in runs]}), flush=True)


if __name__ == "__main__":
    main()
