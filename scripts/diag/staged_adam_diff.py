#!/usr/bin/env python
"""Which parameters differ between the single-launch AdamW and the staged update overlapped with
the next forward (tests/test_model_gpu.py test_staged_adam_overlapped_with_forward_is_bit_identical's
loop, no extra synchronisation): REPEAT overlapped runs against one single-launch run; per run the
losses, and per parameter (name, stage chunk) the max |difference| of the fp32 master weights."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_training_and_deepspeed_amd.data import SyntheticLMDataset  # noqa: E402
from distributed_training_and_deepspeed_amd.models import build_model  # noqa: E402
from distributed_training_and_deepspeed_amd.optim import hf_adamw  # noqa: E402
from distributed_training_and_deepspeed_amd.parallel import DistributedDataParallel  # noqa: E402


def run(overlap, steps):
    model = build_model("base", dtype=torch.bfloat16, device="cuda:0", seed=0)
    ddp = DistributedDataParallel(model)
    opt = hf_adamw(ddp.parameters(), lr=1e-3)
    if overlap:
        opt.overlap_with_forward(model.zero3_units(), root=model)
    ds = SyntheticLMDataset(model.cfg, 2 * steps, seq_len=128, seed=0)
    ids, lab = ds.input_ids.view(steps, 2, 128).cuda(), ds.labels.view(steps, 2, 128).cuda()
    losses = []
    for i in range(steps):
        out = ddp(ids[i], labels=lab[i])
        out.loss.backward()
        opt.step()
        model.rt.rng.advance()
        losses.append(out.loss.detach().float())
    if overlap:
        opt.synchronize()
    torch.cuda.synchronize()
    base = opt.param_flat
    spans = {}
    for n, p in model.named_parameters():
        if p.untyped_storage().data_ptr() == base.untyped_storage().data_ptr():
            off = p.storage_offset() - base.storage_offset()
            spans[n] = (off, off + p.numel())
    chunks = None
    if overlap:
        chunks = [[list(r) for r in rs] for rs in opt._chunks]
    return torch.stack(losses).cpu(), opt.master.detach().clone(), spans, chunks


def main():
    steps = int(os.environ.get("STEPS", 4))
    reps = int(os.environ.get("REPEAT", 3))
    l0, m0, spans, _ = run(False, steps)
    res = []
    for r in range(reps):
        l1, m1, _, chunks = run(True, steps)
        d = (m1 - m0).abs()
        bad = []
        for n, (a, b) in spans.items():
            mx = d[a:b].max().item()
            if mx > 0:
                bad.append([n, a, b, mx, int((d[a:b] > 0).sum().item())])
        res.append({"rep": r, "losses_equal": bool(torch.equal(l0, l1)), "n_diff_elems": int((d > 0).sum().item()),
                    "params_differing": bad[:40], "n_params_differing": len(bad)})
        if r == 0:
            print(json.dumps({"chunks": chunks, "n": m0.numel()}), flush=True)
        print(json.dumps(res[-1]), flush=True)
    # overlapped runs against each other
    print(json.dumps({"summary": [x["n_diff_elems"] for x in res]}), flush=True)


if __name__ == "__main__":
    main()
