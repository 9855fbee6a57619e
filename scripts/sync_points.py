#!/usr/bin/env python
"""List host-device synchronisations inside one eager training step of the default bench
configuration (torch.cuda.set_sync_debug_mode), after warm-up."""
import os
import sys
import warnings

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_and_deepspeed_amd.data import SyntheticLMDataset  # noqa: E402
from distributed_training_and_deepspeed_amd.models import build_model  # noqa: E402
from distributed_training_and_deepspeed_amd.optim import hf_adamw  # noqa: E402
from distributed_training_and_deepspeed_amd.parallel import DistributedDataParallel  # noqa: E402
from distributed_training_and_deepspeed_amd.utils.graphs import mlm_capacity  # noqa: E402
from distributed_training_and_deepspeed_amd.utils.tuning import use_tuned_gemms  # noqa: E402


def main():
    use_tuned_gemms()
    B = int(os.environ.get("B", 32))
    model = build_model("base", dtype=torch.bfloat16, device="cuda", seed=0)
    model.train()
    model.rt.mlm_capacity = -(-mlm_capacity(B * 512) // 256) * 256
    model.rt.mlm_overflow = torch.zeros((), dtype=torch.bool, device="cuda")
    ddp = DistributedDataParallel(model, bucket_cap_mb=64)
    opt = hf_adamw(ddp.parameters(), lr=5e-5)
    ds = SyntheticLMDataset(model.cfg, B, seq_len=512, seed=0)
    ids, lab = ds.input_ids.cuda(), ds.labels.cuda()

    def step():
        ddp(ids, labels=lab).loss.backward()
        opt.step()
        model.rt.rng.advance()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("warn")
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        step()
    torch.cuda.set_sync_debug_mode(0)
    print(f"{len(w)} synchronizing calls in one step", flush=True)
    for x in w:
        print(str(x.message)[:300], "|", x.filename, x.lineno, flush=True)


if __name__ == "__main__":
    main()
