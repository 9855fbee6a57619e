#!/usr/bin/env python
"""Attention-dropout keep-bit generator (attention.hip) at the bench shape (b256 x 12 heads x
S 512): microseconds per call and a checksum of both mask layouts.  DTD_KERNELS_SO=<library>
times another build of the generator (e.g. ops/_dtd_kernels_oldmask.so, the round-4 form)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_and_deepspeed_amd.ops import _lib  # noqa: E402
from distributed_training_and_deepspeed_amd.ops import attention as A  # noqa: E402
from distributed_training_and_deepspeed_amd.ops.rng import RngState  # noqa: E402


def main():
    B, H, S, p = int(os.environ.get("B", 256)), 12, int(os.environ.get("S", 512)), 0.1
    W = (S + 31) // 32
    rg = RngState(5, device="cuda")
    masks = A.alloc_masks(B, H, S, "cuda")
    st = torch.cuda.current_stream().cuda_stream

    def run():
        _lib.call("dtd_attn_masks", masks.data_ptr(), B, S, H, p, rg.state.data_ptr(), 3, st)

    run()
    torch.cuda.synchronize()
    chk = [int((masks[i].to(torch.int64) * torch.arange(1, masks.shape[1] + 1, device="cuda") % 1000003).sum().item())
           for i in range(2)]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(5):
        e0.record()
        for _ in range(20):
            run()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 20 * 1e3)
    ts.sort()
    dec = B * H * S * S
    print(json.dumps({"variant": os.path.basename(os.environ.get("DTD_KERNELS_SO", "default")),
                      "B": B, "S": S, "us": round(ts[2], 1), "Gdecisions_per_s": round(dec / ts[2] / 1e3, 1),
                      "checksum": chk}), flush=True)


if __name__ == "__main__":
    main()
