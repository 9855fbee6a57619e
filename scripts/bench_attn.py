#!/usr/bin/env python
"""Time the flash-attention kernels at the BERT-base training shape for several occupancy
variants (DTD_ATTN_OCC="fwd,dkdv,dq" waves/SIMD).  Prints one JSON line per variant.

fwd_us: forward kernel with the dropout keep bits generated ahead (as in the model, where the
mask kernel runs on a side stream under the forward GEMMs); mask_us: the mask generator alone;
bwd_us: dK/dV + dQ, or the one-kernel fused backward for a variant named "fused" (or "fused:<occ>").
Env: B, H, P, CAUSAL=1 (model FLOPs are quoted for the full square).  """
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_and_deepspeed_amd.ops import attention as A  # noqa: E402
from distributed_training_and_deepspeed_amd.ops.rng import RngState  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    B, S, H, D = int(os.environ.get("B", 32)), int(os.environ.get("S", 512)), int(os.environ.get("H", 12)), 64
    p = float(os.environ.get("P", 0.1))
    causal = os.environ.get("CAUSAL", "0") == "1"
    qkv = torch.randn(B * S, 3 * H * D, device="cuda").to(torch.bfloat16)
    dctx = torch.randn(B * S, H * D, device="cuda").to(torch.bfloat16)
    rng = RngState(1, device="cuda")
    flops_f = 4 * B * H * S * S * D
    # clock / cache warm-up: the first timed configuration otherwise reads ~20 % slow
    for _ in range(50):
        A.attn_fwd(qkv, B, S, H, D, causal, None, p, rng, 3)
    torch.cuda.synchronize()
    for occ in sys.argv[1:] or ["1,1,1", "2,2,2", "3,2,2", "3,2,3"]:
        form = occ.split(":", 1)[0] if occ.startswith("fused") else "split"
        A.set_bwd_form(form)
        occ = occ.split(":", 1)[1] if ":" in occ else ("3,2,3" if form != "split" else occ)
        os.environ["DTD_ATTN_OCC"] = occ
        pend = A.attn_masks_async(B, S, H, D, p, rng, 3, qkv.device) if p > 0 else None
        torch.cuda.synchronize()
        ctx, lse, mk = A.attn_fwd(qkv, B, S, H, D, causal, None, p, rng, 3, masks=pend)
        tf = timeit(lambda: A.attn_fwd(qkv, B, S, H, D, causal, None, p, rng, 3, masks=pend))
        cur = torch.cuda.current_stream()
        tm = timeit(lambda: cur.wait_event(A.attn_masks_async(B, S, H, D, p, rng, 3, qkv.device).event)) \
            if p > 0 else 0.0
        tb = timeit(lambda: A.attn_bwd(dctx, qkv, ctx, lse, B, S, H, D, causal, None, p, rng, 3, mk))
        print(json.dumps({"occ": occ, "bwd_form": form, "B": B, "S": S, "H": H, "causal": causal, "p": p, "fwd_us": round(tf, 1), "mask_us": round(tm, 1),
                          "bwd_us": round(tb, 1), "fwd_TFs": round(flops_f / tf / 1e6, 1),
                          "bwd_TFs": round(2.5 * flops_f / tb / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
