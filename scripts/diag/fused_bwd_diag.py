#!/usr/bin/env python
"""Localise fused-attention-backward errors: for each (S, p) the fused kernel's dq / dk / dv vs the
split kernels, reported per (batch, head, 32-row block) -- which waves / key blocks / query tiles
differ, and by how much.  One JSON line per case."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_training_and_deepspeed_amd.ops import attention as A  # noqa: E402
from distributed_training_and_deepspeed_amd.ops.rng import RngState  # noqa: E402


def main():
    B, H, D = 2, 3, 64
    for S, p in [(128, 0.1), (128, 0.0), (256, 0.1), (384, 0.0), (512, 0.1)]:
        torch.manual_seed(1)
        qkv = torch.randn(B * S, 3 * H * D, device="cuda").to(torch.bfloat16)
        dctx = torch.randn(B * S, H * D, device="cuda").to(torch.bfloat16)
        rg = RngState(5, device="cuda")
        ctx, lse, mk = A.attn_fwd(qkv, B, S, H, D, False, None, p, rg, 3)
        out = {}
        for form in ("split", "fused", "fused2", "fused4"):
            A.set_bwd_form({"split": "split", "fused4": "fused4"}.get(form, "fused"))
            out[form] = A.attn_bwd(dctx, qkv, ctx, lse, B, S, H, D, False, None, p, rg, 3, mk).float()
            torch.cuda.synchronize()
        A.set_bwd_form("split")
        rep = {"S": S, "p": p, "fused_repeatable": bool(torch.equal(out["fused"], out["fused2"])),
               "fused4_vs_split": float((out["fused4"] - out["split"]).abs().max())}
        g = out["fused"].view(B, S // 32, 32, 3, H, D)
        r = out["split"].view(B, S // 32, 32, 3, H, D)
        for i, name in enumerate("qkv"):
            e = (g[:, :, :, i] - r[:, :, :, i]).abs()          # [B, S/32, 32, H, D]
            n = r[:, :, :, i].abs().amax()
            blk = e.amax(dim=(2, 4)) / n                         # [B, S/32, H]
            bad = (blk > 0.05).nonzero().tolist()
            rep[name] = {"max_rel": round(float(e.max() / n), 4), "bad_blocks": bad[:12], "n_bad": len(bad)}
            if name != "q" and bad:
                # which head dims of a bad block
                b0, s0, h0 = bad[0]
                col = e[b0, s0, :, h0].amax(dim=0) / n
                rep[name]["bad_dims_first"] = (col > 0.05).nonzero().flatten().tolist()[:64]
                row = e[b0, s0, :, h0].amax(dim=1) / n
                rep[name]["bad_rows_first"] = (row > 0.05).nonzero().flatten().tolist()
        print(json.dumps(rep), flush=True)


if __name__ == "__main__":
    main()
