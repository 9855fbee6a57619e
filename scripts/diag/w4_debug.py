#!/usr/bin/env python
"""Diagnosis of gemm_w4.hip on small exact problems: prints, per case, NaN count, max error and the
16x16-block map of wrong outputs (row block x column block), so a layout / pipeline error shows its
pattern.  Integer-valued operands make every product exact in fp32."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from distributed_training_and_deepspeed_amd.ops import gemm as G  # noqa: E402


def case(name, a, b, bias=None):
    c = G.gemm_w4(a, b, bias)
    torch.cuda.synchronize()
    ref = a.float() @ b.float().t() + (bias.float() if bias is not None else 0)
    cf = c.float()
    bad = ~torch.isclose(cf, ref, rtol=1e-2, atol=1e-1)
    M, N = c.shape
    blk = bad.view(M // 16, 16, N // 16, 16).any(3).any(1)
    out = {"case": name, "nan": int(torch.isnan(cf).sum()), "bad": int(bad.sum()), "of": M * N,
           "max_err": float((cf - ref).abs().nan_to_num(1e30).max())}
    if out["bad"]:
        rows = [''.join('X' if v else '.' for v in r) for r in blk[:32, :32].cpu().tolist()]
        out["blockmap"] = rows
        i, j = [int(x) for x in bad.nonzero()[0]]
        out["first_bad"] = [i, j, float(cf[i, j]), float(ref[i, j])]
        nz = bad.nonzero()
        out["bad_row16"] = torch.bincount(nz[:, 0] % 16, minlength=16).tolist()
        out["bad_col32"] = torch.bincount(nz[:, 1] % 32, minlength=32).tolist()
        out["bad_vals_zero"] = int((cf[bad] == 0).sum())
    print(json.dumps(out), flush=True)


def main():
    import os
    print(json.dumps({"dbg": os.environ.get("DTD_W4_DBG", "0")}), flush=True)
    torch.manual_seed(0)
    dev = "cuda"
    ri = lambda *s: torch.randint(-3, 4, s, device=dev).bfloat16()  # noqa: E731
    case("256x256x128", ri(256, 128), ri(256, 128))
    case("256x256x256", ri(256, 256), ri(256, 256))
    eye = torch.eye(256, device=dev).bfloat16()
    case("eye_256", eye, ri(256, 256))
    case("512x512x128", ri(512, 128), ri(512, 128))
    case("256x256x128_bias", ri(256, 128), ri(256, 128), ri(256))
    case("2048x768x768", ri(2048, 768), ri(768, 768))
    case("16384x2304x768_bias", ri(16384, 768), ri(2304, 768), ri(2304))


if __name__ == "__main__":
    main()
