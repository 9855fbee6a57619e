"""LayerNorm kernel timings at the BERT-base b256 shape (131072 x 768 bf16), the four calls of a
post-LN layer, in both storage forms:

  fwd   z = r + dropout(y); out = LN(z)      store_z (z kept) / memory-efficient (z not written)
  bwd   LN2 form (dout)  and LN1 form (dout + dout2), from z / from the output (FO)
        x  DTD_LN_BWD_PREFETCH 0 / 1

Prints one JSON line per case: us per call and effective HBM bandwidth (bytes of the [T, h]
tensors the call reads + writes).  Usage: python scripts/bench_ln.py [--rows N] [--iters K]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_training_and_deepspeed_amd.ops import functional as Fx
from distributed_training_and_deepspeed_amd.ops.rng import RngState


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=131072)
    ap.add_argument("--h", type=int, default=768)
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    dev, dt = "cuda", torch.bfloat16
    R, h = args.rows, args.h
    torch.manual_seed(0)
    rng = RngState(seed=1, device=dev)
    y, r, dout, dout2 = (torch.randn(R, h, device=dev, dtype=dt) for _ in range(4))
    gamma = (1 + 0.1 * torch.randn(h, device=dev)).to(dt)
    beta = (0.1 * torch.randn(h, device=dev)).to(dt)
    tb = R * h * 2
    dg, db, dbias = (torch.zeros(h, device=dev) for _ in range(3))
    for store_z in (True, False):
        us = timeit(lambda: Fx.ln_fwd(y, r, gamma, beta, 1e-12, 0.1, rng, 5, store_z=store_z), args.iters)
        n = 4 if store_z else 3
        print(json.dumps({"case": "fwd", "store_z": store_z, "us": round(us, 1),
                          "tb_s": round(n * tb / us / 1e6, 2)}), flush=True)
    z, o, m, rs = Fx.ln_fwd(y, r, gamma, beta, 1e-12, 0.1, rng, 5, store_z=True)
    for pf in ("0", "1"):
        os.environ["DTD_LN_BWD_PREFETCH"] = pf
        for two in (False, True):
            for fo in (False, True):
                kw = dict(xout=o, beta=beta) if fo else {}
                zz = None if fo else z

                def call():
                    Fx.ln_bwd(dout, None, zz, m, rs, gamma, 0.1, rng, 5, want_dz=True, want_dy=True, dgamma=dg,
                              dbeta=db, dbias=dbias, dout2=dout2 if two else None, **kw)
                us = timeit(call, args.iters)
                n = 5 if two else 4
                print(json.dumps({"case": "bwd", "prefetch": int(pf), "dout2": two, "from_output": fo,
                                  "us": round(us, 1), "tb_s": round(n * tb / us / 1e6, 2)}), flush=True)
    # the plain copy bound on this box: torch's device-to-device copy of one [T, h] tensor
    dst = torch.empty_like(y)
    us = timeit(lambda: dst.copy_(y), args.iters)
    print(json.dumps({"case": "copy", "us": round(us, 1), "tb_s": round(2 * tb / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
