#!/usr/bin/env python
"""HBM throughput of the fused elementwise / normalisation kernels at the BERT-base b128 shapes
(T = 65536 tokens): GELU forward, GELU backward (+ bias-gradient partials), LayerNorm fwd/bwd."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_and_deepspeed_amd.ops import functional as Fx  # noqa: E402
from distributed_training_and_deepspeed_amd.ops.rng import RngState  # noqa: E402


def t_us(fn, reps=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    T, h, f = int(os.environ.get("T", 65536)), 768, 3072
    bf = torch.bfloat16
    u = torch.randn(T, f, device="cuda", dtype=bf)
    dy = torch.randn(T, f, device="cuda", dtype=bf)
    db = torch.zeros(f, device="cuda", dtype=torch.float32)
    x = torch.randn(T, h, device="cuda", dtype=bf)
    y = torch.randn(T, h, device="cuda", dtype=bf)
    g = torch.ones(h, device="cuda", dtype=bf)
    b = torch.zeros(h, device="cuda", dtype=bf)
    rng = RngState(3, device="cuda")
    res = {}
    big = torch.empty(T * f * 2, device="cuda", dtype=bf)
    big2 = torch.empty_like(big)
    us = t_us(lambda: big2.copy_(big))
    res["copy_ref"] = (round(us, 1), round(2 * big.numel() * 2 / us / 1e6, 2))   # HBM roofline proxy
    del big, big2
    us = t_us(lambda: Fx.act_fwd(u, "gelu"))
    res["gelu_fwd"] = (round(us, 1), round(2 * u.numel() * 2 / us / 1e6, 2))
    us = t_us(lambda: Fx.act_bwd(dy, u, "gelu", dbias=db))
    res["gelu_bwd"] = (round(us, 1), round(3 * u.numel() * 2 / us / 1e6, 2))
    us = t_us(lambda: Fx.bias_grad(dy, db))
    res["bias_grad"] = (round(us, 1), round(u.numel() * 2 / us / 1e6, 2))
    z, out, m, r = Fx.ln_fwd(y, x, g, b, 1e-12, 0.1, rng, 5)
    us = t_us(lambda: Fx.ln_fwd(y, x, g, b, 1e-12, 0.1, rng, 5))
    res["ln_fwd"] = (round(us, 1), round(4 * x.numel() * 2 / us / 1e6, 2))
    dg = torch.zeros(h, device="cuda", dtype=torch.float32)
    dbb = torch.zeros(h, device="cuda", dtype=torch.float32)
    us = t_us(lambda: Fx.ln_bwd(out, None, z, m, r, g, 0.1, rng, 5, want_dz=True, want_dy=True, dgamma=dg, dbeta=dbb))
    res["ln_bwd"] = (round(us, 1), round(4 * x.numel() * 2 / us / 1e6, 2))
    print(json.dumps({"T": T, "us, TB/s": res}))


if __name__ == "__main__":
    main()
