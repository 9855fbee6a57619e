#!/usr/bin/env python
"""Hand-written MFMA GEMM + fused FFN epilogues vs hipBLASLt + elementwise kernels at the
BERT-base b128 FFN shapes (T = 65536 tokens, h = 768, ffn = 3072)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_and_deepspeed_amd.ops import functional as Fx  # noqa: E402
from distributed_training_and_deepspeed_amd.ops import gemm as G  # noqa: E402


def t_us(fn, reps=20):
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
    if "--tuned" in sys.argv:
        from distributed_training_and_deepspeed_amd.utils.tuning import use_tuned_gemms
        use_tuned_gemms()
    T, H, F = int(os.environ.get("T", 65536)), 768, 3072
    bf = torch.bfloat16
    x = torch.randn(T, H, device="cuda", dtype=bf)
    w1 = (torch.randn(F, H, device="cuda") * 0.05).to(bf)
    b1 = torch.randn(F, device="cuda", dtype=bf)
    w2 = (torch.randn(H, F, device="cuda") * 0.05).to(bf)
    w2t = w2.t().contiguous()
    dy = torch.randn(T, H, device="cuda", dtype=bf)
    u = torch.randn(T, F, device="cuda", dtype=bf)
    db = torch.zeros(F, device="cuda", dtype=torch.float32)
    fl = 2.0 * T * H * F
    r = {}
    r["hipblaslt_fc1"] = t_us(lambda: torch.nn.functional.linear(x, w1, b1))
    r["mine_fc1"] = t_us(lambda: G.gemm_bt(x, w1, b1))
    r["unfused_fc1_gelu"] = t_us(lambda: Fx.act_fwd(torch.nn.functional.linear(x, w1, b1), "gelu"))
    r["fused_fc1_gelu"] = t_us(lambda: G.linear_gelu(x, w1, b1))
    r["hipblaslt_dgrad"] = t_us(lambda: dy @ w2)
    r["unfused_dgrad_gelu_bwd"] = t_us(lambda: Fx.act_bwd(dy @ w2, u, "gelu", dbias=(db, False)))
    r["fused_dgrad_gelu_bwd"] = t_us(lambda: G.gelu_bwd_gemm(dy, w2t, u, dbias=(db, False)))
    out = {k: round(v, 1) for k, v in r.items()}
    out["mine_fc1_TF"] = round(fl / r["mine_fc1"] / 1e6, 1)
    out["hipblaslt_fc1_TF"] = round(fl / r["hipblaslt_fc1"] / 1e6, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
