#!/usr/bin/env python
"""The 8-wave persistent GEMM (ops/csrc/gemm.hip) with its LDS-DMA pieces spread inside the MFMA
blocks (dtd_gemm_set_spread(1), the default) vs bunched ahead of each phase's barrier (0), on the
fused FFN products of the BERT-base step and one plain product, interleaved rounds in one process.
T tokens (default 524288 = the b1024 step).  One JSON line per product: median us per call."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_and_deepspeed_amd.ops import _lib  # noqa: E402
from distributed_training_and_deepspeed_amd.ops import gemm as G  # noqa: E402


def timed(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    T = int(os.environ.get("T", 524288))
    rounds = int(os.environ.get("ROUNDS", 5))
    H, F = 768, 3072
    bf = torch.bfloat16
    torch.manual_seed(0)
    x = torch.randn(T, H, device="cuda", dtype=bf)
    dy = torch.randn(T, H, device="cuda", dtype=bf)
    g = torch.rand(T, F, device="cuda", dtype=bf)
    w1 = (torch.randn(F, H, device="cuda") * 0.03).to(bf)
    b1 = torch.randn(F, device="cuda", dtype=bf) * 0.1
    w2t = (torch.randn(F, H, device="cuda") * 0.03).to(bf)   # fc2's W^T [ffn, hidden]
    db = torch.zeros(F, device="cuda", dtype=torch.float32)
    cases = {
        "fc1_gelu_grad": lambda: G.linear_act_grad(x, w1, b1),
        "fc2_dgrad_mul": lambda: G.mul_bwd_gemm(dy, w2t, g, dbias=(db, False)),
        "fc1_plain": lambda: G.gemm_bt(x, w1, b1),
    }
    fl = 2 * T * H * F
    # correctness: spread and bunched forms must agree bit for bit
    outs = {}
    for sp in (0, 1):
        _lib.call("dtd_gemm_set_spread", sp)
        outs[sp] = [c() for c in cases.values()]
    same = {k: all(torch.equal(a, b) for a, b in zip(o0 if isinstance(o0, tuple) else (o0,),
                                                     o1 if isinstance(o1, tuple) else (o1,)))
            for k, o0, o1 in zip(cases, outs[0], outs[1])}
    print(json.dumps({"bitwise_equal": same}), flush=True)
    del outs
    times = {k: {0: [], 1: []} for k in cases}
    for _ in range(rounds):
        for k, fn in cases.items():
            for sp in (0, 1):
                _lib.call("dtd_gemm_set_spread", sp)
                times[k][sp].append(timed(fn, 5))
    _lib.call("dtd_gemm_set_spread", 1)
    for k in cases:
        b, s = statistics.median(times[k][0]), statistics.median(times[k][1])
        print(json.dumps({k: {"bunched_us": round(b, 1), "spread_us": round(s, 1), "speedup": round(b / s, 3),
                              "spread_TF": round(fl / s / 1e6, 1)}}), flush=True)


if __name__ == "__main__":
    main()
