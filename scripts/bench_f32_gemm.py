#!/usr/bin/env python
"""fp32 GEMM throughput of the vendor library (hipBLASLt / rocBLAS through torch) at the BERT-base
projection shapes, against the 157 TF/s f32 MFMA peak: decides whether the reference-precision
path needs a hand-written f32 GEMM (cdna_hip_programming.md §3: an untuned f32-MFMA kernel
reaches 122 TF/s at 4096^3)."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=5):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    T = int(os.environ.get("T", 32768))
    H, F = 768, 3072
    torch.manual_seed(0)
    x = torch.randn(T, H, device="cuda")
    xf = torch.randn(T, F, device="cuda")
    w = {"qkv": torch.randn(3 * H, H, device="cuda"), "o": torch.randn(H, H, device="cuda"),
         "fc1": torch.randn(F, H, device="cuda"), "fc2": torch.randn(H, F, device="cuda")}
    L = torch.nn.functional.linear
    cases = {"fwd_qkv": (x, w["qkv"]), "fwd_o": (x, w["o"]), "fwd_fc1": (x, w["fc1"]), "fwd_fc2": (xf, w["fc2"])}
    out = {}
    for k, (a, b) in cases.items():
        fl = 2 * a.shape[0] * a.shape[1] * b.shape[0]
        ts = [timed(lambda a=a, b=b: L(a, b)) for _ in range(3)]
        t = statistics.median(ts)
        out[k] = {"us": round(t, 1), "TF": round(fl / t / 1e6, 1)}
        print(json.dumps({k: out[k]}), flush=True)
    # the hand-written f32-MFMA kernel (ops/csrc/gemm_f32.hip): NT forward and split-K TN wgrad
    from distributed_training_and_deepspeed_amd.ops import gemm as G
    G.set_f32(True)
    for k, (a, b) in cases.items():
        fl = 2 * a.shape[0] * a.shape[1] * b.shape[0]
        t = statistics.median([timed(lambda a=a, b=b: G.gemm_f32_nt(a, b)) for _ in range(3)])
        out["hand_" + k] = {"us": round(t, 1), "TF": round(fl / t / 1e6, 1)}
        print(json.dumps({"hand_" + k: out["hand_" + k]}), flush=True)
    dy = {"qkv": torch.randn(T, 3 * H, device="cuda"), "o": x, "fc1": torch.randn(T, F, device="cuda"), "fc2": x}
    xin = {"qkv": x, "o": x, "fc1": x, "fc2": xf}
    for k in ("qkv", "o", "fc1", "fc2"):
        fl = 2 * T * dy[k].shape[1] * xin[k].shape[1]
        t = statistics.median([timed(lambda k=k: dy[k].t() @ xin[k]) for _ in range(3)])
        out["wgrad_" + k] = {"us": round(t, 1), "TF": round(fl / t / 1e6, 1)}
        t = statistics.median([timed(lambda k=k: G.gemm_f32_tn(dy[k], xin[k]).sum(0)) for _ in range(3)])
        out["hand_wgrad_" + k] = {"us": round(t, 1), "TF": round(fl / t / 1e6, 1)}
        print(json.dumps({k: [out["wgrad_" + k], out["hand_wgrad_" + k]]}), flush=True)
    # input gradients dY W [out, in]: library matmul vs the hand NN form (no transposed weight copy)
    for k in ("qkv", "o", "fc1", "fc2"):
        wk = w[k]
        d = dy[k] if k in ("qkv", "fc1") else (x if k == "o" else x)
        fl = 2 * T * wk.shape[0] * wk.shape[1]
        t = statistics.median([timed(lambda d=d, wk=wk: d @ wk) for _ in range(3)])
        out["dgrad_" + k] = {"us": round(t, 1), "TF": round(fl / t / 1e6, 1)}
        t = statistics.median([timed(lambda d=d, wk=wk: G.gemm_f32_nn(d, wk)) for _ in range(3)])
        out["hand_dgrad_" + k] = {"us": round(t, 1), "TF": round(fl / t / 1e6, 1)}
        print(json.dumps({"dgrad_" + k: [out["dgrad_" + k], out["hand_dgrad_" + k]]}), flush=True)
    # the same with TF32-like reduced precision explicitly off (torch's default for fp32 matmul)
    print(json.dumps({"T": T, "allow_tf32": torch.backends.cuda.matmul.allow_tf32, "results": out}), flush=True)


if __name__ == "__main__":
    main()
