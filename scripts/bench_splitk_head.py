"""LM-head input gradient dX = dLogits [M, V] . E [V, h] at small M (bloom-560m at micro-batch 1:
M = 511, V = 250880, h = 1024): the library's one-pass GEMM has 128 output tiles for a
V-long reduction.  Times it against the K-split strided-batch form (fp32 partials + one sum)."""
import json
import statistics
import sys

import torch


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps * 1e3


def splitk(a, b, s):
    M, K = a.shape
    part = torch.bmm(a.view(M, s, K // s).transpose(0, 1), b.view(s, K // s, b.shape[1]), out_dtype=torch.float32)
    return part.sum(0).to(a.dtype)


def main():
    out = {}
    for M, V, h in ((511, 250880, 1024), (2047, 250880, 1024), (511, 50304, 768)):
        a = torch.randn(M, V, device="cuda", dtype=torch.bfloat16) * 1e-2
        b = torch.randn(V, h, device="cuda", dtype=torch.bfloat16)
        ref = a.float() @ b.float()
        rec = {"lib_us": statistics.median(timed(lambda: a @ b) for _ in range(3)),
               "lib_rel": ((a @ b).float() - ref).norm().item() / ref.norm().item()}
        for s in (2, 4, 8, 16, 32):
            if V % s:
                continue
            rec[f"s{s}_us"] = statistics.median(timed(lambda s=s: splitk(a, b, s)) for _ in range(3))
            rec[f"s{s}_rel"] = (splitk(a, b, s).float() - ref).norm().item() / ref.norm().item()
        out[f"{M}x{V}x{h}"] = rec
        print(json.dumps({f"{M}x{V}x{h}": rec}), flush=True)
        del a, b, ref
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(out, f)


if __name__ == "__main__":
    main()
