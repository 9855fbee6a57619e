#!/usr/bin/env python
"""Micro-benchmark of the BERT GEMM shapes on MI355X: hipBLASLt default vs split-K batched
weight-gradient GEMMs (and TunableOp when PYTORCH_TUNABLEOP_ENABLED=1).

Weight-gradient GEMMs dW[out,in] = dY^T[out,T] @ X[T,in] have a huge K (= tokens) and a small
output (144 tiles of 128x128 for a 768x3072 weight): a single GEMM fills only part of the 256
CUs.  Splitting K into `s` slices as one batched GEMM multiplies the tile count by s.
"""
import json
import sys

import torch


def t_ms(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    dev = "cuda"
    bf = torch.bfloat16
    res = []
    for T in (16384, 2048):
        for (o, i) in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
            dy = torch.randn(T, o, device=dev, dtype=bf)
            x = torch.randn(T, i, device=dev, dtype=bf)
            w = torch.randn(o, i, device=dev, dtype=bf)
            g16 = torch.empty(o, i, device=dev, dtype=bf)
            g32 = torch.empty(o, i, device=dev, dtype=torch.float32)
            fl = 2.0 * T * o * i
            row = {"T": T, "out": o, "in": i}
            row["fwd"] = t_ms(lambda: torch.nn.functional.linear(x, w))
            row["dgrad"] = t_ms(lambda: dy @ w)
            row["wgrad_bf16"] = t_ms(lambda: torch.mm(dy.t(), x, out=g16))
            try:
                row["wgrad_f32out"] = t_ms(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32, out=g32))
            except Exception as ex:  # noqa
                row["wgrad_f32out"] = str(ex)[:60]
            for s in (2, 4, 8, 16):
                if T % s:
                    continue
                a3 = dy.view(s, T // s, o).transpose(1, 2)
                b3 = x.view(s, T // s, i)

                def f(a3=a3, b3=b3):
                    p = torch.bmm(a3, b3)
                    torch.sum(p, 0, dtype=torch.float32, out=g32)
                row[f"splitk{s}"] = t_ms(f)

                def f32(a3=a3, b3=b3):
                    p = torch.bmm(a3, b3, out_dtype=torch.float32)
                    torch.sum(p, 0, out=g32)
                try:
                    row[f"splitk{s}_f32"] = t_ms(f32)
                except Exception as ex:  # noqa
                    row[f"splitk{s}_f32"] = str(ex)[:60]
            best = min((v, k) for k, v in row.items() if k.startswith(("wgrad", "splitk")) and isinstance(v, float))
            row["best"] = best[1]
            row["best_TF"] = round(fl / best[0] / 1e9, 1)
            row["fwd_TF"] = round(fl / row["fwd"] / 1e9, 1)
            row["wgrad_TF"] = round(fl / row["wgrad_bf16"] / 1e9, 1)
            res.append(row)
            print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in row.items()}), flush=True)


if __name__ == "__main__":
    sys.exit(main())
