#!/usr/bin/env python
"""The 8-phase MFMA GEMM (ops/csrc/gemm.hip) vs hipBLASLt at the BERT-base training shapes.

T tokens (default 131072 = bench.py's 256 x 512).  For every projection of a layer: forward
(x W^T + b), input-gradient (dy W via the transposed weight) and the fused FFN variants
(bias+GELU forward, GELU-backward dgrad with the bias-gradient partials) against hipBLASLt +
the unfused elementwise kernels.  Variants are timed in interleaved rounds in one process
(cdna_hip_programming.md §5.4 rule 24); the JSON line has the median us and TF/s per row.
Correctness: each fused output is compared against an fp32 reference on a 1024-row slice.
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_and_deepspeed_amd.ops import functional as Fx  # noqa: E402
from distributed_training_and_deepspeed_amd.ops import gemm as G  # noqa: E402


def timed(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def main():
    if "--untuned" not in sys.argv:
        from distributed_training_and_deepspeed_amd.utils.tuning import use_tuned_gemms
        use_tuned_gemms()
    T = int(os.environ.get("T", 131072))
    rounds = int(os.environ.get("ROUNDS", 5))
    H, F = 768, 3072
    bf = torch.bfloat16
    dev = "cuda"
    torch.manual_seed(0)
    x = torch.randn(T, H, device=dev, dtype=bf)
    xf = torch.randn(T, F, device=dev, dtype=bf)
    dy3 = torch.randn(T, 3 * H, device=dev, dtype=bf)
    w = {n: (torch.randn(o, i, device=dev) * 0.03).to(bf)
         for n, (o, i) in {"qkv": (3 * H, H), "o": (H, H), "fc1": (F, H), "fc2": (H, F)}.items()}
    b = {n: torch.randn(t.shape[0], device=dev, dtype=bf) * 0.1 for n, t in w.items()}
    wt = {n: t.t().contiguous() for n, t in w.items()}
    u = torch.randn(T, F, device=dev, dtype=bf)
    db = torch.zeros(F, device=dev, dtype=torch.float32)
    res = torch.randn(T, H, device=dev, dtype=bf)

    # ---- correctness on a slice (fp32 reference)
    S = 1024
    chk = {}
    chk["fwd_qkv"] = rel(G.linear(x[:S], w["qkv"], b["qkv"]), x[:S].float() @ w["qkv"].float().t() + b["qkv"].float())
    uu, aa = G.linear_gelu(x[:S], w["fc1"], b["fc1"])
    chk["fwd_fc1_u"] = rel(uu, x[:S].float() @ w["fc1"].float().t() + b["fc1"].float())
    chk["fwd_fc1_gelu_exact"] = float(torch.equal(aa, Fx.act_fwd(uu, "gelu")))
    chk["dgrad_fc1"] = rel(G.matmul_nt(xf[:S], wt["fc1"]), xf[:S].float() @ w["fc1"].float())
    r2 = res[:S].clone()
    G.matmul_nt_add_(r2, dy3[:S], wt["qkv"])
    chk["dgrad_add_qkv"] = rel(r2, res[:S].float() + dy3[:S].float() @ w["qkv"].float())
    dbs = torch.zeros(F, device=dev, dtype=torch.float32)
    du = G.gelu_bwd_gemm(x[:S], wt["fc2"], u[:S], dbias=(dbs, False))
    ug = u[:S].float()
    gp = 0.5 * (1 + torch.erf(ug / 2 ** 0.5)) + ug * torch.exp(-0.5 * ug * ug) / (2 * torch.pi) ** 0.5
    duref = (x[:S].float() @ w["fc2"].float()) * gp
    chk["dgrad_gelu_bwd"] = rel(du, duref)
    chk["dgrad_gelu_dbias"] = rel(dbs, duref.sum(0))
    print(json.dumps({"check": {k: round(v, 6) for k, v in chk.items()}}), flush=True)

    L = torch.nn.functional.linear
    cases = {
        # name: (flops, hipblaslt fn, ours fn)
        "fwd_qkv": (2 * T * H * 3 * H, lambda: L(x, w["qkv"], b["qkv"]), lambda: G.linear(x, w["qkv"], b["qkv"])),
        "fwd_o": (2 * T * H * H, lambda: L(x, w["o"], b["o"]), lambda: G.linear(x, w["o"], b["o"])),
        "fwd_fc1": (2 * T * H * F, lambda: L(x, w["fc1"], b["fc1"]), lambda: G.linear(x, w["fc1"], b["fc1"])),
        "fwd_fc1_gelu": (2 * T * H * F, lambda: Fx.act_fwd(L(x, w["fc1"], b["fc1"]), "gelu"),
                         lambda: G.linear_gelu(x, w["fc1"], b["fc1"])),
        "fwd_fc2": (2 * T * H * F, lambda: L(xf, w["fc2"], b["fc2"]), lambda: G.linear(xf, w["fc2"], b["fc2"])),
        "dgrad_qkv": (2 * T * H * 3 * H, lambda: dy3 @ w["qkv"], lambda: G.matmul_nt(dy3, wt["qkv"])),
        "dgrad_add_qkv": (2 * T * H * 3 * H, lambda: res.addmm_(dy3, w["qkv"]), lambda: G.matmul_nt_add_(res, dy3, wt["qkv"])),
        "dgrad_o": (2 * T * H * H, lambda: x @ w["o"], lambda: G.matmul_nt(x, wt["o"])),
        "dgrad_fc1": (2 * T * H * F, lambda: xf @ w["fc1"], lambda: G.matmul_nt(xf, wt["fc1"])),
        "dgrad_fc2": (2 * T * H * F, lambda: x @ w["fc2"], lambda: G.matmul_nt(x, wt["fc2"])),
        "dgrad_fc2_gelu_bwd": (2 * T * H * F, lambda: Fx.act_bwd(x @ w["fc2"], u, "gelu", dbias=(db, False)),
                               lambda: G.gelu_bwd_gemm(x, wt["fc2"], u, dbias=(db, False))),
        # derivative-storing pair (the model default): the forward also emits gelu'(u), the
        # backward epilogue multiplies (the hipBLASLt column is the same unfused baseline)
        "fwd_fc1_gelu_grad": (2 * T * H * F, lambda: Fx.act_fwd(L(x, w["fc1"], b["fc1"]), "gelu"),
                              lambda: G.linear_act_grad(x, w["fc1"], b["fc1"])),
        "dgrad_fc2_mul_bwd": (2 * T * H * F, lambda: Fx.act_bwd(x @ w["fc2"], u, "gelu", dbias=(db, False)),
                              lambda: G.mul_bwd_gemm(x, wt["fc2"], u, dbias=(db, False))),
        "transpose_fc1": (0, lambda: None, lambda: G.transpose(w["fc1"])),
        # input gradients as the model's default issues them: hipBLASLt in the NT form on the
        # transposed weight (its forward-layout kernels), vs the same kernel as above
        "dgradnt_qkv": (2 * T * H * 3 * H, lambda: L(dy3, wt["qkv"]), lambda: G.matmul_nt(dy3, wt["qkv"])),
        "dgradnt_add_qkv": (2 * T * H * 3 * H, lambda: res.addmm_(dy3, wt["qkv"].t()),
                            lambda: G.matmul_nt_add_(res, dy3, wt["qkv"])),
        "dgradnt_o": (2 * T * H * H, lambda: L(x, wt["o"]), lambda: G.matmul_nt(x, wt["o"])),
        "dgradnt_fc1": (2 * T * H * F, lambda: L(xf, wt["fc1"]), lambda: G.matmul_nt(xf, wt["fc1"])),
    }
    # weight gradients: hipBLASLt split-K (16 x T/16-token slices, bf16 partials) + reduce vs the
    # TN kernel (fp32 partials, one wave of workgroups) + reduce
    from distributed_training_and_deepspeed_amd.ops.grad import splitk_reduce
    gw = {n: torch.empty(t.shape, device=dev, dtype=bf) for n, t in w.items()}

    def hip_wgrad(dy_, x_, dst):
        o_, i_ = dy_.shape[1], x_.shape[1]
        splitk_reduce(torch.bmm(dy_.view(16, T // 16, o_).transpose(1, 2), x_.view(16, T // 16, i_)), dst, False)

    for n, (dy_, x_) in {"qkv": (dy3, x), "o": (x, x), "fc1": (xf, x), "fc2": (x, xf)}.items():
        fl = 2 * T * dy_.shape[1] * x_.shape[1]
        cases[f"wgrad_{n}"] = (fl, lambda dy_=dy_, x_=x_, d=gw[n]: hip_wgrad(dy_, x_, d),
                               lambda dy_=dy_, x_=x_, d=gw[n]: splitk_reduce(G.wgrad_tn(dy_, x_), d, False))
    chk["wgrad_fc1"] = rel(G.wgrad_tn(xf[:S], x[:S]).sum(0), xf[:S].float().t() @ x[:S].float())
    print(json.dumps({"check_wgrad": round(chk["wgrad_fc1"], 6)}), flush=True)
    times = {k: ([], []) for k in cases}
    for k, (_, f0, f1) in cases.items():   # warm-up (TunableOp lookups, code objects)
        f0(), f1()
    torch.cuda.synchronize()
    for _ in range(rounds):
        for k, (_, f0, f1) in cases.items():
            times[k][0].append(timed(f0, 10))
            times[k][1].append(timed(f1, 10))
    out = {}
    for k, (fl, _, _) in cases.items():
        t0, t1 = statistics.median(times[k][0]), statistics.median(times[k][1])
        row = {"hipblaslt_us": round(t0, 1), "ours_us": round(t1, 1), "speedup": round(t0 / t1, 3)}
        if fl:
            row["hipblaslt_TF"] = round(fl / t0 / 1e6, 1)
            row["ours_TF"] = round(fl / t1 / 1e6, 1)
        out[k] = row
        print(json.dumps({k: row}), flush=True)
    print(json.dumps({"T": T, "rounds": rounds, "results": out}), flush=True)


if __name__ == "__main__":
    main()
