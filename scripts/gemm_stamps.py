#!/usr/bin/env python
"""Where a GEMM tile's time goes: in-kernel s_memtime stamps (diagnostic build of gemm.hip).

``--build`` (CPU, here): compiles every kernel source with -DDTD_GEMM_STAMPS into
``ops/_dtd_kernels_stamps.so`` (in-tree, so it travels to the GPU box).
Run (GPU): loads that library through DTD_KERNELS_SO, runs C = A B^T once per shape with a
stamp buffer and prints, per shape, the median shader cycles of each segment of a tile:
tile form   : prologue (DMA of K-step 0 + wait), main loop, LDS image write, row stores issued,
              stores drained, and the gap between consecutive workgroups on one CU (dispatch);
persistent  : main loop, epilogue, and the whole tile.
"""
import json
import os
import statistics
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "distributed_training_and_deepspeed_amd"
SO = PKG / "ops" / "_dtd_kernels_stamps.so"


def build():
    srcs = sorted((PKG / "ops" / "csrc").glob("*.hip")) + sorted((PKG / "comm" / "csrc").glob("*.hip"))
    objs = []
    od = PKG / "ops" / "build_stamps"
    od.mkdir(exist_ok=True)
    for s in srcs:
        o = od / (s.stem + ".o")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", str(s), "-o", str(o),
                        "-I", str(PKG / "ops" / "csrc"), "-fvisibility=hidden", "-DDTD_GEMM_STAMPS"], check=True)
        objs.append(str(o))
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", str(SO), *objs], check=True)
    print("built", SO)


def run():
    os.environ["DTD_KERNELS_SO"] = str(SO)
    sys.path.insert(0, str(ROOT))
    import torch
    from distributed_training_and_deepspeed_amd.ops import _lib
    from distributed_training_and_deepspeed_amd.ops import gemm as G
    variant = int(os.environ.get("DTD_GEMM_VARIANT", "1"))
    M = int(os.environ.get("M", 131072))
    shapes = [(768, 768), (2304, 768), (768, 3072), (768, 6144)]
    res = {}
    for N, K in shapes:
        a = torch.rand(M, K, device="cuda", dtype=torch.bfloat16) * 2 - 1
        b = torch.rand(N, K, device="cuda", dtype=torch.bfloat16) * 2 - 1
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        ntiles = (M // 256) * (N // 256)
        nwg = ntiles if variant == 0 else 256
        st = torch.zeros(nwg * 32 * 8, dtype=torch.int64, device="cuda")
        for _ in range(3):
            G._call(G.EPI_STORE, a, b, c)
        _lib.lib().dtd_gemm_set_stamps(ctypes_ptr(st))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        G._call(G.EPI_STORE, a, b, c)
        e1.record()
        torch.cuda.synchronize()
        _lib.lib().dtd_gemm_set_stamps(None)
        us = e0.elapsed_time(e1) * 1e3
        s = st.view(nwg, 32, 8).cpu().numpy().astype("uint64")
        seg = {}
        if variant == 0:
            w = s[:, 0, :]
            names = ["prologue", "mainloop", "image", "stores_issue", "stores_drain"]
            for i, n in enumerate(names):
                seg[n] = int(statistics.median((w[:, i + 1] - w[:, i]).astype("int64").tolist()))
            # dispatch gaps: consecutive workgroups on the same CU (XCC id, HW_ID bits 8..15)
            cu = {}
            for k in range(nwg):
                key = (int(w[k, 7]) >> 32, (int(w[k, 7]) >> 8) & 0xFF)
                cu.setdefault(key, []).append((int(w[k, 0]), int(w[k, 5])))
            gaps = []
            for v in cu.values():
                v.sort()
                gaps += [v[i + 1][0] - v[i][1] for i in range(len(v) - 1)]
            seg["dispatch_gap"] = int(statistics.median(gaps)) if gaps else -1
            seg["cus_seen"] = len(cu)
            span = [int(w[:, 5].max()) - int(w[:, 0].min())]
        else:
            ml, ep, tot = [], [], []
            for k in range(nwg):
                for it in range(32):
                    r = s[k, it]
                    if r[0] == 0 or r[4] == 0:
                        continue
                    ml.append(int(r[2]) - int(r[0]))
                    ep.append(int(r[4]) - int(r[2]))
                    if it + 1 < 32 and s[k, it + 1, 0] != 0:
                        tot.append(int(s[k, it + 1, 0]) - int(r[0]))
            seg = {"mainloop": int(statistics.median(ml)), "epilogue": int(statistics.median(ep)),
                   "tile": int(statistics.median(tot)) if tot else -1}
            span = [int(s[:, :, 4].max()) - int(s[s[:, :, 0] > 0][:, 0].min())]
        seg["kernel_us"] = round(us, 1)
        seg["span_cycles"] = span[0]
        seg["MHz_est"] = round(span[0] / us, 0)
        res[f"N{N}_K{K}"] = seg
        print(json.dumps({f"N{N}_K{K}": seg}), flush=True)
    print(json.dumps({"variant": variant, "M": M, "segments_cycles": res}), flush=True)


def ctypes_ptr(t):
    return t.data_ptr()


if __name__ == "__main__":
    if "--build" in sys.argv:
        build()
    else:
        run()
