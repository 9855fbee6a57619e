#!/usr/bin/env python
"""Generate attn_fwd_traced.hip: a copy of ops/csrc/attention.hip whose register-ring forward
kernel writes s_memrealtime stamps (entry, after the prologue barrier, after tiles 0 / nt-2 /
nt-1, before / after the epilogue) per workgroup into a device buffer.  Build and run:

  python scripts/experiments/make_traced_attn.py
  cd scripts/experiments && hipcc --offload-arch=gfx950 -O3 -std=c++17 \
      -I../../distributed_training_and_deepspeed_amd/ops/csrc attn_trace_main.hip -o attn_trace
  ./attn_trace 32 512 trace.csv && python attn_trace_stats.py trace.csv      (on the GPU box)
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "..", "..", "distributed_training_and_deepspeed_amd", "ops", "csrc", "attention.hip")


def find(lines, pat, start=0):
    for i in range(start, len(lines)):
        if pat in lines[i]:
            return i
    raise SystemExit(f"pattern not found: {pat}")


def main():
    lines = open(SRC).read().split("\n")
    stamp = "if (threadIdx.x == 0) g_trace[wg_ * 8 + {k}] = __builtin_amdgcn_s_memrealtime();"
    k = find(lines, "attn_fwd_kernel(FwdArgs a) {")
    e = find(lines, "  xcd_tile(tx, ty);", k)
    lines[e] += "\n  const int wg_ = blockIdx.x + gridDim.x * blockIdx.y;\n  " + stamp.format(k=0)
    p = find(lines, "  __syncthreads();", k)
    lines[p] += "\n  " + stamp.format(k=1)
    t = find(lines, "    __syncthreads();", p + 1)
    lines[t] += ("\n    if (t == 0) { " + stamp.format(k=2) + " }"
                 "\n    if (t == nt - 2) { " + stamp.format(k=3) + " }"
                 "\n    if (t == nt - 1) { " + stamp.format(k=4) + " }")
    r = find(lines, "  if (!qvalid) return;", t)
    lines[r] = "  " + stamp.format(k=5) + "\n" + lines[r]
    l_ = find(lines, "  if (hh == 0) a.lse[(size_t)bh * S + q] = (m + log2f(l)) * kLn2;", r)
    lines[l_] += "\n  __syncthreads();\n  " + stamp.format(k=6)
    out = "\n".join(lines).replace("using namespace dtd;",
                                   "using namespace dtd;\n__device__ unsigned long long* g_trace;", 1)
    open(os.path.join(HERE, "attn_fwd_traced.hip"), "w").write(out)


if __name__ == "__main__":
    main()
