#!/usr/bin/env bash
# Kernel-library A/B on one box: ops/_dtd_kernels_base.so (baseline build) vs the tree's build.
# Usage: bash scripts/gpu_so_ab.sh [pytest-target]   (attention micro-benchmark + whole-step A/B)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${1:-tests/test_attention_gpu.py}
timeout -k 10 300 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_ab.log 2>&1 || { tail -30 gpurun_out/pt_ab.log; exit 1; }
tail -1 gpurun_out/pt_ab.log
BASE=$PWD/distributed_training_and_deepspeed_amd/ops/_dtd_kernels_base.so
for i in 1 2; do
  DTD_KERNELS_SO=$BASE B=128 P=0.1 timeout -k 10 60 python scripts/bench_attn.py 3,2,3 2>/dev/null | sed "s/^/base /" || exit 1
  B=128 P=0.1 timeout -k 10 60 python scripts/bench_attn.py 3,2,3 2>/dev/null | sed "s/^/new  /" || exit 1
done
timeout -k 10 900 python scripts/ab.py base_so base --rounds 3 -- --steps 12 --warmup 4
