#!/usr/bin/env bash
# GEMM limiter probe 2: DMA latency vs issue (diag 8: DMA never waited for), one-barrier variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
OPS=$PWD/distributed_training_and_deepspeed_amd/ops
for r in 1 2; do
  step diag_base_$r 120 python -u scripts/gemm_diag.py
  step diag8_$r 120 env DTD_KERNELS_SO=$OPS/_dtd_kernels_diag8.so python -u scripts/gemm_diag.py
  step onebar_$r 120 env DTD_KERNELS_SO=$OPS/_dtd_kernels_onebar.so python -u scripts/gemm_diag.py
done
echo done
