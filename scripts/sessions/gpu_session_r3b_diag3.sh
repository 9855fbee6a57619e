#!/usr/bin/env bash
# GEMM limiter probe 3: L2-hot staging source (diag 16) and A-only staging (diag 32).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
OPS=$PWD/distributed_training_and_deepspeed_amd/ops
for r in 1 2; do
  step diag_base_$r 120 python -u scripts/gemm_diag.py
  step diag16_$r 120 env DTD_KERNELS_SO=$OPS/_dtd_kernels_diag16.so python -u scripts/gemm_diag.py
  step diag32_$r 120 env DTD_KERNELS_SO=$OPS/_dtd_kernels_diag32.so python -u scripts/gemm_diag.py
done
echo done
