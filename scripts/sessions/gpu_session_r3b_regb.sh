#!/usr/bin/env bash
# Register-staged B panel in the persistent GEMM (DTD_GEMM_REGB=1 build): GEMM tests under it,
# limiter probe base vs regb, bench_gemm8 with it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
OPS=$PWD/distributed_training_and_deepspeed_amd/ops
step pytest_gemm_regb 300 env DTD_KERNELS_SO=$OPS/_dtd_kernels_regb.so python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread
for r in 1 2; do
  step diag_base_$r 120 python -u scripts/gemm_diag.py
  step diag_regb_$r 120 env DTD_KERNELS_SO=$OPS/_dtd_kernels_regb.so python -u scripts/gemm_diag.py
done
step gemm8_regb 300 env DTD_KERNELS_SO=$OPS/_dtd_kernels_regb.so python -u scripts/bench_gemm8.py
echo done
