#!/usr/bin/env bash
# GEMM LDS-DMA placement variants: correctness (GEMM tests) for order 2 and no-prio, limiter timing
# for base / order1 / order2 / noprio / order2+noprio.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
OPS=$PWD/distributed_training_and_deepspeed_amd/ops
step pytest_o2 300 env DTD_KERNELS_SO=$OPS/_dtd_kernels_order2.so python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread
step pytest_o1 300 env DTD_KERNELS_SO=$OPS/_dtd_kernels_order1.so python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread
for r in 1 2; do
  step t_base_$r 120 python -u scripts/gemm_diag.py
  for v in order1 order2 noprio o2np; do step t_${v}_$r 120 env DTD_KERNELS_SO=$OPS/_dtd_kernels_$v.so python -u scripts/gemm_diag.py; done
done
echo done
