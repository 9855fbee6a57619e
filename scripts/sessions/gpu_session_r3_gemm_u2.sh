#!/usr/bin/env bash
# GEMM: uniform wave index (scalar LDS-DMA destinations) in v1; U2 = K loop unrolled by two with
# compile-time buffers and branch-free staging.  Tests under both forms, timings vs hipBLASLt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step gemm_tests_v1 400 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread
step gemm_tests_v2 400 env DTD_GEMM_VARIANT=2 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread
step bench_v2 600 env VNEW=2 ROUNDS=5 python scripts/bench_gemm_v2.py
step bench_base 600 env VNEW=1 ROUNDS=5 DTD_KERNELS_SO=distributed_training_and_deepspeed_amd/ops/_dtd_kernels_base.so python scripts/bench_gemm_v2.py
echo done
