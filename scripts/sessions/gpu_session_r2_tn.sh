#!/usr/bin/env bash
# TN weight-gradient kernel with the XCD-aware split order: GEMM tests + wgrad rows vs hipBLASLt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step tests 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/tests.log && ! grep -q "failed" gpurun_out/tests.log || exit 1
ROUNDS=3 step gemm_bench 600 python -u scripts/bench_gemm8.py
echo done
