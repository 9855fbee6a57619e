#!/usr/bin/env bash
# TN weight-gradient GEMM: tests, then model-shape A/B incl. wgrad rows, then the bench A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step gemm_tests 300 python -u -m pytest tests/test_gemm_gpu.py -x -v --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/gemm_tests.log && ! grep -q "failed" gpurun_out/gemm_tests.log || exit 1
step gemm_bench 500 python -u scripts/bench_gemm8.py
echo done
