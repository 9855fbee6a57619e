#!/usr/bin/env bash
# Persistent 8-phase GEMM: tests under both kernel forms, then the A/B bench for each form.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step gemm_tests_p 300 python -u -m pytest tests/test_gemm_gpu.py -x -v --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/gemm_tests_p.log && ! grep -q "failed" gpurun_out/gemm_tests_p.log || exit 1
DTD_GEMM_VARIANT=0 step gemm_tests_t 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread
step gemm_bench_p 400 python -u scripts/bench_gemm8.py
DTD_GEMM_VARIANT=0 step gemm_bench_t 400 python -u scripts/bench_gemm8.py
echo done
