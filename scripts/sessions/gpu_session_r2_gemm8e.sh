#!/usr/bin/env bash
# k-half phase layout (variant 2) vs quadrant layout (variant 1): tests, probe, stamps, model shapes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
DTD_GEMM_VARIANT=2 step gemm_tests_2 300 python -u -m pytest tests/test_gemm_gpu.py -x -v --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/gemm_tests_2.log && ! grep -q "failed" gpurun_out/gemm_tests_2.log || exit 1
DTD_GEMM_VARIANT=2 step probe_2 300 python -u scripts/gemm_probe.py
DTD_GEMM_VARIANT=1 step probe_1 300 python -u scripts/gemm_probe.py
DTD_GEMM_VARIANT=2 step stamps_2 200 python -u scripts/gemm_stamps.py
DTD_GEMM_VARIANT=2 step gemm_bench_2 400 python -u scripts/bench_gemm8.py
echo done
