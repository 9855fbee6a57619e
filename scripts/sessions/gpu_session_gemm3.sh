#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
step pytest_gemm128 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread
DTD_GEMM_BN=256 step pytest_gemm256 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread
step bench128 300 python scripts/bench_gemm_fused.py --tuned
DTD_GEMM_BN=256 step bench256 300 python scripts/bench_gemm_fused.py --tuned
echo done
