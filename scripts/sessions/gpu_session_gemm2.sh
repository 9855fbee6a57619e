#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
step pytest_gemm 300 python -u -m pytest tests/test_gemm_gpu.py -x -v --timeout 120 --timeout-method thread
step bench_gemm_fused 300 python scripts/bench_gemm_fused.py --tuned
echo done
