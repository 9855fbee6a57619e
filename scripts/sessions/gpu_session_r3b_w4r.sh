#!/usr/bin/env bash
# W4R (4 waves, register-staged operands) GEMM form: correctness (bench_gemm_v2 check + GEMM tests
# with DTD_GEMM_VARIANT=4) and timing vs v1 / hipBLASLt at the BERT shapes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step w4r_v2bench 400 env VNEW=4 python -u scripts/bench_gemm_v2.py
step pytest_gemm_w4r 300 env DTD_GEMM_VARIANT=4 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread
echo done
