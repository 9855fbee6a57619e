#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step tests 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread
echo done
