#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
step pytest_k 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread
step elem 300 python scripts/bench_elementwise.py
step elem2 300 python scripts/bench_elementwise.py
echo done
