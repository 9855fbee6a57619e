#!/usr/bin/env bash
# Round 5 session 37: projection GEMM with B packed in fragment order (ops/csrc/proj.hip): numerics,
# then per-product timing against hipBLASLt
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step proj_tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_proj_gpu.py
step bench_proj 400 env ROUNDS=5 python -u scripts/bench_proj.py
echo done
