#!/usr/bin/env bash
# Round 5 session 7: wgrad.hip four-wave form (one wave per SIMD, 128x128 per wave)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step tests_wgrad 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -k "wgrad"
step bench_wgrad 400 env ROUNDS=5 VARIANTS=44,84 python -u scripts/bench_wgrad.py
echo done
