#!/usr/bin/env bash
# Round 5 session 2: wgrad.hip after the B-fragment swizzle fix -- numerics, per-shape A/B
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step tests_wgrad2 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -k "wgrad"
step bench_wgrad 400 env ROUNDS=7 python -u scripts/bench_wgrad.py
echo done
