#!/usr/bin/env bash
# Round 5 session 8: ring-pipelined projection GEMM (gemm_nt.hip) -- numerics and per-product A/B
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step tests_nt 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -k "gemm_nt"
step bench_nt 400 env ROUNDS=5 python -u scripts/bench_gemm_nt.py
echo done
