#!/usr/bin/env bash
# Round 5 session 1: ring-pipelined TN weight-gradient kernel (ops/csrc/wgrad.hip) -- numerics,
# then the per-shape A/B against the library path and the round-3 TN kernel; baseline bench
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step tests_wgrad2 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -k "wgrad"
step bench_wgrad 400 env ROUNDS=5 python -u scripts/bench_wgrad.py
step bench_base 300 python -u bench.py --steps 20 --warmup 5
echo done
