#!/usr/bin/env bash
# Round 5 session 5: wgrad.hip -- K loop unrolled by the ring (static LDS offsets), pinned read groups
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step tests_wgrad 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -k "wgrad"
step bench_wgrad 400 env ROUNDS=7 VARIANTS=4,44,5 python -u scripts/bench_wgrad.py
echo done
