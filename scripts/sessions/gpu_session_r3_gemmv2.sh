#!/usr/bin/env bash
# GEMM v2 (deferred quadrant epilogue): correctness + timing vs v1 and hipBLASLt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step gemm_v2 300 env VNEW=5 python scripts/bench_gemm_v2.py
echo done
