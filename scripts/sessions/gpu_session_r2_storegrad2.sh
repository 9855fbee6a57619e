#!/usr/bin/env bash
# Kernel times of the derivative-storing FFN epilogue pair vs the u-storing pair, and a b256
# kernel summary of the default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
ROUNDS=3 step gemm_bench 600 python -u scripts/bench_gemm8.py
step bench 600 python -u bench.py --steps 20 --warmup 5
echo done
