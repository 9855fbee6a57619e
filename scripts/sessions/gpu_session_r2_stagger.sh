#!/usr/bin/env bash
# persistent GEMM start stagger sweep (DTD_GEMM_STAGGER="store,gelu" in units of 8128-cycle sleeps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
for v in 0,0 1,1 2,2 3,3 0,0; do
  ROUNDS=3 DTD_GEMM_STAGGER=$v step "stg_${v/,/_}" 400 python -u scripts/bench_gemm8.py
done
echo done
