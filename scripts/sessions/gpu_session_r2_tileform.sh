#!/usr/bin/env bash
# persistent vs one-tile-per-workgroup GEMM form on the store-heavy fused FFN epilogues.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
ROUNDS=3 step g_pers 600 python -u scripts/bench_gemm8.py
ROUNDS=3 DTD_GEMM_VARIANT=0 step g_tile 600 python -u scripts/bench_gemm8.py
step ab 900 python -u scripts/ab.py base gemm_tile --rounds 3
echo done
