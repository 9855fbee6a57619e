#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
DTD_GEMM_BN=256 step g_base 300 python scripts/bench_gemm_fused.py
DTD_GEMM_BN=256 DTD_GEMM_DIAG=1 step g_nodma 300 python scripts/bench_gemm_fused.py
DTD_GEMM_BN=256 DTD_GEMM_DIAG=2 step g_prio 300 python scripts/bench_gemm_fused.py
echo done
