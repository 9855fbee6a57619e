#!/usr/bin/env bash
# Round 4 session 10: fused projection + LN with weight fragments straight to registers (PIPE 2)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step tests_gemm_ln 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_ln_gpu.py
step bench_gemm_ln_p2 300 python -u scripts/bench_gemm_ln.py 131072 7
DTD_GEMM_LN_PIPE=1 step bench_gemm_ln_p1 300 python -u scripts/bench_gemm_ln.py 131072 7
step ab_gemm_ln 600 python scripts/ab.py base gemm_ln --rounds 2
echo done
