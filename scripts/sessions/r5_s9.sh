#!/usr/bin/env bash
# Round 5 session 9: fused projection + LayerNorm kernel (gemm_ln.hip) re-measured with LDS-DMA in
# inline asm (no compiler vmcnt(0) drains), standalone and whole step
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step bench_gemm_ln_p1 300 python -u scripts/bench_gemm_ln.py 131072 7
DTD_GEMM_LN_PIPE=0 step bench_gemm_ln_p0 300 python -u scripts/bench_gemm_ln.py 131072 7
step ab_gemm_ln 900 python -u scripts/ab.py base gemm_ln gemm_ln_p0 --rounds 3
echo done
