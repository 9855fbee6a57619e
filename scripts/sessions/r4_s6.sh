#!/usr/bin/env bash
# Round 4 session 6: same-box A/B of the whole step -- base_so = the tree before the dK/dV dropout
# dS' rewrite (ops/_dtd_kernels_base.so), GEMM start stagger, fused attention backward.
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step ab 900 python scripts/ab.py base base_so gemm_stagger4 attn_bwd_fused --rounds 3
step attn_ab 200 env B=256 python scripts/bench_attn.py 3,2,3 3,2,3
echo done
