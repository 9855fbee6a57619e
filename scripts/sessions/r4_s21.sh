#!/usr/bin/env bash
# Round 4 session 21: the attention keep-mask generator's side stream restricted to a CU subset
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step ab_maskcu 1000 python scripts/ab.py base mask_cu_half mask_cu_quarter mask_cu_3q --rounds 3
echo done
