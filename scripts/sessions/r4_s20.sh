#!/usr/bin/env bash
# Round 4 session 20: marginal cost of the side-stream attention keep-mask generator
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step ab_mask 900 python scripts/ab.py base mask_x2 --rounds 3
echo done
