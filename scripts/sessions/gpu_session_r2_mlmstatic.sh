#!/usr/bin/env bash
# static-capacity sparse MLM head in eager mode (fixed GEMM M, no nonzero() host sync) vs dynamic.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step ab 900 python -u scripts/ab.py base mlm_dynamic --rounds 4
echo done
