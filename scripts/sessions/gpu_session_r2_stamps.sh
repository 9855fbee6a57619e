#!/usr/bin/env bash
# In-kernel stamps of the GEMM tile (tile form and persistent form).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
DTD_GEMM_VARIANT=0 step stamps_t 200 python -u scripts/gemm_stamps.py
DTD_GEMM_VARIANT=1 step stamps_p 200 python -u scripts/gemm_stamps.py
echo done
