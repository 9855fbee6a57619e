#!/usr/bin/env bash
# Round 4 session 41: same-process GEMM / copy rates before and after RCCL init
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step clock_ab 200 python scripts/diag/rccl_clock_ab.py
echo done
