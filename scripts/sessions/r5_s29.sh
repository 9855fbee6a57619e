#!/usr/bin/env bash
# Round 5 session 29: weight-gradient GEMMs on a second stream (--async-wgrad) now that they run on
# wgrad.hip (round 4: 5-9x slower with hipBLASLt's stream-K kernels)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step ab_async 600 python -u scripts/ab.py base async_wgrad --rounds 3
echo done
