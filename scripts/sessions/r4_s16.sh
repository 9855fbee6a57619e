#!/usr/bin/env bash
# Round 4 session 16: more split-K slices for the weight-gradient GEMMs (16 -> 32 / 64)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step ab_wgrad 900 python scripts/ab.py base wgrad_s32 wgrad_s64 --rounds 3
echo done
