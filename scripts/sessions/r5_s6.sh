#!/usr/bin/env bash
# Round 5 session 6: wgrad.hip limiter probe (timing-only diag builds: no DMA / no barrier / no reads)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step bench_wgrad_diag 400 env ROUNDS=5 VARIANTS=44,441,442,443,447 python -u scripts/bench_wgrad.py
echo done
