#!/usr/bin/env bash
# Round 5 session 20: Adam per-element math with contraction off (staged == single launch), then the
# full GPU suite
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step staged_diff 300 env REPEAT=1 python -u scripts/diag/staged_adam_diff.py
step gpu_suite 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
echo done
