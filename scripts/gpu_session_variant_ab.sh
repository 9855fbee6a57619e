#!/usr/bin/env bash
# Model / kernel GPU tests + whole-step A/B of one ab.py variant against the tree (VARIANT env).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step tests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step ab 900 python scripts/ab.py ${VARIANT:-no_fused_xent} base --rounds ${ROUNDS:-4} -- --steps 12 --warmup 4
echo done
