#!/usr/bin/env bash
# Staged Adam overlapped with the next forward: bit-identity test + whole-step A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step t_overlap 300 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread
step ab 900 python scripts/ab.py opt_overlap_off base --rounds ${ROUNDS:-4} -- --steps 12 --warmup 4
echo done
