#!/usr/bin/env bash
# Batched NT-operand transposes at the start of the backward: full GPU suite, then whole-step A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
rm -f gpurun_out/session.log
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
step ab 800 python -u scripts/ab.py base wt_batch_off --rounds 3
echo done
