#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
step wgrad_sweep 300 python scripts/wgrad_sweep.py
step wgrad_tune 900 python scripts/wgrad_sweep.py --tune
echo done
