#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
step pytest_async 600 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread -k "async or loss_decreases"
step ab 600 python scripts/ab.py base async_wgrad --rounds 3
echo done
