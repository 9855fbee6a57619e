#!/usr/bin/env bash
# Attention-dropout mask look-ahead: all layers at forward start (base) vs 1 / 2 layers ahead.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
rm -f gpurun_out/session.log
step model_tests 300 env DTD_MASK_AHEAD=1 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_model_gpu.py tests/test_graph_gpu.py
step ab 1000 python -u scripts/ab.py base mask_ahead1 mask_ahead2 --rounds 3
echo done
