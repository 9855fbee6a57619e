#!/usr/bin/env bash
# Input-gradient GEMMs in the NT form (F.linear(dY, W^T)): model tests, whole-step A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step model_tests 600 python -u -m pytest tests/test_model_gpu.py tests/test_graph_gpu.py -x -q --timeout 120 --timeout-method thread
step ab 1000 python scripts/ab.py base dgrad_nn dkdv_bm64 --rounds 3
echo done
