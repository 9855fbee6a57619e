#!/usr/bin/env bash
# Sparse MLM head: one-pass scatter backward of the labelled-row gather. Tests, then A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
rm -f gpurun_out/session.log
step tests 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_scatter_rows_gpu.py tests/test_model_gpu.py tests/test_graph_gpu.py tests/test_kernels_gpu.py
step ab 800 python -u scripts/ab.py base mlm_scatter_off --rounds 3
echo done
