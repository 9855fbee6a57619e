#!/usr/bin/env bash
# Round 5 session 27: captured RCCL cases in fresh processes; ZeRO capture deferral on; graph +
# parallel GPU tests
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step graph_subset 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_graph_gpu.py -k "rccl or zero"
step graph_par 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_graph_gpu.py tests/test_parallel_gpu.py
echo done
