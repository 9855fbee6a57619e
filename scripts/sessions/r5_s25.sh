#!/usr/bin/env bash
# Round 5 session 25: comm.destroy() releases the graphs captured with its group first; the s22-s24
# subset (captured ZeRO steps then captured DDP with RCCL) with the ZeRO capture deferral on
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step graph_subset 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_graph_gpu.py -k "rccl or zero"
step graph_all 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_graph_gpu.py tests/test_parallel_gpu.py
echo done
