#!/usr/bin/env bash
# Round 5 session 28: RCCL watchdog drained before capture: captured RCCL cases in fresh processes,
# then in-process after the captured ZeRO tests (the s22-s26 ordering)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp

DTD_RCCL_CAPTURE_INPROC=1 step graph_inproc 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_graph_gpu.py -k "rccl or zero"
echo done
