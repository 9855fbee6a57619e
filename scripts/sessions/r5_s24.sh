#!/usr/bin/env bash
# Round 5 session 24: bisect the captured-DDP replay segfault (s22/s23): same test subset with the
# ZeRO capture deferral off, then the DDP case alone
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
DTD_ZERO_CAPTURE_DEFER=0 step graph_nodefer 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_graph_gpu.py -k "rccl or zero"
step ddp_alone 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_graph_gpu.py -k "rccl_collectives"
echo done
