#!/usr/bin/env bash
# Round 5 session 22: collectives issued on the capturing stream with deferred waits (ZeRO's
# captured-step form); captured DDP / ZeRO-2 / ZeRO-3 steps vs eager; ZeRO GPU tests
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step cap_deferred 200 python -u scripts/diag/capture_collectives.py origin_deferred_wait reduce_scatter_async_wait
step graph_tests 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_graph_gpu.py -k "rccl or zero"
step zero_tests 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_parallel_gpu.py
echo done
