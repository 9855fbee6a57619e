#!/usr/bin/env bash
# Round 5 session 23: captured ZeRO steps with deferred collective waits, no Work outliving its
# capture; captured DDP / ZeRO steps vs eager; ZeRO GPU tests
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step graph_tests 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_graph_gpu.py -k "rccl or zero"
step zero_tests 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_parallel_gpu.py
echo done
