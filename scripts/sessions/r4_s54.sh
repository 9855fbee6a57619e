#!/usr/bin/env bash
# Round 4 session 54: final check after the prewarm's empty_cache -- N>1-path bench, the ZeRO /
# DDP script tests that create RCCL groups
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step fc 200 python bench.py --force-collectives
step tests 600 python -u -m pytest tests/test_graph_gpu.py tests/test_parallel_gpu.py -q -x --timeout 180 --timeout-method thread
step bench 200 python bench.py
echo done
