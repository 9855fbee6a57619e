#!/usr/bin/env bash
# Round 4 session 13: captured ZeRO-2/3 steps with RCCL collectives vs eager; DDP RCCL + optimizer
# overlap vs the local path
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step tests_rccl 600 python -u -m pytest -v --timeout 180 --timeout-method thread tests/test_graph_gpu.py tests/test_parallel_gpu.py -k "rccl or share_one_gpu"
echo done
