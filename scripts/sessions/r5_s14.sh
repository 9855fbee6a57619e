#!/usr/bin/env bash
# Round 5 session 14: stage-per-process pipeline on the GPU (2 ranks share cuda:0 over gloo)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step stage_pipe 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_stage_pipeline_gpu.py tests/test_graph_gpu.py -k "stage or model_parallel"
echo done
