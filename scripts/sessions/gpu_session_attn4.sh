#!/usr/bin/env bash
# Attention softmax changes: permlane32 swaps, defer-max, keep-word shift -> tests + timing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
step pytest_attn 600 python -u -m pytest tests/test_attention_gpu.py tests/test_model_gpu.py -x -v --timeout 120 --timeout-method thread
step bench_attn 300 python scripts/bench_attn.py 2,2,2 3,2,3
P=0.0 step bench_attn_nodrop 300 python scripts/bench_attn.py 2,2,2 3,2,3
step bench_default 300 python bench.py
echo done
