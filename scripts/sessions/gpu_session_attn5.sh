#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
step pytest_attn 600 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread
step bench_attn 300 python scripts/bench_attn.py 2,2,2 3,2,3
P=0.0 step bench_attn_nodrop 300 python scripts/bench_attn.py 2,2,2 3,2,3
echo done
