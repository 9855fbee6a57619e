#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
DTD_ATTN_OCC=3,2,3 DTD_ATTN_TILE=64,64 step pytest_attn_ring1 600 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread
B=128 step bench_attn_dq128 300 python scripts/bench_attn.py 3,2,2 3,2,2
B=128 DTD_ATTN_TILE=64,64 step bench_attn_dq64 300 python scripts/bench_attn.py 3,2,3 3,2,2 3,2,3
echo done
