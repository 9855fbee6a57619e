#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
DTD_ATTN_TILE=32,64 step pytest_attn_bn32 600 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread
B=128 step bench_attn 300 python scripts/bench_attn.py 3,2,3 3,2,3
B=128 DTD_ATTN_TILE=32,64 step bench_attn_bn32 300 python scripts/bench_attn.py 3,2,3 3,2,3
echo done
