#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
DTD_ATTN_OCC=4,2,2 step pytest_attn_ring1 600 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread
B=128 step bench_attn 300 python scripts/bench_attn.py 2,2,2 4,2,2 3,2,2 2,2,2 4,2,2
B=128 P=0 step bench_attn_nodrop 300 python scripts/bench_attn.py 2,2,2 4,2,2
echo done
