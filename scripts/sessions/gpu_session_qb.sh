#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
step pytest_attn 600 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread
DTD_ATTN_FWD_QB=2 DTD_ATTN_OCC=1,2,2 step pytest_attn_qb2 600 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread
B=128 step bench_attn_qb1 300 python scripts/bench_attn.py 2,2,2
B=128 DTD_ATTN_FWD_QB=2 step bench_attn_qb2 300 python scripts/bench_attn.py 1,2,2 2,2,2
B=128 P=0 DTD_ATTN_FWD_QB=2 step bench_attn_qb2_nodrop 300 python scripts/bench_attn.py 1,2,2
B=128 P=0 step bench_attn_qb1_nodrop 300 python scripts/bench_attn.py 2,2,2
echo done
