#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
step bench_attn 300 python scripts/bench_attn.py 2,2,2 1,1,1 1,2,1 2,1,2
DTD_ATTN_TILE=128,128 step bench_attn_t128 300 python scripts/bench_attn.py 1,1,1 2,2,2
DTD_ATTN_TILE=128,128 DTD_ATTN_DKDV_BM=64 step bench_attn_t128_bm64 300 python scripts/bench_attn.py 1,1,1
echo done
