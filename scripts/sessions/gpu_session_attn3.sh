#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
step build 300 python -c "import __graft_entry__ as g; g.build()"
step pytest_attn 600 python -m pytest tests/test_attention_gpu.py -q -x
DTD_ATTN_DKDV_BM=64 step attn_bm64 300 python scripts/bench_attn.py 3,2,3
DTD_ATTN_DKDV_BM=128 step attn_bm128 300 python scripts/bench_attn.py 3,2,3
DTD_ATTN_DKDV_BM=128 DTD_ATTN_TILE=64,128 step attn_dq128 300 python scripts/bench_attn.py 3,2,3
DTD_ATTN_DKDV_BM=128 DTD_ATTN_TILE=128,128 step attn_all128 300 python scripts/bench_attn.py 3,2,3
DTD_ATTN_DKDV_BM=64 step attn_bm64_again 300 python scripts/bench_attn.py 3,2,3
DTD_ATTN_DKDV_BM=128 DTD_ATTN_TILE=128,128 step pytest_attn_128 600 python -m pytest tests/test_attention_gpu.py -q -x
echo done
