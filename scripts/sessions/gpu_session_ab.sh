#!/usr/bin/env bash
# Same-box A/B: attention restructure (tests + micro-bench), tuned vs untuned GEMM table at b64/b128.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
step build 300 python -c "import __graft_entry__ as g; g.build()"
step pytest_attn 600 python -m pytest tests/test_attention_gpu.py tests/test_model_gpu.py -q -x
step bench_attn 300 python scripts/bench_attn.py 3,2,3 2,2,2 2,2,3
DTD_ATTN_DKDV_BM=64 step bench_attn_bm64 300 python scripts/bench_attn.py 3,2,3 2,2,3
step pytest_gpu 900 python -m pytest tests -m gpu -q -x
step b64_tuned 300 python bench.py --batch-size 64
step b64_untuned 300 python bench.py --batch-size 64 --no-tuned-gemms
step b128_tuned 300 python bench.py --batch-size 128 --steps 10 --warmup 3
step b128_untuned 300 python bench.py --batch-size 128 --steps 10 --warmup 3 --no-tuned-gemms
step b64_tuned_again 300 python bench.py --batch-size 64
echo done
