#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
step build 300 python -c "import __graft_entry__ as g; g.build()"
step pytest_attn 600 python -m pytest tests/test_attention_gpu.py tests/test_model_gpu.py -q -x
step bench_attn 300 python scripts/bench_attn.py 2,2,2 3,2,3 2,2,3 2,2,2
P=0.0 step bench_attn_nodrop 300 python scripts/bench_attn.py 2,2,2 3,2,3
step pytest_gpu 900 python -m pytest tests -m gpu -q -x
step bench_default 300 python bench.py
step bench_b32 300 python bench.py --batch-size 32
echo done
