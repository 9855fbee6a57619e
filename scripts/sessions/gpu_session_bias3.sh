#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
step pytest_attn 600 python -u -m pytest tests/test_attention_gpu.py tests/test_model_gpu.py tests/test_graph_gpu.py -x -q --timeout 120 --timeout-method thread
DBIAS=0 step bench_attn_nobias 300 python scripts/bench_attn.py 2,2,2
DBIAS=1 step bench_attn_bias 300 python scripts/bench_attn.py 2,2,2
step bench_default 300 python bench.py
step bench_default2 300 python bench.py
echo done
