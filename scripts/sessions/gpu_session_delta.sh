#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
step pytest_attn 600 python -u -m pytest tests/test_attention_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread
B=128 step bench_attn 300 python scripts/bench_attn.py 3,2,3 3,2,3
step ab 500 python scripts/ab.py base --rounds 3
echo done
