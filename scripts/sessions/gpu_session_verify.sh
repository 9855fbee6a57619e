#!/usr/bin/env bash
# Re-entry verification: GPU tests, attention micro-bench, default + b32 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
step bench_attn 300 python scripts/bench_attn.py 2,2,2 3,2,3
step bench_default 300 python bench.py
step bench_b32 300 python bench.py --batch-size 32
echo done
