#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench_default 300 python bench.py
step ablate 300 python scripts/ablate_attn_dropout.py
step trace_b128 400 rocprofv3 --kernel-trace -d gpurun_out/trace_b128 -o run --output-format csv -- python bench.py --steps 4 --warmup 3
echo done
