#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step pytest_k 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread
step prof_b128 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_embed -o run --output-format csv -- python bench.py --steps 5 --warmup 2
echo done
