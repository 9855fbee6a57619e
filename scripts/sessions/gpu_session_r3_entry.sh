#!/usr/bin/env bash
# Round-3 entry check: GPU test suite, smoke, default bench, kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 300 python bench.py
step prof_default 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default -o run --output-format csv -- python bench.py --steps 5 --warmup 2
step gemm8 400 python scripts/bench_gemm8.py
echo done
