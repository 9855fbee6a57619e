#!/usr/bin/env bash
# Round-3 checkpoint: full GPU test suite, smoke, default + ZeRO-2 bench, kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 300 python bench.py
step bench_zero2 300 python bench.py --zero-stage 2
step prof_default 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default -o run --output-format csv -- python bench.py --steps 5 --warmup 2
step prof_summary 60 python scripts/prof_summary.py gpurun_out/prof_default/run_kernel_stats.csv 7 40
echo done
