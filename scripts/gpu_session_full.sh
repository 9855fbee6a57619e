#!/usr/bin/env bash
# Full GPU test suite + default bench x2 (+ optional rocprof kernel stats).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench_default 300 python bench.py
step bench_default2 300 python bench.py
if [ -n "$PROF" ]; then
  step prof_default 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default -o run --output-format csv -- python bench.py --steps 5 --warmup 2
fi
echo done
