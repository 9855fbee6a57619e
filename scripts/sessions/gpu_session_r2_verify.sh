#!/usr/bin/env bash
# Full verification: GPU tests, smoke(), default bench, kernel stats of the default step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q "failed" gpurun_out/pytest_gpu.log || exit 1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench_default 300 python bench.py
step prof_default 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default -o run --output-format csv -- python bench.py --steps 5 --warmup 2
echo done
