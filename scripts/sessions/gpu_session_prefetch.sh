#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
step build 300 python -c "import __graft_entry__ as g; g.build()"
step pytest_gpu 900 python -m pytest tests -m gpu -q -x
step bench_default 300 python bench.py
step bench_default2 300 python bench.py
step bench_b32 300 python bench.py --batch-size 32
export TMPDIR=/tmp
step rocprof_default 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b128 -o run --output-format csv -- python bench.py --steps 5 --warmup 2
echo done
