#!/usr/bin/env bash
# Build, all GPU tests, default bench (b64) x2, b128, graph b64, rocprof of the default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
step build 300 python -c "import __graft_entry__ as g; g.build()"
step pytest_gpu 900 python -m pytest tests -m gpu -q -x
step bench_default 300 python bench.py
step bench_default2 300 python bench.py
step bench_b128 300 python bench.py --batch-size 128 --steps 10 --warmup 3
step bench_b64_graph 300 python bench.py --graph on
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
export TMPDIR=/tmp
step rocprof_b64 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b64 -o run --output-format csv -- python bench.py --steps 5 --warmup 2
echo done
