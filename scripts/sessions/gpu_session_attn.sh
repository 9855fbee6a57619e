#!/usr/bin/env bash
# Attention occupancy sweep + GPU tests + bench + profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
step build 300 python -c "import __graft_entry__ as g; g.build()"
step pytest_gpu 900 python -m pytest tests -m gpu -q -x
step bench_attn 300 python scripts/bench_attn.py 1,1,1 2,2,2 3,2,2 3,2,3 2,1,2
step bench_b32 300 python bench.py --steps 10 --warmup 3 --batch-size 32
export TMPDIR=/tmp
step rocprof_b32 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b32 -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --batch-size 32
echo done
