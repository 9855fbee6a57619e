#!/usr/bin/env bash
# Kernel timeline of the default bench (b128) for gap / overlap analysis (scripts/timeline.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step trace_b128 400 rocprofv3 --kernel-trace -d gpurun_out/trace_b128 -o run --output-format csv -- python bench.py --steps 4 --warmup 3
echo done
