#!/usr/bin/env bash
# Kernel timeline of the default bench step (rocprofv3 kernel trace; scripts/timeline.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step trace 400 rocprofv3 --kernel-trace -d gpurun_out/trace -o run --output-format csv -- python bench.py --steps 6 --warmup 3
echo done
