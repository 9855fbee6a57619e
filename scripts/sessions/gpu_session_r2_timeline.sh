#!/usr/bin/env bash
# Kernel timeline of the default bench: GPU idle gaps, exposed side-stream mask generation.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step trace 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o run -- python3 bench.py --steps 6 --warmup 3
f=$(find gpurun_out/tl -name '*kernel_trace.csv' | head -n 1)
python3 scripts/timeline.py "$f" 4 > gpurun_out/timeline.txt 2>&1
cat gpurun_out/timeline.txt
rm -rf gpurun_out/tl
echo done
