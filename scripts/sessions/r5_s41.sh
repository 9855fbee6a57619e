#!/usr/bin/env bash
# Round 5 session 41: full GPU suite on the current tree; b512 kernel budget
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step gpu_suite 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s41 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2
python scripts/prof_summary.py gpurun_out/prof_s41/run_kernel_stats.csv 7 40 > gpurun_out/r5_s41_kernel_summary.txt 2>&1
echo done
