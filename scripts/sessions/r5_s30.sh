#!/usr/bin/env bash
# Round 5 session 30: why --async-wgrad is 9x slower (GPU idle): HIP API + kernel trace of 2 steps
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step prof_async 300 rocprofv3 --hip-trace --kernel-trace --stats -d gpurun_out/prof_async -o run --output-format csv -- python3 bench.py --async-wgrad on --steps 2 --warmup 1
echo done
