#!/usr/bin/env bash
# Round 5 session 31: --async-wgrad slowdown vs step count (2 steps under rocprofv3 ran at 1.43 M)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step async_2 200 python -u bench.py --async-wgrad on --steps 2 --warmup 1
step async_10 200 python -u bench.py --async-wgrad on --steps 10 --warmup 1
step async_20 300 python -u bench.py --async-wgrad on --steps 20 --warmup 5
echo done
