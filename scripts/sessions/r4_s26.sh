#!/usr/bin/env bash
# Round 4 session 26: which interaction makes the async weight-gradient stream 5x slower
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step async_nooverlap 240 python bench.py --async-wgrad on --opt-overlap off --steps 10 --warmup 3
DTD_DEFER_FINALIZE=0 step async_nodefer 240 python bench.py --async-wgrad on --steps 10 --warmup 3
DTD_DEFER_FINALIZE=0 step async_neither 240 python bench.py --async-wgrad on --opt-overlap off --steps 10 --warmup 3
step async_hiptrace 300 rocprofv3 --hip-trace --kernel-trace --stats -d gpurun_out/async_prof -o run --output-format csv -- python bench.py --async-wgrad on --steps 3 --warmup 2
echo done
