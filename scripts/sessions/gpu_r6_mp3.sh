#!/bin/bash
# Round 6: the max-params ZeRO-3 step (largest 1-GPU model) on the current engine: plain timing run,
# then the same under a kernel trace.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
timeout -k 10 500 python -u bench/max_params.py --measure --stage 3 --steps 4 > gpurun_out/r6_mp3_plain.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r6_mp3 -o run -- \
  python bench/max_params.py --measure --stage 3 --steps 2 > gpurun_out/r6_mp3_prof.log 2>&1
echo "prof_rc=$?" >> gpurun_out/r6_mp3_prof.log
