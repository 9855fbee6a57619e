#!/usr/bin/env bash
# ZeRO trainer (bloom-560m, b1 and b8) timing + kernel profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step zero_s0_b1 300 python zero_dp_training.py --stage 0 --training-steps 30 --quiet
step zero_s0_b1_nomem 300 python zero_dp_training.py --stage 0 --training-steps 30 --quiet --no-memstats
step zero_s3_b1 300 python zero_dp_training.py --stage 3 --training-steps 30 --quiet --no-memstats
step zero_s0_b8 300 python zero_dp_training.py --stage 0 --training-steps 30 --quiet --no-memstats --batch-size 8
step zero_s0_b1_ref 300 python zero_dp_training.py --stage 0 --training-steps 30 --quiet --no-memstats --impl reference
step prof_zero_s0 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_zero -o run --output-format csv -- python zero_dp_training.py --stage 0 --training-steps 10 --quiet --no-memstats
step prof_zero_s3 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_zero3 -o run --output-format csv -- python zero_dp_training.py --stage 3 --training-steps 10 --quiet --no-memstats
echo done
