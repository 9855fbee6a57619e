#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step zero_s0_b8 300 python zero_dp_training.py --stage 0 --training-steps 40 --quiet --no-memstats --batch-size 8
step zero_s2_b8 300 python zero_dp_training.py --stage 2 --training-steps 40 --quiet --no-memstats --batch-size 8
step zero_s3_b8 300 python zero_dp_training.py --stage 3 --training-steps 40 --quiet --no-memstats --batch-size 8
step prof_zero_b8 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_zero_b8 -o run --output-format csv -- python zero_dp_training.py --stage 0 --training-steps 10 --quiet --no-memstats --batch-size 8
echo done
