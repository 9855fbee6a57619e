#!/usr/bin/env bash
# Where does the time go in the reference-default ZeRO run (bloom-560m, b1) and in GPipe?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step zero_bloom_default 300 python zero_dp_training.py --training-steps 60 --quiet
step zero_bloom_nomem 300 python zero_dp_training.py --training-steps 60 --quiet --no-memstats
step zero_bloom_s2_nomem 300 python zero_dp_training.py --training-steps 60 --quiet --no-memstats --stage 2
step prof_zero_bloom 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_zero -o run --output-format csv -- python zero_dp_training.py --training-steps 30 --quiet --no-memstats
step gpipe_large 300 python model_parallel_training.py --model bert-large-cased --devices cuda:0,cuda:0 --pipeline --training-steps 20
step prof_gpipe 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gpipe -o run --output-format csv -- python model_parallel_training.py --model bert-large-cased --devices cuda:0,cuda:0 --pipeline --training-steps 10
echo done
