#!/usr/bin/env bash
# Naive MP (2 stages on one GPU, BERT-base b16): where does the step time go?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step mp_naive 300 python model_parallel_training.py --devices cuda:0,cuda:0 --training-steps 30
step prof_mp 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mp -o run --output-format csv -- python model_parallel_training.py --devices cuda:0,cuda:0 --training-steps 10
echo done
