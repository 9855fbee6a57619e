#!/usr/bin/env bash
# Non-blocking idle-time collection: naive MP / GPipe on 2 stages of one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step pytest_par 300 python -u -m pytest tests/test_parallel_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step mp_base 300 python model_parallel_training.py --devices cuda:0,cuda:0 --training-steps 30
step gpipe_base 300 python model_parallel_training.py --devices cuda:0,cuda:0 --training-steps 30 --pipeline
step mp_large 300 python model_parallel_training.py --model bert-large-cased --devices cuda:0,cuda:0 --training-steps 20
step gpipe_large 300 python model_parallel_training.py --model bert-large-cased --devices cuda:0,cuda:0 --training-steps 20 --pipeline
step prof_mp 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mp2 -o run --output-format csv -- python model_parallel_training.py --devices cuda:0,cuda:0 --training-steps 10
echo done
