#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
step build 300 python -c "import __graft_entry__ as g; g.build()"
step pytest_gpu 900 python -m pytest tests -m gpu -q
step bench_b32 300 python bench.py --steps 10 --warmup 3 --batch-size 32
step zero_bloom_s0 300 python zero_dp_training.py --stage 0 --training-steps 10 --no-memstats --quiet
step zero_bloom_s3 300 python zero_dp_training.py --stage 3 --training-steps 10 --quiet
step mp_naive 300 python model_parallel_training.py --devices cuda:0,cuda:0 --training-steps 10
step mp_pipe 300 python model_parallel_training.py --devices cuda:0,cuda:0 --pipeline --training-steps 10
step est_w4 300 python estimate_transformer_memory.py --mi355x-report
echo done
