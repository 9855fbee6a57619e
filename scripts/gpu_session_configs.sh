#!/usr/bin/env bash
# One measured number per BASELINE.json config that fits one MI355X (multi-GPU ones at world 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source scripts/gpu_step.sh
step cfg_bert_large_ddp 300 python bench.py --model large --batch-size 64 --steps 10 --warmup 3
step cfg_bert_large_mp2 300 python model_parallel_training.py --model large --devices cuda:0,cuda:0 --batch-size 16 --training-steps 30
step cfg_bert_large_gpipe2 300 python model_parallel_training.py --model large --devices cuda:0,cuda:0 --batch-size 16 --training-steps 30 --pipeline --micro-batch-count 4
step cfg_bert_base_zero2 300 python zero_dp_training.py --model-name bert-base-cased --stage 2 --batch-size 32 --training-steps 30 --quiet --no-memstats
step cfg_gpt2m_zero3 300 python zero_dp_training.py --model-name gpt2-medium --stage 3 --batch-size 16 --training-steps 30 --quiet --no-memstats
echo done
