#!/usr/bin/env bash
# Round-2 numbers for the other BASELINE.json configs that fit one MI355X, through bench.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step cfg_bert_base_zero2 300 python bench.py --zero-stage 2 --steps 10 --warmup 3
step cfg_bert_large_ddp 300 python bench.py --model large --batch-size 64 --steps 10 --warmup 3
step cfg_gpt2m_ddp 300 python bench.py --model gpt2-medium --batch-size 32 --steps 10 --warmup 3
step cfg_gpt2m_zero3 300 python bench.py --model gpt2-medium --zero-stage 3 --batch-size 32 --steps 10 --warmup 3
step cfg_bert_large_mp2 300 python model_parallel_training.py --model large --devices cuda:0,cuda:0 --batch-size 16 --training-steps 30
echo done
