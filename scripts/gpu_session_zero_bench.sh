#!/usr/bin/env bash
# BASELINE configs 4/5 through bench.py's timing contract on one GPU: BERT-base ZeRO-2 and
# GPT-2-medium ZeRO-3 (plus DDP at the same shapes for the engine overhead).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source scripts/gpu_step.sh
step zero2_base_b128 300 python bench.py --zero-stage 2 --steps 10 --warmup 3
step zero1_base_b128 300 python bench.py --zero-stage 1 --steps 10 --warmup 3
step ddp_gpt2m_b32 300 python bench.py --model gpt2-medium --batch-size 32 --steps 10 --warmup 3
step zero3_gpt2m_b32 300 python bench.py --model gpt2-medium --zero-stage 3 --batch-size 32 --steps 10 --warmup 3
echo done
