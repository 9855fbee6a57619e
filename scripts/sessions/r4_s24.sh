#!/usr/bin/env bash
# Round 4 session 24: the other BASELINE configs on the round-4 tree
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step cfg_bert_base_zero2 300 python bench.py --zero-stage 2 --steps 10 --warmup 3
step cfg_bert_large_ddp 300 python bench.py --model large --batch-size 64 --steps 10 --warmup 3
step cfg_gpt2m_ddp 300 python bench.py --model gpt2-medium --batch-size 32 --steps 10 --warmup 3
step cfg_gpt2m_zero3 300 python bench.py --model gpt2-medium --zero-stage 3 --batch-size 32 --steps 10 --warmup 3
step cfg_opt125m_ddp 300 python bench.py --model opt-125m --batch-size 32 --steps 10 --warmup 3
step cfg_bert_base_b32 300 python bench.py --batch-size 32 --steps 20 --warmup 5
step cfg_bert_base_b4_graph 300 python bench.py --batch-size 4 --graph on --steps 50 --warmup 10
echo done
