#!/usr/bin/env bash
# Round 4 session 3: world-8 rehearsal of the shaped tail buckets (A/B), dense-MLM-head bench row,
# fp32 (reference precision) bench + kernel profile with the hand-written fp32 weight gradients,
# BERT-large model-parallel / GPipe with and without the whole-step hipGraph.
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step n8_tail 300 env OCC=0,32 BUSBW=150,300 STEPS=8 WARM=3 python scripts/n8_rehearsal.py
step n8_notail 300 env DTD_DDP_TAIL_BUCKET_MB=0 OCC=0,32 BUSBW=150,300 STEPS=8 WARM=3 python scripts/n8_rehearsal.py
step bench_dense_head 200 python bench.py --dense-mlm-head
step bench_fp32_b32 200 python bench.py --dtype fp32 --batch-size 32 --steps 5 --warmup 2
step prof_fp32 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fp32 -o run --output-format csv -- python bench.py --dtype fp32 --batch-size 32 --steps 3 --warmup 2
step mp_large_graph 200 python model_parallel_training.py --model bert-large-cased --devices cuda:0,cuda:0 --batch-size 16 --training-steps 40 --graph on
step mp_large_eager 200 python model_parallel_training.py --model bert-large-cased --devices cuda:0,cuda:0 --batch-size 16 --training-steps 40 --graph off
step gpipe_large_graph 200 python model_parallel_training.py --model bert-large-cased --devices cuda:0,cuda:0 --batch-size 16 --training-steps 40 --pipeline --graph on
step gpipe_large_eager 200 python model_parallel_training.py --model bert-large-cased --devices cuda:0,cuda:0 --batch-size 16 --training-steps 40 --pipeline --graph off
echo done
