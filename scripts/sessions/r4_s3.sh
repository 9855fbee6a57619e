#!/usr/bin/env bash
# Round 4 session 3: multi-GPU rehearsal of the shaped tail buckets (A/B), dense-MLM-head bench row,
# ZeRO-2 with real RCCL collectives, full GPU test suite.
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step n8_tail 400 env OCC=0,32 BUSBW=150,300 STEPS=8 WARM=3 python scripts/n8_rehearsal.py
step n8_notail 400 env DTD_DDP_TAIL_BUCKET_MB=0 OCC=0,32 BUSBW=150,300 STEPS=8 WARM=3 python scripts/n8_rehearsal.py
step bench_dense_head 300 python bench.py --dense-mlm-head
step bench_zero2_force 300 python bench.py --zero-stage 2 --force-collectives
step prof_fp32 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fp32 -o run --output-format csv -- python bench.py --dtype fp32 --batch-size 32 --steps 3 --warmup 2
step mp_large_graph 300 python model_parallel_training.py --model bert-large-cased --devices cuda:0,cuda:0 --batch-size 16 --training-steps 40 --graph on
step gpipe_large_graph 300 python model_parallel_training.py --model bert-large-cased --devices cuda:0,cuda:0 --batch-size 16 --training-steps 40 --pipeline --graph on
step gpipe_large_eager 300 python model_parallel_training.py --model bert-large-cased --devices cuda:0,cuda:0 --batch-size 16 --training-steps 40 --pipeline --graph off
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread
echo done
