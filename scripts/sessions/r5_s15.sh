#!/usr/bin/env bash
# Round 5 session 15: stage-per-process entry script on one GPU (gloo), full log
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step mp_sp_fp32 200 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 model_parallel_training.py --model bert-tiny --batch-size 8 --training-steps 5 --seq-len 64 --pipeline --micro-batch-count 4 --schedule 1f1b --pipe-backend gloo --dtype fp32
step mp_sp_bf16 200 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 model_parallel_training.py --model bert-tiny --batch-size 8 --training-steps 5 --seq-len 64 --pipeline --micro-batch-count 4 --schedule gpipe --pipe-backend gloo
echo done
