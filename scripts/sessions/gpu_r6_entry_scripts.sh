#!/usr/bin/env bash
# Round 6 closing: every reference entry point on the GPU box once (the reference's CLI surface).
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
MASTER_PORT=29811 step ep_ddp_b4 300 python data_parallel_training.py --training-steps 50 --quiet
MASTER_PORT=29812 step ep_zero2 300 python zero_dp_training.py --stage 2 --training-steps 30 --quiet --no-memstats
MASTER_PORT=29813 step ep_zero3_eager 300 python zero_dp_training.py --stage 3 --graph off --training-steps 10 --quiet
step ep_mp 300 python model_parallel_training.py --training-steps 20
step ep_gpipe 300 python model_parallel_training.py --pipeline --training-steps 20
step ep_allreduce 300 python pytorch_allreduce.py --world-size 2 --backend gloo
step ep_est_nn 120 python estimate_nn_memory.py
step ep_est_tf 120 python estimate_transformer_memory.py
step ep_fp32 300 python bench.py --dtype fp32 --batch-size 32 --steps 10 --warmup 3
echo done
