#!/usr/bin/env bash
# Extend the TunableOp table with the b128 shapes of the current step (split-K 16 x 4096 slices).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
cp distributed_training_and_deepspeed_amd/tuning/tunableop_mi355x.csv gpurun_out/tune0.csv
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune%d.csv
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=100
step tune_b128 1000 python bench.py --steps 2 --warmup 1 --batch-size 128
echo done
