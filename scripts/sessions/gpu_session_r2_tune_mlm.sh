#!/usr/bin/env bash
# Extend the TunableOp table with the static-capacity MLM-head shapes of the b256 bench step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
cp distributed_training_and_deepspeed_amd/tuning/tunableop_mi355x.csv gpurun_out/tune0.csv
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune%d.csv
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=200
step tune 900 python bench.py --steps 2 --warmup 1
echo done
