#!/usr/bin/env bash
# Round 5 session 47: TunableOp rows for the b1024 shapes, merged; same-box A/B
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_b1024_%d.csv \
  step tune_b1024 700 python -u bench.py --steps 2 --warmup 1 --no-tuned-gemms
python scripts/merge_tunable.py distributed_training_and_deepspeed_amd/tuning/tunableop_mi355x.csv gpurun_out/tunableop_b1024_0.csv gpurun_out/tunableop_merged1024.csv
step base1 400 python -u bench.py --steps 8 --warmup 3
DTD_TUNED_TABLE=$PWD/gpurun_out/tunableop_merged1024.csv step tuned1 400 python -u bench.py --steps 8 --warmup 3
step base2 400 python -u bench.py --steps 8 --warmup 3
DTD_TUNED_TABLE=$PWD/gpurun_out/tunableop_merged1024.csv step tuned2 400 python -u bench.py --steps 8 --warmup 3
echo done
