#!/usr/bin/env bash
# Round 5 session 39: TunableOp rows for the per-GPU batch 512 GEMM shapes, merged into the table;
# b256 vs b512 on the merged table
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_b512_%d.csv \
  step tune_b512 600 python -u bench.py --batch-size 512 --steps 2 --warmup 1 --no-tuned-gemms
python scripts/merge_tunable.py distributed_training_and_deepspeed_amd/tuning/tunableop_mi355x.csv gpurun_out/tunableop_b512_0.csv gpurun_out/tunableop_merged.csv
DTD_TUNED_TABLE=$PWD/gpurun_out/tunableop_merged.csv step m256 300 python -u bench.py --steps 10 --warmup 3
DTD_TUNED_TABLE=$PWD/gpurun_out/tunableop_merged.csv step m512 300 python -u bench.py --steps 10 --warmup 3 --batch-size 512
step o512 300 python -u bench.py --steps 10 --warmup 3 --batch-size 512
echo done
