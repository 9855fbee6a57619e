#!/bin/bash
# Round 6: TunableOp tables for the reference's own default configurations (bloom-560m ZeRO b1 and
# BERT-base DDP b4: their small-M GEMM shapes are not in the bench table), eager steps with tuning on.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=20
MASTER_PORT=29931 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tun_bloom%d.csv \
  timeout -k 10 500 python zero_dp_training.py --stage 3 --graph off --training-steps 3 --quiet --no-memstats > gpurun_out/tun_bloom.log 2>&1 || exit 1
MASTER_PORT=29932 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tun_ddp_b4%d.csv \
  timeout -k 10 500 python data_parallel_training.py --batch-size 4 --training-steps 3 --graph off --quiet > gpurun_out/tun_ddp_b4.log 2>&1
