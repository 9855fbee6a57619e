#!/bin/bash
# Round 6: TunableOp rows for the b1024 step's hipBLASLt shapes (fc2 forward, fc1 input gradient,
# qkv residual-add input gradient, MLM decoder at 524288 tokens), one tuning step.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=30 \
PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tun_b1024%d.csv \
  timeout -k 10 900 python -u bench.py --steps 1 --warmup 1 > gpurun_out/tun_b1024.log 2>&1
