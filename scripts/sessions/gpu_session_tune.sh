#!/usr/bin/env bash
# Extend the TunableOp (hipBLASLt/rocBLAS) solution table with the b64 / b128 GEMM shapes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
step build 300 python -c "import __graft_entry__ as g; g.build()"
cp distributed_training_and_deepspeed_amd/tuning/tunableop_mi355x.csv gpurun_out/tune0.csv
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune%d.csv
step tune_b64 1000 python bench.py --steps 2 --warmup 1 --batch-size 64
step tune_b128 1000 python bench.py --steps 2 --warmup 1 --batch-size 128
export PYTORCH_TUNABLEOP_TUNING=0
step tuned_b64 300 python bench.py --batch-size 64
step tuned_b128 300 python bench.py --batch-size 128 --steps 10 --warmup 3
echo done
