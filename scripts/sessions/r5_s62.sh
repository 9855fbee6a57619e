#!/usr/bin/env bash
# Round 5 session 62: at the b1024 default the library GEMMs are power-held at 1.74-1.81 GHz while
# the hand-written persistent kernels hold 1.93-2.00 -- does the all-native GEMM mode (DTD_GEMM_ALL=1:
# plain forward / input-gradient products on gemm_bt; 2.9 % slower at b256) win there?  3 rounds
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
for r in 1 2 3; do
  step base_$r 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
  step allnative_$r 400 env DTD_GEMM_ALL=1 python -u bench.py --gpus 1 --steps 20 --warmup 5
done
echo done
