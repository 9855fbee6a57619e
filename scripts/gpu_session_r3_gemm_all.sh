#!/bin/bash
# All-native GEMM mode: parity test, then a same-box A/B of the whole step (default vs DTD_GEMM_ALL=1).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_model_gpu.py -k "all_native or fused_gpu_matches" > gpurun_out/gemm_all_test.log 2>&1 &&
timeout -k 10 600 python -u scripts/ab.py base gemm_all --rounds 2 -- --steps 10 --warmup 5 \
  > gpurun_out/gemm_all_ab.jsonl 2> gpurun_out/gemm_all_ab.err
