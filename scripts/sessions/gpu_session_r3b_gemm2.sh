#!/usr/bin/env bash
# GEMM round 3b: NT-form dgrad baselines, no-SLP epilogue build, all-native GEMM A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
OPS=$PWD/distributed_training_and_deepspeed_amd/ops
step gemm8_new 300 python -u scripts/bench_gemm8.py
step gemm8_noslp 300 env DTD_KERNELS_SO=$OPS/_dtd_kernels_noslp.so python -u scripts/bench_gemm8.py
step pytest_allnative 300 python -u -m pytest tests/test_model_gpu.py -x -q -k "all_native" --timeout 200 --timeout-method thread
step ab_all 900 python -u scripts/ab.py base gemm_all --rounds 3 -- --steps 12 --warmup 4
echo done
