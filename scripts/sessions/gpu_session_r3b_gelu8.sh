#!/usr/bin/env bash
# fc1 + GELU + GELU' epilogue computed stage by stage over 8 values (no hazard s_nops): GEMM tests,
# bench_gemm8 new vs base build, whole-step A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
OPS=$PWD/distributed_training_and_deepspeed_amd/ops
step pytest_gemm 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread
step gemm8_new 300 python -u scripts/bench_gemm8.py
step gemm8_base 300 env DTD_KERNELS_SO=$OPS/_dtd_kernels_base.so python -u scripts/bench_gemm8.py
step ab 900 python -u scripts/ab.py base_so base --rounds 3 -- --steps 12 --warmup 4
echo done
