#!/usr/bin/env bash
# Kernel tests + fused-GEMM timing (tile-order A/B, quiet and with CUs occupied) for the base build
# vs the tree's build + whole-step A/B of the two builds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
BASE=$PWD/distributed_training_and_deepspeed_amd/ops/_dtd_kernels_base.so
step ktests 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread
step gemm_base 120 env DTD_KERNELS_SO=$BASE OCC=0 python -u scripts/bench_gemm_sched.py
step gemm_new 180 python -u scripts/bench_gemm_sched.py
step ab 900 python scripts/ab.py base_so base --rounds ${ROUNDS:-3} -- --steps 12 --warmup 4
echo done
