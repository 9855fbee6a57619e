#!/usr/bin/env bash
# W4R latency probe: the register-staged 4-wave GEMM with its loads re-reading K-step 0 (L2-hot,
# timing only) vs the real staging.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
OPS=$PWD/distributed_training_and_deepspeed_amd/ops
step w4r_real 400 env VNEW=4 DTD_KERNELS_SO=$OPS/_dtd_kernels_w4r0.so python -u scripts/bench_gemm_v2.py
step w4r_hot 400 env VNEW=4 DTD_KERNELS_SO=$OPS/_dtd_kernels_w4r1.so python -u scripts/bench_gemm_v2.py
echo done
