#!/usr/bin/env bash
# Round 5 session 3: LDS-DMA as inline asm (no compiler vmcnt(0) drains) in the GEMM kernels +
# weight gradients on wgrad.hip by default -- numerics, per-shape GEMM A/B, whole-step A/B,
# kernel summary, full GPU suite
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step tests_gemm 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_gemm_ln_gpu.py
step gemm8_asm 300 env ROUNDS=5 python -u scripts/bench_gemm8.py
step gemm8_builtin 300 env ROUNDS=5 DTD_KERNELS_SO=$PWD/distributed_training_and_deepspeed_amd/ops/_dtd_kernels_dmabuiltin.so python -u scripts/bench_gemm8.py
step ab_step 900 python -u scripts/ab.py base no_wgrad2 dmabuiltin_so --rounds 3
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s3 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2
python scripts/prof_summary.py gpurun_out/prof_s3/run_kernel_stats.csv 7 40 > gpurun_out/r5_s3_kernel_summary.txt 2>&1
step gpu_suite 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
echo done
