#!/usr/bin/env bash
# Round-3 re-entry: GEMM epilogue change (peeled K-step 0, packed bf16 conversion, swap-free LDS
# image) -- GEMM tests, GEMM micro-bench new vs base build, full GPU suite, smoke, bench, whole-step
# A/B against the base build (ops/_dtd_kernels_base.so = previous commit's kernels).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
BASE=$PWD/distributed_training_and_deepspeed_amd/ops/_dtd_kernels_base.so
step pytest_gemm 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread
step gemm8_new 300 python -u scripts/bench_gemm8.py
step gemm8_base 300 env DTD_KERNELS_SO=$BASE python -u scripts/bench_gemm8.py
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 300 python bench.py
step ab 900 python -u scripts/ab.py base_so base --rounds 3 -- --steps 12 --warmup 4
echo done
