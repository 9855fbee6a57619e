#!/usr/bin/env bash
# GEMM split-buffer form ([A0|A1|B0|B1] LDS, K loop unrolled by two, branch-free staging):
# tests under it, timings vs v1 and hipBLASLt (plain + fused epilogues), whole-step A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step gemm_tests_split 400 env DTD_GEMM_VARIANT=2 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread
step bench_split 600 env VNEW=2 ROUNDS=5 python scripts/bench_gemm_v2.py
step gemm8_v1 600 python scripts/bench_gemm8.py
step gemm8_split 600 env DTD_GEMM_VARIANT=2 python scripts/bench_gemm8.py
step ab 900 python scripts/ab.py base gemm_split --rounds 3
echo done
