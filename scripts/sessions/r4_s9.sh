#!/usr/bin/env bash
# Round 4 session 9: fused projection + LayerNorm kernel -- numerics, then the standalone A/B
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step tests_gemm_ln 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_ln_gpu.py
step bench_gemm_ln 300 python -u scripts/bench_gemm_ln.py 131072 7
echo done
