#!/usr/bin/env bash
# Deferred GELU-forward activation in the persistent GEMM: GEMM tests + fc1 GELU rows, defer off / on.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step tests 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/tests.log && ! grep -q "failed" gpurun_out/tests.log || exit 1
DTD_GEMM_DEFER=0 ROUNDS=3 step gemm_defer0 600 python -u scripts/bench_gemm8.py
DTD_GEMM_DEFER=1 ROUNDS=3 step gemm_defer1 600 python -u scripts/bench_gemm8.py
echo done
