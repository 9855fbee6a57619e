#!/usr/bin/env bash
# FFN up-projection stores gelu'(u) (backward epilogue = multiply): GEMM/model tests, bench A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step tests 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/tests.log && ! grep -q "failed" gpurun_out/tests.log || exit 1
step ab 900 python -u scripts/ab.py base no_ffn_store_grad --rounds 4
echo done
