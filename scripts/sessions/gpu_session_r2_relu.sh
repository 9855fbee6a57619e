#!/usr/bin/env bash
# ReLU GEMM epilogues (OPT FFN fusions): GEMM + model tests, OPT-125m A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step tests 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/tests.log && ! grep -q "failed" gpurun_out/tests.log || exit 1
step ab_opt 900 python -u scripts/ab.py base no_gemm --rounds 3 -- --model opt-125m --batch-size 64 --steps 10 --warmup 3
echo done
