#!/usr/bin/env bash
# Round 5 session 58: fp32 b32 step with the forward products + weight gradients on the hand kernel
# and the input gradients on the library (DTD_GEMM_F32=fwd), interleaved with library / wgrad / all
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step f32_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_f32_gpu.py
for r in 1 2 3; do
  for v in 0 wgrad fwd 1; do
    step fp32_${v}_$r 300 env DTD_GEMM_F32=$v python -u bench.py --dtype fp32 --batch-size 32 --steps 10 --warmup 3
  done
done
echo done
