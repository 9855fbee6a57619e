#!/usr/bin/env bash
# Round 5 session 66: NN fp32 form with 4-float vector slots for its dwordx3 [k][n] operand (the
# loads land in place: no copy / early wait inside the loop) -- tests, per-shape timings, fp32 b32
# step: library / wgrad / all with NT input gradients / all with NN input gradients
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step f32_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_f32_gpu.py
step f32_bench_16k 300 env T=16384 python -u scripts/bench_f32_gemm.py
for r in 1 2; do
  step fp32_0_$r 300 env DTD_GEMM_F32=0 python -u bench.py --dtype fp32 --batch-size 32 --steps 10 --warmup 3
  step fp32_wgrad_$r 300 env DTD_GEMM_F32=wgrad python -u bench.py --dtype fp32 --batch-size 32 --steps 10 --warmup 3
  step fp32_1nt_$r 300 env DTD_GEMM_F32=1 python -u bench.py --dtype fp32 --batch-size 32 --steps 10 --warmup 3
  step fp32_1nn_$r 300 env DTD_GEMM_F32=1 DTD_GEMM_F32_DGRAD=nn python -u bench.py --dtype fp32 --batch-size 32 --steps 10 --warmup 3
done
echo done
