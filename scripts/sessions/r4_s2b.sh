#!/usr/bin/env bash
# Round 4 session 2b: fused attention backward (numerics, kernel time, whole step), the fp32 GEMM,
# ZeRO at world 2 on one GPU, the gemm4 probe and the force-collectives benches.
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step tests_attn_fused 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_attention_gpu.py -k fused
if grep -q " passed" gpurun_out/tests_attn_fused.log && ! grep -q "failed" gpurun_out/tests_attn_fused.log; then
  step bench_attn 200 env B=256 python scripts/bench_attn.py 3,2,3 fused 3,2,3 fused
  step bench_fused 300 env DTD_ATTN_BWD=fused python bench.py
fi
step bench_default 300 python bench.py
step gemm_stagger 240 python scripts/bench_gemm_stagger.py
step tests_gemm_f32 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gemm_f32_gpu.py
step bench_f32_gemm 200 python scripts/bench_f32_gemm.py
step tests_zero_w2 400 python -u -m pytest -v --timeout 180 --timeout-method thread tests/test_parallel_gpu.py -k two_ranks
step bench_force 300 python bench.py --force-collectives
step gemm4_probe 400 python scripts/gemm4_probe.py
echo done
