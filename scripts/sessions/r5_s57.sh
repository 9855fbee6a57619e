#!/usr/bin/env bash
# Round 5 session 57: fp32 GEMM with 128 x 96 wave tiles everywhere N allows (396 / 448 registers per
# wave: a side-stream kernel's small wave still fits on the SIMD) -- tests on every form, then the
# fp32 b32 step interleaved: library / wgrad / wgrad+96 / all / all+96
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step f32_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_f32_gpu.py
for r in 1 2; do
  step fp32_lib_$r 300 env DTD_GEMM_F32=0 python -u bench.py --dtype fp32 --batch-size 32 --steps 10 --warmup 3
  step fp32_wgrad_$r 300 env DTD_GEMM_F32=wgrad python -u bench.py --dtype fp32 --batch-size 32 --steps 10 --warmup 3
  step fp32_wgrad96_$r 300 env DTD_GEMM_F32=wgrad DTD_GEMM_F32_NB3=1 python -u bench.py --dtype fp32 --batch-size 32 --steps 10 --warmup 3
  step fp32_all_$r 300 env DTD_GEMM_F32=1 python -u bench.py --dtype fp32 --batch-size 32 --steps 10 --warmup 3
  step fp32_all96_$r 300 env DTD_GEMM_F32=1 DTD_GEMM_F32_NB3=1 python -u bench.py --dtype fp32 --batch-size 32 --steps 10 --warmup 3
done
export DTD_GEMM_F32=1 DTD_GEMM_F32_NB3=1
step fp32_trace96 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s57 -o run --output-format csv -- python3 bench.py --dtype fp32 --batch-size 32 --steps 5 --warmup 2
python scripts/prof_summary.py gpurun_out/prof_s57/run_kernel_stats.csv 7 30 > gpurun_out/r5_s57_fp32_all96_kernels.txt 2>&1
echo done
