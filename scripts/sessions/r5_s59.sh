#!/usr/bin/env bash
# Round 5 session 59: fp32 b32 step -- NT products on 128 x 96 wave tiles wherever they fill the round
# (DTD_GEMM_F32_NT96=1: 396 registers, so the side-stream keep-mask generator and Adam fit beside them)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
for r in 1 2 3; do
  step fp32_0_$r 300 env DTD_GEMM_F32=0 python -u bench.py --dtype fp32 --batch-size 32 --steps 10 --warmup 3
  step fp32_wgrad_$r 300 env DTD_GEMM_F32=wgrad python -u bench.py --dtype fp32 --batch-size 32 --steps 10 --warmup 3
  step fp32_fwd96_$r 300 env DTD_GEMM_F32=fwd DTD_GEMM_F32_NT96=1 python -u bench.py --dtype fp32 --batch-size 32 --steps 10 --warmup 3
  step fp32_all96_$r 300 env DTD_GEMM_F32=1 DTD_GEMM_F32_NT96=1 python -u bench.py --dtype fp32 --batch-size 32 --steps 10 --warmup 3
done
export DTD_GEMM_F32=1 DTD_GEMM_F32_NT96=1
step fp32_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s59 -o run --output-format csv -- python3 bench.py --dtype fp32 --batch-size 32 --steps 5 --warmup 2
python scripts/prof_summary.py gpurun_out/prof_s59/run_kernel_stats.csv 7 30 > gpurun_out/r5_s59_fp32_all_nt96_kernels.txt 2>&1
echo done
