#!/usr/bin/env bash
# Round 5 session 54: fp32 GEMM -- input gradients as NT on batched W^T copies with fused accumulate:
# tests, per-shape timings (register form vs the LDS form vs hipBLASLt), fp32 BERT-base b32 step
# with the library / hand wgrad / all hand (NT and NN input gradients), kernel traces, counters
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step f32_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_f32_gpu.py
step f32_bench_16k 300 env T=16384 python -u scripts/bench_f32_gemm.py
step f32_bench_16k_lds 300 env T=16384 DTD_GEMM_F32_KERNEL=lds python -u scripts/bench_f32_gemm.py
step f32_bench_32k 300 env T=32768 python -u scripts/bench_f32_gemm.py
for r in 1 2; do
  for v in 0 wgrad 1; do
    step fp32_b32_${v}_$r 300 env DTD_GEMM_F32=$v python -u bench.py --dtype fp32 --batch-size 32 --steps 10 --warmup 3
  done
done
step fp32_b32_1_nn 300 env DTD_GEMM_F32=1 DTD_GEMM_F32_DGRAD=nn python -u bench.py --dtype fp32 --batch-size 32 --steps 10 --warmup 3
export DTD_GEMM_F32=1
step fp32_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s54 -o run --output-format csv -- python3 bench.py --dtype fp32 --batch-size 32 --steps 5 --warmup 2
python scripts/prof_summary.py gpurun_out/prof_s54/run_kernel_stats.csv 7 30 > gpurun_out/r5_s54_fp32_all_hand_kernels.txt 2>&1
export DTD_GEMM_F32=0
step fp32_trace_lib 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s54l -o run --output-format csv -- python3 bench.py --dtype fp32 --batch-size 32 --steps 5 --warmup 2
python scripts/prof_summary.py gpurun_out/prof_s54l/run_kernel_stats.csv 7 30 > gpurun_out/r5_s54_fp32_lib_kernels.txt 2>&1
unset DTD_GEMM_F32
export T=16384
step f32_pmc 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d gpurun_out/pmc_s54 -o run --output-format csv -- python3 scripts/bench_f32_gemm.py
python scripts/step_pmc_summary.py gpurun_out/pmc_s54/run_counter_collection.csv 1 name > gpurun_out/r5_s54_pmc.txt 2>&1
echo done
