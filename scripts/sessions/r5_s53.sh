#!/usr/bin/env bash
# Round 5 session 53: register-direct fp32 GEMM with the NN input-gradient form (no transposed weight copy) and
# fused accumulate: tests, per-shape timings (register form vs the LDS
# form vs hipBLASLt), fp32 BERT-base b32 step with the library / hand wgrad / all hand, counters
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
export T=16384
step f32_pmc 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d gpurun_out/pmc_s53 -o run --output-format csv -- python3 scripts/bench_f32_gemm.py
python scripts/step_pmc_summary.py gpurun_out/pmc_s53/run_counter_collection.csv 1 name > gpurun_out/r5_s53_pmc.txt 2>&1
echo done
