#!/usr/bin/env bash
# Round 5 session 49: fp32 GEMM -- hand f32-MFMA kernel vs hipBLASLt at the fp32 config's shapes
# (T 16384 = b32 x seq 512): timings, then one counter pass (clock, MFMA busy, wait shares)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
export T=16384
step f32_bench 300 python -u scripts/bench_f32_gemm.py
step f32_pmc 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d gpurun_out/pmc_s49 -o run --output-format csv -- python3 scripts/bench_f32_gemm.py
python scripts/step_pmc_summary.py gpurun_out/pmc_s49/run_counter_collection.csv 1 name > gpurun_out/r5_s49_pmc.txt 2>&1
echo done
