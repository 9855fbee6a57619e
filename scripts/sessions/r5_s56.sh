#!/usr/bin/env bash
# Round 5 session 56: bf16 driver bench x2 on the current tree, then the b1024 default's kernel
# budget (kernel trace) and per-kernel clock / MFMA-busy / VALU-per-MFMA (one counter pass)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step bench1 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench2 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
step prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s56 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2
python scripts/prof_summary.py gpurun_out/prof_s56/run_kernel_stats.csv 5 40 > gpurun_out/r5_s56_kernel_summary_b1024.txt 2>&1
step pmc 400 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU -d gpurun_out/pmc_s56 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1
python scripts/step_pmc_summary.py gpurun_out/pmc_s56/run_counter_collection.csv 3 > gpurun_out/r5_s56_step_pmc.txt 2>&1
echo done
