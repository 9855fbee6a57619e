#!/usr/bin/env bash
# Round 6 closing: per-kernel held clock / MFMA-busy / VALU-per-MFMA of the b1024 step (one
# counter pass, kernel trace only -- no sys / runtime trace with --pmc).
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step pmc 400 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU -d gpurun_out/pmc_r6 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1
python scripts/step_pmc_summary.py gpurun_out/pmc_r6/run_counter_collection.csv 3 > gpurun_out/r6_step_pmc.txt 2>&1
echo done
