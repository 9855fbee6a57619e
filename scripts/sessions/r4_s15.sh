#!/usr/bin/env bash
# Round 4 session 15: per-kernel clock / MFMA-busy / VALU-per-MFMA of the round-4 step (one PMC pass)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step step_pmc 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVE_CYCLES -d gpurun_out/step_pmc -o run --output-format csv -- python bench.py --steps 2 --warmup 1
echo done
