#!/usr/bin/env bash
# Attention keep-mask generator alone: timing + two counter passes (VALU issue vs waits).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
rm -f gpurun_out/session.log
step mask_time 120 python -u scripts/bench_mask.py
step mask_pmc1 90 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY -d gpurun_out/mask_pmc1 -o run --output-format csv -- python scripts/bench_mask.py
step mask_pmc2 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM -d gpurun_out/mask_pmc2 -o run --output-format csv -- python scripts/bench_mask.py
echo done
