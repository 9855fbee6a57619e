#!/usr/bin/env bash
# GEMM main-loop probe: K sweep (slope = per-K-step cost, intercept = per-tile overhead) for both
# kernel forms, and one PMC pass on the tile form at K = 768 and K = 6144.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
DTD_GEMM_VARIANT=0 step probe_t 300 python -u scripts/gemm_probe.py
DTD_GEMM_VARIANT=1 step probe_p 300 python -u scripts/gemm_probe.py
PMC="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
DTD_GEMM_VARIANT=0 step pmc768 120 timeout -s KILL 90 rocprofv3 --pmc $PMC -d gpurun_out/pmc768 -o run --output-format csv -- python scripts/gemm_probe.py --once 768
DTD_GEMM_VARIANT=0 step pmc6144 120 timeout -s KILL 90 rocprofv3 --pmc $PMC -d gpurun_out/pmc6144 -o run --output-format csv -- python scripts/gemm_probe.py --once 6144
echo done
