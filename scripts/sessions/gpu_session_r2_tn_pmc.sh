#!/usr/bin/env bash
# PMC passes over the TN wgrad kernel vs the NT kernel (scripts/tn_probe.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step pmc_a 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/tn_a -o run --output-format csv -- python scripts/tn_probe.py
step pmc_b 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU -d gpurun_out/tn_b -o run --output-format csv -- python scripts/tn_probe.py
echo done
