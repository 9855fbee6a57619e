#!/usr/bin/env bash
# PMC counters of the attention kernels (B=32 S=512 H=12 D=64 p=0.1), one counter group per pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step pmc_a 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES -d gpurun_out/pmc_a -o run --output-format csv -- python scripts/bench_attn.py 3,2,3
step pmc_b 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/pmc_b -o run --output-format csv -- python scripts/bench_attn.py 3,2,3
step pmc_c 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU -d gpurun_out/pmc_c -o run --output-format csv -- python scripts/bench_attn.py 3,2,3
echo done
