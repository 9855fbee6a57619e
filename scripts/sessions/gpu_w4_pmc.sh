#!/bin/bash
# PMC passes of gemm_w4.hip vs hipBLASLt (scripts/gemm_pmc_probe.py w4); one rocprofv3 run per pass.
set -e
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
timeout -k 10 200 python -c "import torch; torch.zeros(1, device='cuda')"
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P -d gpurun_out/w4pmc$i -o run --output-format csv -- python scripts/gemm_pmc_probe.py w4 > gpurun_out/w4pmc$i.log 2>&1
done
python scripts/gemm_pmc_probe.py summarize $(find gpurun_out/w4pmc1 gpurun_out/w4pmc2 -name '*counter_collection.csv') > gpurun_out/w4_pmc.json
