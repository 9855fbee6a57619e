#!/usr/bin/env bash
# Round 5 session 4: PMC passes on the wgrad.hip kernel vs hipBLASLt (fc1 weight gradient, 131k tokens)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  step pmc$i 120 timeout -s KILL 110 rocprofv3 --kernel-trace --pmc $P -d gpurun_out/s4_pmc$i -o run --output-format csv -- python scripts/gemm_pmc_probe.py wgrad
done
python scripts/gemm_pmc_probe.py summarize gpurun_out/s4_pmc1/run_counter_collection.csv gpurun_out/s4_pmc2/run_counter_collection.csv gpurun_out/s4_pmc3/run_counter_collection.csv > gpurun_out/r5_s4_wgrad_pmc.json
rm -rf gpurun_out/s4_pmc1 gpurun_out/s4_pmc2 gpurun_out/s4_pmc3
echo done
