#!/usr/bin/env bash
# GEMM main-loop limiter probe (diagnostic builds, timing only) + TN weight-gradient PMC.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
OPS=$PWD/distributed_training_and_deepspeed_amd/ops
for r in 1 2; do
  step diag_base_$r 120 python -u scripts/gemm_diag.py
  for d in 1 2 4 7; do step diag${d}_$r 120 env DTD_KERNELS_SO=$OPS/_dtd_kernels_diag$d.so python -u scripts/gemm_diag.py; done
done
step pmc_tn1 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_tn1 -o run --output-format csv -- python scripts/gemm_pmc_probe.py wgrad
step pmc_tn2 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d gpurun_out/pmc_tn2 -o run --output-format csv -- python scripts/gemm_pmc_probe.py wgrad
step attn_p0 200 env B=256 P=0 python -u scripts/bench_attn.py 3,2,3
step attn_p1 200 env B=256 P=0.1 python -u scripts/bench_attn.py 3,2,3
echo done
