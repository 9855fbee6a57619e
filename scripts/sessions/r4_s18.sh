#!/usr/bin/env bash
# Round 4 session 18: where the attention kernels' wave cycles go (issue / parked / stalled), one
# PMC pass of 8 SQ counters over the attention kernels alone at B 64
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
B=64 step attn_stall 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/attn_stall -o run --output-format csv -- python scripts/bench_attn.py 3,2,3
step bench_table 300 python bench.py
echo done
