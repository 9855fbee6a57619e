#!/usr/bin/env bash
# Per-kernel effective clock and MFMA busy share inside the real BERT-base b256 training step
# (one counter pass over bench.py; PMC serialises the kernels, so side-stream overlap is absent).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
rm -f gpurun_out/session.log
step step_pmc 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVE_CYCLES -d gpurun_out/step_pmc -o run --output-format csv -- python bench.py --steps 2 --warmup 1
echo done
