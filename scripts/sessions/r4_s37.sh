#!/usr/bin/env bash
# Round 4 session 37: HIP device state before / after RCCL init; NCCL_SET_STACK_SIZE A/B
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step state 120 python scripts/diag/rccl_state.py
NCCL_SET_STACK_SIZE=0 step state_ss0 120 python scripts/diag/rccl_state.py
NCCL_SET_STACK_SIZE=0 step rccl_ss0 200 python bench.py --comm-init rccl
step rccl 200 python bench.py --comm-init rccl
echo done
