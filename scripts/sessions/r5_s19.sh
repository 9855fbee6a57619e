#!/usr/bin/env bash
# Round 5 session 19: which parameters differ between the staged (overlapped) and single-launch AdamW
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step staged_diff 300 python -u scripts/diag/staged_adam_diff.py
step staged_diff_old 300 env DTD_KERNELS_SO=$PWD/distributed_training_and_deepspeed_amd/ops/_dtd_kernels_oldmask.so REPEAT=1 python -u scripts/diag/staged_adam_diff.py
echo done
