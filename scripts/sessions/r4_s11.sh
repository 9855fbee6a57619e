#!/usr/bin/env bash
# Round 4 session 11: ZeRO capture with collectives issued on the capture stream
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step zerobisect 600 python -u scripts/diag/zero_capture_bisect.py s1_fwd_only s1_fwd_bwd_only s1_step_only s1 s2 s3 s2_no_overlap_comm s2_one_bucket
echo done
