#!/usr/bin/env bash
# Round 4 session 8: is the ZeRO capture crash the side comm stream or the autograd thread?
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
step capcoll 300 python -u scripts/diag/capture_collectives.py side_stream_rs autograd_rs autograd_side_stream_rs
step zerobisect 400 python -u scripts/diag/zero_capture_bisect.py s1_fwd_bwd_nostream s1_step_only_nostream s2_nostream
echo done
