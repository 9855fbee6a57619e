#!/usr/bin/env bash
# Round 5 session 11: RCCL-init slowdown with the round-5 kernels (prewarm at the bench batch; the
# eager-code-object-loading experiment, logged), then the capture crash candidates (crash last)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step ab_prewarm 900 python -u scripts/ab.py base fc fc_prewarm_l1b --rounds 3
step capture 300 python -u scripts/diag/capture_collectives.py side_stream_rs_keepwork side_stream_rs_evcache side_stream_rs
echo done
