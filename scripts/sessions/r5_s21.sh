#!/usr/bin/env bash
# Round 5 session 21: hipGraph capture of a side-stream RCCL collective -- is the crash the nested
# fork (RCCL's stream joined only into the side stream, never into the capturing stream)?
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step cap_join 200 python -u scripts/diag/capture_collectives.py side_stream_rs_join_origin side_stream_rs_origin_only
echo done
