#!/usr/bin/env bash
# Round 4 session 45: the code objects alone did not help (s44); a batch-1 model forward/backward
# before init did (s43).  torch's side-stream pools created before RCCL's streams?
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step fc_full 200 python bench.py --force-collectives
DTD_COMM_PREWARM=streams step fc_streams 200 python bench.py --force-collectives
DTD_COMM_PREWARM=kernels step fc_kernels 200 python bench.py --force-collectives
DTD_COMM_PREWARM=0 step fc_pw_tiny 200 python bench.py --force-collectives --prewarm tiny
step base 200 python bench.py
echo done
