#!/usr/bin/env bash
# Round 4 session 43: RCCL init after the warm-up steps costs nothing (s42).  Is it the code objects
# loaded after the communicator (prewarm tiny: one batch-1 forward/backward first) or the memory
# the step allocates after it (prewarm full: one bench-batch forward/backward first)?
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step rccl_pw_tiny 200 python bench.py --comm-init rccl --prewarm tiny
step rccl_pw_full 200 python bench.py --comm-init rccl --prewarm full
step fc_pw_tiny 200 python bench.py --force-collectives --prewarm tiny
step rccl 200 python bench.py --comm-init rccl
step base 200 python bench.py
echo done
