#!/usr/bin/env bash
# Round 4 session 39: the slowdown after RCCL init survives comm destroy (s33) and needs no
# collective (s38 trace): RCCL's process-wide RAS thread?  (NCCL_RAS_ENABLE=0)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
NCCL_RAS_ENABLE=0 step rccl_noras 200 python bench.py --comm-init rccl
step rccl 200 python bench.py --comm-init rccl
NCCL_RAS_ENABLE=0 step fc_noras 200 python bench.py --force-collectives
NCCL_RAS_ENABLE=0 step rccl_noras2 200 python bench.py --comm-init rccl
step base 200 python bench.py
echo done
