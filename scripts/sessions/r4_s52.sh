#!/usr/bin/env bash
# Round 4 session 52: RCCL stream priority on the N>1 path at world 1, now with the pre-group
# warm-up (s31 measured it before the fix)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step fc_hp1 200 python bench.py --force-collectives
DTD_RCCL_HIGH_PRIORITY=0 step fc_hp0 200 python bench.py --force-collectives
step fc_hp1b 200 python bench.py --force-collectives
DTD_RCCL_HIGH_PRIORITY=0 step fc_hp0b 200 python bench.py --force-collectives
step base 200 python bench.py
echo done
