#!/usr/bin/env bash
# Round 4 session 31: RCCL internal streams at high priority (comm.init default) vs normal, on the
# N>1 path at world 1 (DDP and ZeRO-2 with real collectives), interleaved
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step fc_hp1 200 python bench.py --force-collectives
DTD_RCCL_HIGH_PRIORITY=0 step fc_hp0 200 python bench.py --force-collectives
step fc_hp1b 200 python bench.py --force-collectives
DTD_RCCL_HIGH_PRIORITY=0 step fc_hp0b 200 python bench.py --force-collectives
step z2fc_hp1 200 python bench.py --zero-stage 2 --force-collectives
DTD_RCCL_HIGH_PRIORITY=0 step z2fc_hp0 200 python bench.py --zero-stage 2 --force-collectives
step base 200 python bench.py
echo done
