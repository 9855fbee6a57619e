#!/usr/bin/env bash
# Round 4 session 35: RCCL init pins the calling thread to the GPU's NUMA cores ("Setting affinity
# for GPU 0", s34 log) -- is that the N>1 step's ~10 % (the host thread that launches every kernel)?
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step affinity 120 python scripts/diag/rccl_affinity.py
NCCL_IGNORE_CPU_AFFINITY=1 step affinity_ign 120 python scripts/diag/rccl_affinity.py
NCCL_IGNORE_CPU_AFFINITY=1 step rccl_ign 200 python bench.py --comm-init rccl
step rccl 200 python bench.py --comm-init rccl
NCCL_IGNORE_CPU_AFFINITY=1 step fc_ign 200 python bench.py --force-collectives
step base 200 python bench.py
echo done
