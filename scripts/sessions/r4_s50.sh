#!/usr/bin/env bash
# Round 4 session 50: the fused Adam kernel was first launched after the RCCL group (s49: 245 us
# per call vs 74 in the plain step); the prewarm now runs one optimizer step too
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step fc 200 python bench.py --force-collectives
step base 200 python bench.py
step fc_b 200 python bench.py --force-collectives
step z2fc 200 python bench.py --zero-stage 2 --force-collectives
step base_b 200 python bench.py
echo done
