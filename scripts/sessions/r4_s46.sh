#!/usr/bin/env bash
# Round 4 session 46: bench.py now runs a 1-layer batch-1 copy of the model before creating the
# RCCL group (utils/prewarm.py).  Enough, or does it need the full depth (s43: tiny)?
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step fc_layer1 200 python bench.py --force-collectives
step fc_tiny 200 python bench.py --force-collectives --prewarm tiny
step fc_none 200 python bench.py --force-collectives --prewarm none
step z2fc_layer1 200 python bench.py --zero-stage 2 --force-collectives
step base 200 python bench.py
step fc_layer1b 200 python bench.py --force-collectives
echo done
