#!/usr/bin/env bash
# Round 4 session 32: isolate the N>1 path's cost at world 1 -- an initialised RCCL group with no
# collectives; collectives all launched after the backward (no overlap); the normal overlapped form
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step base 200 python bench.py
step pg_only 200 python bench.py --comm-init
step fc_post 200 python bench.py --force-collectives --ddp-overlap off
step fc 200 python bench.py --force-collectives
step pg_only2 200 python bench.py --comm-init
step base2 200 python bench.py
echo done
