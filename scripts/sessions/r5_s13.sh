#!/usr/bin/env bash
# Round 5 session 13: N > 1 data path after restoring 8 HW queues (the boxes export 4)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step ab_fc 900 python -u scripts/ab.py base fc fc_no_wgrad2 --rounds 3
echo done
