#!/usr/bin/env bash
# Round 4 session 19: the merged TunableOp table vs the previous one, same box
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step ab_table2 900 python scripts/ab.py base table_prev --rounds 4
echo done
