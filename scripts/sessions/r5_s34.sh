#!/usr/bin/env bash
# Round 5 session 34: eager --async-wgrad with the side-stream inputs held to the join (no
# record_stream); then same-box A/B against the default step
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step aw_hold10 200 python -u bench.py --async-wgrad on --steps 10 --warmup 1
step aw_hold20 300 python -u bench.py --async-wgrad on --steps 20 --warmup 5
step ab_aw 900 python -u scripts/ab.py base async_wgrad --rounds 3
echo done
