#!/usr/bin/env bash
# Round 4 session 25: is the async weight-gradient stream erratic (one A/B round ran at 286 k)?
# three runs with the tuned table, three without; loss values recorded by each bench line
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step async_t1 240 python bench.py --async-wgrad on
step async_t2 240 python bench.py --async-wgrad on
step async_t3 240 python bench.py --async-wgrad on
step async_u1 240 python bench.py --async-wgrad on --no-tuned-gemms
step async_u2 240 python bench.py --async-wgrad on --no-tuned-gemms
step base_1 240 python bench.py
echo done
