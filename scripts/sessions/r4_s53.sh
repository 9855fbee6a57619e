#!/usr/bin/env bash
# Round 4 session 53: is the async weight-gradient pathology (5-9x slower) another first-launch
# effect?  The same run with the 1-layer warm-up first.
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step async 200 python bench.py --async-wgrad on --steps 10 --warmup 3
step async_pw 200 python bench.py --async-wgrad on --prewarm layer1 --steps 10 --warmup 3
echo done
