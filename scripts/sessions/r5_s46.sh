#!/usr/bin/env bash
# Round 5 session 46: bench.py through ZeRO-2 / ZeRO-3 at the b1024 default
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step zero2 500 python -u bench.py --zero-stage 2 --steps 6 --warmup 2
step zero3 500 python -u bench.py --zero-stage 3 --steps 6 --warmup 2
echo done
