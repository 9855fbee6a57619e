#!/usr/bin/env bash
# Round 5 session 42: per-GPU batch 512 / 768 / 1024
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step c512 300 python -u bench.py --steps 8 --warmup 3
step c768 300 python -u bench.py --steps 8 --warmup 3 --batch-size 768
step c1024 400 python -u bench.py --steps 8 --warmup 3 --batch-size 1024
echo done
