#!/usr/bin/env bash
# Round 5 session 38: per-GPU batch 256 / 384 / 512 (the TunableOp table has rows for b256 only)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step b256 300 python -u bench.py --steps 10 --warmup 3
step b384 300 python -u bench.py --steps 10 --warmup 3 --batch-size 384
step b512 300 python -u bench.py --steps 10 --warmup 3 --batch-size 512
echo done
