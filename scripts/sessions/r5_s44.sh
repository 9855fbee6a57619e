#!/usr/bin/env bash
# Round 5 session 44: the driver's command at the b1024 default; the N > 1 data path at world 1
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step bench 500 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_fc 500 python -u bench.py --force-collectives --steps 10 --warmup 3
echo done
