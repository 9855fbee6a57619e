#!/usr/bin/env bash
# Round 5 session 40: bench default per-GPU batch 512: the driver's command, the N > 1 data path at
# world 1, smoke
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step bench 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_fc 400 python -u bench.py --force-collectives --steps 10 --warmup 3
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
echo done
