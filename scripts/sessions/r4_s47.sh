#!/usr/bin/env bash
# Round 4 session 47: verification with the pre-group kernel warm-up in the entry scripts -- GPU
# suite, smoke, bench, the N>1 path at world 1 (DDP, ZeRO-2), data_parallel_training.py
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step pytest_gpu 1000 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 200 python bench.py
step fc 200 python bench.py --force-collectives
step z2fc 200 python bench.py --zero-stage 2 --force-collectives
step bench2 200 python bench.py
echo done
