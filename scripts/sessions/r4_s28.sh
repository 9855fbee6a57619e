#!/usr/bin/env bash
# Round 4 session 28: verification with the entry scripts' new hardware-queue default (8) --
# full GPU suite, smoke, default bench x2, force-collectives bench (the N>1 step's path)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step pytest_gpu 1000 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 300 python bench.py
step fc 300 python bench.py --force-collectives
step bench2 300 python bench.py
echo done
