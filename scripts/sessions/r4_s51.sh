#!/usr/bin/env bash
# Round 4 session 51: closing verification of the final tree (GPU suite, smoke, bench x2,
# force-collectives)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step pytest_gpu 1000 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 200 python bench.py
step fc 200 python bench.py --force-collectives
step bench2 200 python bench.py
echo done
