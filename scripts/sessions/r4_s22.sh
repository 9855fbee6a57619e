#!/usr/bin/env bash
# Round 4 session 22: closing verification of the final tree -- full GPU suite, smoke, bench x2
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step pytest_gpu 1000 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 300 python bench.py
step bench2 300 python bench.py
echo done
