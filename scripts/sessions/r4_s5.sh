#!/usr/bin/env bash
# Round 4 session 5: the full GPU test suite and smoke() on the committed tree.
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step pytest_gpu 1000 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -x
step smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
echo done
