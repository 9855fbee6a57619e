#!/usr/bin/env bash
# Round 6 closing check on the final tree: full GPU suite, smoke, driver bench command.
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step gpu_suite 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')"
step bench 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
echo done
