#!/usr/bin/env bash
# Round 5 session 67: closing validation after the NN-slot change -- full GPU suite, smoke, driver bench, fp32 default step
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step gpu_suite 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')"
step bench 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
step fp32_b32_default 300 python -u bench.py --dtype fp32 --batch-size 32 --steps 10 --warmup 3
echo done
