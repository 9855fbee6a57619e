#!/usr/bin/env bash
# Round-3 closing verification of the committed tree: full GPU suite, smoke, bench x2, ZeRO-2 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
rm -f gpurun_out/session.log
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 300 python bench.py
step bench_default2 300 python bench.py
step bench_zero2 300 python bench.py --zero-stage 2
echo done
