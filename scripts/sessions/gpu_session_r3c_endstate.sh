#!/usr/bin/env bash
# End-of-round state: smoke, bench x2, ZeRO-2 bench, kernel stats of the default step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
rm -f gpurun_out/session.log
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 300 python bench.py
step bench_default2 300 python bench.py
step bench_zero2 300 python bench.py --zero-stage 2
step prof_default 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_end -o run --output-format csv -- python bench.py --steps 5 --warmup 2
echo done
