#!/usr/bin/env bash
# Sustained throughput: the default bench for 200 timed steps (~20 s of back-to-back steps,
# past the chip's DVFS settling) next to the driver's default short run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
rm -f gpurun_out/session.log
step bench_short 300 python bench.py
step bench_200 300 python bench.py --steps 200 --warmup 10
step bench_short2 300 python bench.py
echo done
