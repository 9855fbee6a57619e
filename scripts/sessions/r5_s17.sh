#!/usr/bin/env bash
# Round 5 session 17: step kernel budget with the bit-plane mask generator, full GPU suite,
# smoke(), the driver's bench command
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s17 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2
python scripts/prof_summary.py gpurun_out/prof_s17/run_kernel_stats.csv 7 40 > gpurun_out/r5_s17_kernel_summary.txt 2>&1
step gpu_suite 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
echo done
