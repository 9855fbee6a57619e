#!/usr/bin/env bash
# Round 5 session 12: why the N > 1 data path (force_collectives) runs 17 % below the plain step
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step ab_fc 900 python -u scripts/ab.py fc fc_no_wgrad2 --rounds 2
step trace_fc 300 rocprofv3 --kernel-trace -d gpurun_out/s12_fc -o run --output-format csv -- python3 bench.py --force-collectives --steps 4 --warmup 2
python scripts/prof_summary.py gpurun_out/s12_fc/run_kernel_trace.csv 6 30 > gpurun_out/r5_s12_fc_kernels.txt 2>&1 || true
echo done
