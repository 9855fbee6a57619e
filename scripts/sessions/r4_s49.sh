#!/usr/bin/env bash
# Round 4 session 49: kernel trace of the N>1 path at world 1 with the pre-group warm-up (RCCL
# kernels in the step, the rest at their plain-step durations)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step fc_trace 300 rocprofv3 --kernel-trace -d gpurun_out/s49_fc -o run -- python bench.py --force-collectives --steps 6 --warmup 3
python scripts/prof_summary.py gpurun_out/s49_fc/run_results.db 9 > gpurun_out/s49_fc_kernels.txt 2>&1
python scripts/diag/step_kernels.py gpurun_out/s49_fc/run_results.db > gpurun_out/s49_fc_steps.txt 2>&1
rm -rf gpurun_out/s49_fc
echo done
