#!/usr/bin/env bash
# Round 4 session 38: HIP device state before / after RCCL init (probe fixed); kernel trace of the
# step after RCCL init with no collectives, for per-kernel comparison against the plain step
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step state 120 python scripts/diag/rccl_state.py
step trace 300 rocprofv3 --kernel-trace -d gpurun_out/s38_rccl -o run -- python bench.py --comm-init rccl --steps 6 --warmup 3
python scripts/prof_summary.py gpurun_out/s38_rccl/run_results.db 9 > gpurun_out/s38_rccl_kernels.txt 2>&1
python scripts/diag/step_kernels.py gpurun_out/s38_rccl/run_results.db > gpurun_out/s38_rccl_steps.txt 2>&1
rm -rf gpurun_out/s38_rccl
echo done
