#!/usr/bin/env bash
# Round 6: kernel-time breakdown of the reference's default ZeRO config (bloom-560m, stage 3,
# micro-batch 1 x 512, hipGraph) to see where its 13 ms step goes.
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 MASTER_PORT=29311
R="${GRAFT_REPO_ROOT}"
cd /tmp
step bloom_z3_prof 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/bloomprof" -o bloom -- python3 "$R/zero_dp_training.py" --stage 3 --quiet --no-memstats --training-steps 200
echo done
