#!/usr/bin/env bash
# Round 6: the reference's default configurations with the extended TunableOp table, tuned vs
# untuned (DTD_TUNED_GEMMS=0), interleaved.
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
for r in 1 2; do
  for t in 0 1; do
    DTD_TUNED_GEMMS=$t MASTER_PORT=291$r$t step bloom_z3_t${t}_r$r 300 python zero_dp_training.py --stage 3 --quiet --no-memstats
    DTD_TUNED_GEMMS=$t MASTER_PORT=292$r$t step ddp_b4_t${t}_r$r 300 python data_parallel_training.py --batch-size 4 --training-steps 300 --quiet --metrics-json gpurun_out/ddp_b4_t${t}_r$r.json
  done
done
echo done
