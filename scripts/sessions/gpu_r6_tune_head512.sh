#!/usr/bin/env bash
# Round 6: TunableOp rows for bloom-560m's head GEMMs at 512 rows (the causal head now runs every
# position), then an interleaved A/B of the merged table vs the committed one at the defaults.
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
T=distributed_training_and_deepspeed_amd/tuning/tunableop_mi355x.csv
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=20 \
  PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tun_bloom512_%d.csv MASTER_PORT=29961 \
  step tune 500 python zero_dp_training.py --stage 3 --graph off --training-steps 3 --quiet --no-memstats
python scripts/merge_tunable.py "$T" gpurun_out/tun_bloom512_0.csv gpurun_out/table_head512.csv || exit 1
for r in 1 2; do
  MASTER_PORT=2997$r step ab_old_r$r 300 python zero_dp_training.py --stage 3 --quiet --no-memstats
  MASTER_PORT=2998$r DTD_TUNED_TABLE=gpurun_out/table_head512.csv step ab_new_r$r 300 python zero_dp_training.py --stage 3 --quiet --no-memstats
done
echo done
