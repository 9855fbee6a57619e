#!/usr/bin/env bash
# Round 6: the reference's own configurations on the current tree (graphs replayed on one HW queue):
# bloom-560m ZeRO 0/3 at zero_dp_training.py defaults, BERT-large 2-stage MP / GPipe (one GPU),
# data_parallel_training.py at the reference batch.
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
export MASTER_ADDR=127.0.0.1
MASTER_PORT=29901 step bloom_z0 300 python zero_dp_training.py --stage 0 --quiet --no-memstats
MASTER_PORT=29902 step bloom_z3 300 python zero_dp_training.py --stage 3 --quiet --no-memstats
step mp_large_graph 200 python model_parallel_training.py --model bert-large-cased --devices cuda:0,cuda:0 --batch-size 16 --training-steps 40 --graph on
step gpipe_large_graph 200 python model_parallel_training.py --model bert-large-cased --devices cuda:0,cuda:0 --batch-size 16 --training-steps 40 --pipeline --graph on
step b4_graph_fc 300 python bench.py --batch-size 4 --graph on --steps 200 --warmup 20 --force-collectives
echo done
