#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
step ddp_b4_eager 300 python data_parallel_training.py --training-steps 200 --quiet
step ddp_b4_graph 300 python data_parallel_training.py --training-steps 200 --quiet --graph
step ddp_b32_graph 300 python data_parallel_training.py --training-steps 100 --batch-size 32 --quiet --graph
step bench_b4_graph 300 python bench.py --batch-size 4 --graph on --steps 50 --warmup 10
echo done
