#!/usr/bin/env bash
# Graph warm-up on the first real batches: graph and eager runs train the same steps on the
# same batches, so their final losses must match.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step pytest_graph 300 python -u -m pytest tests/test_graph_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step zero_eager 300 python zero_dp_training.py --training-steps 40 --quiet
step zero_graph 300 python zero_dp_training.py --training-steps 40 --quiet --graph
step ddp_eager 300 python data_parallel_training.py --batch-size 4 --training-steps 200 --quiet
step ddp_graph 300 python data_parallel_training.py --batch-size 4 --training-steps 200 --quiet --graph
echo done
