#!/usr/bin/env bash
# Round 6: causal LM head over all B*S positions (last position label -100) -- the model / ZeRO /
# graph GPU tests, then bloom-560m ZeRO b1 stages 0 and 3.
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
step tests 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_model_gpu.py tests/test_parallel_gpu.py tests/test_graph_gpu.py tests/test_head_splitk_gpu.py tests/test_kernels_gpu.py
for r in 1 2; do
  MASTER_PORT=2934$r step bloom_z3_rows_r$r 300 python zero_dp_training.py --stage 3 --quiet --no-memstats
  MASTER_PORT=2935$r step bloom_z0_rows_r$r 300 python zero_dp_training.py --stage 0 --quiet --no-memstats
done
echo done
