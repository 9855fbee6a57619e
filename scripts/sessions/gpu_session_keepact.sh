#!/usr/bin/env bash
# keep_ffn_act verification + bench, and a host-side cProfile of the ZeRO trainer at b1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
step pytest_model 600 python -u -m pytest tests/test_model_gpu.py tests/test_graph_gpu.py -x -q --timeout 120 --timeout-method thread
step bench_default 300 python bench.py
step bench_default2 300 python bench.py
step cprof_zero 300 python -m cProfile -o gpurun_out/zero_s0.prof zero_dp_training.py --stage 0 --training-steps 30 --quiet --no-memstats
step cprof_bert_b4 300 python -m cProfile -o gpurun_out/bert_b4.prof bench.py --batch-size 4 --steps 30
echo done
