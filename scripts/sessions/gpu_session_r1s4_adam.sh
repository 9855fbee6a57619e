#!/usr/bin/env bash
# Flat-grid non-temporal fused Adam + zero_dp_training.py --graph (stages 0/1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step pytest_sel 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py tests/test_parallel_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step zero_bloom_eager 300 python zero_dp_training.py --training-steps 60 --quiet --no-memstats
step zero_bloom_graph 300 python zero_dp_training.py --training-steps 60 --quiet --no-memstats --graph
step zero_bloom_graph_mem 300 python zero_dp_training.py --training-steps 60 --quiet --graph
step prof_zero_graph 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_zero_graph -o run --output-format csv -- python zero_dp_training.py --training-steps 30 --quiet --no-memstats --graph
step bench_default 300 python bench.py
step prof_bench 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python bench.py --steps 5 --warmup 2
echo done
