#!/bin/bash
# Round 6: gemm_w4 tests (EPI_ADD asm prefetch, tile-count dispatch rule), EPI_ADD bench, the graph
# tests with the RCCL capture cases in-process, and the b4 graph / b1024 step.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemm_w4_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/w4_test.log 2>&1 || exit 1
ONLY=dgrad_qkv_add,dgrad_fc1,fwd_qkv ROUNDS=3 timeout -k 10 300 python -u scripts/bench_gemm_w4.py > gpurun_out/r6_w4add.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_graph_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r6_graph_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --batch-size 4 --graph on --steps 200 --warmup 20 > gpurun_out/r6_b4g.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 6 --warmup 2 > gpurun_out/r6_b1024.log 2>&1 || exit 1
DTD_GEMM_W4_ADD=1 timeout -k 10 300 python bench.py --steps 6 --warmup 2 > gpurun_out/r6_b1024_add.log 2>&1
