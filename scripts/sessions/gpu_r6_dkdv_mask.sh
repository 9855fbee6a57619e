#!/bin/bash
# Round 6: dK/dV without the hoisted causal / sequence-end mask code (MASK=false instantiation):
# attention tests, kernel times at B = 256 under a kernel trace, b1024 step.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_dkdv_mask_tests.log 2>&1 || exit 1
P=0.1 B=256 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r6_dkdv_mask -o run -- python scripts/bench_attn.py 3,2,3 > gpurun_out/r6_dkdv_mask_attn.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r6_dkdv_mask_bench.log 2>&1
