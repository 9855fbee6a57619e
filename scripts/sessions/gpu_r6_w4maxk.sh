#!/bin/bash
# Round 6: gemm_w4 for every plain product (DTD_GEMM_W4_MAX_K=4096) vs the long-K products (fc2
# forward, fc1 input gradient) left on hipBLASLt (2304), b1024 step, interleaved, fresh processes.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
out=gpurun_out/r6_w4maxk.jsonl
: > $out
for r in 1 2 3; do
  for k in 4096 2304; do
    DTD_GEMM_W4_MAX_K=$k timeout -k 10 300 python bench.py --steps 10 --warmup 3 > /tmp/mk.log 2>&1 || { tail -5 /tmp/mk.log; exit 1; }
    echo "{\"round\": $r, \"DTD_GEMM_W4_MAX_K\": $k, \"bench\": $(grep '^{' /tmp/mk.log | tail -1)}" >> $out
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gemm_w4_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_w4maxk_tests.log 2>&1
