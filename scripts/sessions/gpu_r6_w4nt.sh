#!/bin/bash
# Round 6: gemm_w4 with non-temporal epilogue stores (schedule variant 2) vs the default --
# per-product timings and the b1024 step, interleaved, fresh processes.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
SCHEDS=2 ROUNDS=3 timeout -k 10 300 python -u scripts/bench_gemm_w4.py > gpurun_out/r6_w4nt_gemm.log 2>&1 || exit 1
out=gpurun_out/r6_w4nt.jsonl
: > $out
for r in 1 2; do
  for sc in 0 2; do
    DTD_GEMM_W4_SCHED=$sc timeout -k 10 300 python bench.py --steps 10 --warmup 3 > /tmp/nt.log 2>&1 || { tail -5 /tmp/nt.log; exit 1; }
    echo "{\"round\": $r, \"DTD_GEMM_W4_SCHED\": $sc, \"bench\": $(grep '^{' /tmp/nt.log | tail -1)}" >> $out
  done
done
DTD_GEMM_W4_SCHED=2 timeout -k 10 300 python -u -m pytest tests/test_gemm_w4_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_w4nt_tests.log 2>&1
