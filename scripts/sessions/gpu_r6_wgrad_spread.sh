#!/bin/bash
# Round 6: wgrad.hip with its K-step DMA pieces spread over the MFMA groups (variant 46) vs the
# default (44): per-shape timings at b1024's token count, then the b1024 step interleaved.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
T=524288 ROUNDS=3 VARIANTS=44,46 timeout -k 10 300 python -u scripts/bench_wgrad.py > gpurun_out/r6_wgrad_spread.log 2>&1 || exit 1
out=gpurun_out/r6_wgrad_spread_step.jsonl
: > $out
for r in 1 2; do
  for v in 44 46; do
    DTD_WGRAD_VARIANT=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 > /tmp/wg.log 2>&1 || { tail -5 /tmp/wg.log; exit 1; }
    echo "{\"round\": $r, \"DTD_WGRAD_VARIANT\": $v, \"bench\": $(grep '^{' /tmp/wg.log | tail -1)}" >> $out
  done
done
DTD_WGRAD_VARIANT=46 timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q -k wgrad --timeout 120 --timeout-method thread > gpurun_out/r6_wgrad_spread_tests.log 2>&1
