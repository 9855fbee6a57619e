#!/bin/bash
# Round 6: non-temporal epilogue stores in the fused FFN GEMMs (DTD_GEMM_NT_STORE) -- b1024 step,
# interleaved A/B in fresh processes, then the GEMM tests with the knob on.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
out=gpurun_out/r6_ntstore.jsonl
: > $out
for r in 1 2; do
  for nt in 0 1; do
    DTD_GEMM_NT_STORE=$nt timeout -k 10 300 python bench.py --steps 10 --warmup 3 > /tmp/nt.log 2>&1 || { tail -5 /tmp/nt.log; exit 1; }
    echo "{\"round\": $r, \"DTD_GEMM_NT_STORE\": $nt, \"bench\": $(grep '^{' /tmp/nt.log | tail -1)}" >> $out
  done
done
DTD_GEMM_NT_STORE=1 timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_ntstore_tests.log 2>&1
