#!/bin/bash
# Round 6: LayerNorm backward with the software-pipelined row loop (DTD_LN_BWD_PREFETCH=1) vs the
# default at b1024, interleaved.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
out=gpurun_out/r6_lnpf.jsonl
: > $out
for r in 1 2; do
  for pf in 0 1; do
    DTD_LN_BWD_PREFETCH=$pf timeout -k 10 300 python bench.py --steps 10 --warmup 3 > /tmp/lp.log 2>&1 || { tail -5 /tmp/lp.log; exit 1; }
    echo "{\"round\": $r, \"DTD_LN_BWD_PREFETCH\": $pf, \"bench\": $(grep '^{' /tmp/lp.log | tail -1)}" >> $out
  done
done
