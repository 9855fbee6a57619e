#!/bin/bash
# Round 6: the b1024 step with the TunableOp table extended by its own shapes vs no table, interleaved.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
out=gpurun_out/r6_tuned_b1024_ab.jsonl
: > $out
for r in 1 2 3; do
  for t in off on; do
    if [ $t = off ]; then f=--no-tuned-gemms; else f=""; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 $f > /tmp/tb.log 2>&1 || { tail -5 /tmp/tb.log; exit 1; }
    echo "{\"round\": $r, \"table\": \"$t\", \"bench\": $(grep '^{' /tmp/tb.log | tail -1)}" >> $out
  done
done
