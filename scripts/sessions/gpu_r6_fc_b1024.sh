#!/bin/bash
# Round 6: the N > 1 data path at world 1 (--force-collectives: RCCL bucket all-reduces, prewarm
# before comm.init) vs the plain step, b1024, interleaved.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
out=gpurun_out/r6_fc_b1024.jsonl
: > $out
for r in 1 2; do
  for fc in "" "--force-collectives"; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 $fc > /tmp/fc.log 2>&1 || { tail -5 /tmp/fc.log; exit 1; }
    echo "{\"round\": $r, \"fc\": \"$fc\", \"bench\": $(grep '^{' /tmp/fc.log | tail -1)}" >> $out
  done
done
