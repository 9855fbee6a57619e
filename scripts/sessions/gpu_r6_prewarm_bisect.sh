#!/bin/bash
# Round 6: bisect of the pre-communicator prewarm (the post-RCCL-init slowdown): the N > 1 data
# path at world 1 (--force-collectives), b256, with each prewarm arm before comm.init, two
# interleaved rounds in fresh processes.
cd "$(dirname "$0")/../.."
out=gpurun_out/r6_prewarm_bisect.jsonl
: > $out
for r in 1 2; do
  for arm in none auto blas reserve custom; do
    timeout -k 10 240 python bench.py --batch-size 256 --force-collectives --steps 30 --warmup 5 \
      --prewarm $arm --reserve-gb 45 > /tmp/pw.log 2>&1 || { tail -20 /tmp/pw.log; exit 1; }
    echo "{\"round\": $r, \"arm\": \"$arm\", \"bench\": $(grep '^{' /tmp/pw.log | tail -1)}" >> $out
  done
done
