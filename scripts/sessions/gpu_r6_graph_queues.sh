#!/bin/bash
# Round 6: cost of single-queue graph replay (DEBUG_HIP_FORCE_GRAPH_QUEUES=1, the workaround for the
# HIP runtime's parallel-stream overrun in hipGraphLaunch) on the captured b4 steps, same box, fresh
# processes, interleaved.
cd "$(dirname "$0")/../.."
out=gpurun_out/r6_graph_queues.jsonl
: > $out
for i in 1 2; do
  for q in default 1; do
    for fc in "" "--force-collectives"; do
      if [ $q = default ]; then e=""; else e="DEBUG_HIP_FORCE_GRAPH_QUEUES=1"; fi
      env $e timeout -k 10 300 python bench.py --batch-size 4 --graph on --steps 200 --warmup 20 $fc > /tmp/b.log 2>&1 || exit 1
      echo "{\"run\": $i, \"queues\": \"$q\", \"fc\": \"$fc\", \"bench\": $(grep '^{' /tmp/b.log | tail -1)}" >> $out
    done
  done
done
