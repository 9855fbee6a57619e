#!/bin/bash
# Round 6: stage-per-process GPipe, 2 ranks on the one GPU over gloo (activations staged through host
# memory: the transfer is comparable to the compute), posted receives + non-blocking sends vs the
# blocking form, interleaved.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
out=gpurun_out/r6_pipe_overlap.jsonl
: > $out
i=0
for r in 1 2; do
  for ov in off on; do
    i=$((i+1))
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port $((29760 + i)) model_parallel_training.py --pipeline --model bert-base-cased --batch-size 16 \
      --training-steps 12 --micro-batch-count 4 --pipe-backend gloo --pipe-overlap $ov > /tmp/po.log 2>&1 || { tail -20 /tmp/po.log; exit 1; }
    echo "{\"round\": $r, \"overlap\": \"$ov\", \"result\": $(grep '^{' /tmp/po.log | tail -1)}" >> $out
  done
done
