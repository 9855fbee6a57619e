#!/bin/bash
# Round 6: BERT-base b1024 step with the plain projections on gemm_w4.hip vs hipBLASLt (interleaved
# same-box A/B), then one kernel-trace profile of the w4 step.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
out=gpurun_out/r6_w4_step.jsonl
: > $out
for i in 1 2; do
  for w in 0 1; do
    DTD_GEMM_W4=$w timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r6_step_w$w.$i.log 2>&1 || exit 1
    echo "{\"run\": $i, \"DTD_GEMM_W4\": $w, \"bench\": $(grep '^{' gpurun_out/r6_step_w$w.$i.log | tail -1)}" >> $out
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r6_prof_w4 -o run -- python bench.py --steps 5 --warmup 2 > gpurun_out/r6_prof_w4.log 2>&1 || exit 1
python scripts/prof_summary.py $(find gpurun_out/r6_prof_w4 -name '*kernel_stats.csv' | head -1) 7 30 > gpurun_out/r6_kernel_summary_w4.txt
