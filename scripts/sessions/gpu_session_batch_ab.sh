#!/usr/bin/env bash
# Same-box A/B of the bench's per-GPU batch: 256 (default) vs 384 vs 512, alternating runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
for r in 1 2 3; do
  for b in 256 384 512; do
    step "ab_b${b}_r${r}" 300 python bench.py --batch-size $b --steps 15 --warmup 4
  done
done
grep -h '"metric"' gpurun_out/ab_b*_r*.log > gpurun_out/batch_ab.jsonl
echo done
