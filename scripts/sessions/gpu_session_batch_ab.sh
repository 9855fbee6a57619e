#!/usr/bin/env bash
# Same-box per-GPU batch A/B of the default bench (b256 vs b384), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
for r in 1 2 3; do
  step b256_$r 200 python bench.py --batch-size 256
  step b384_$r 200 python bench.py --batch-size 384
done
echo done
