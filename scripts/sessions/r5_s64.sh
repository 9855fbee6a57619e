#!/usr/bin/env bash
# Round 5 session 64: exposed share of the side-stream keep-mask generator at the b1024 default
# (generator launched twice per layer, DTD_ATTN_MASK_REPEAT=2), 3 interleaved rounds
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
for r in 1 2 3; do
  step base_$r 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
  step mask2_$r 400 env DTD_ATTN_MASK_REPEAT=2 python -u bench.py --gpus 1 --steps 20 --warmup 5
done
echo done
