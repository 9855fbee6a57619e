#!/usr/bin/env bash
# Round 5 session 61: same-box A/B of the bf16 driver bench -- HEAD vs 30b71c1 (the tree before the
# fp32 GEMM work, a git worktree in ab_old/ with its own build), 3 interleaved rounds
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
for r in 1 2 3; do
  step head_$r 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
  step old_$r 400 bash -c "cd ab_old && python -u bench.py --gpus 1 --steps 20 --warmup 5"
done
echo done
