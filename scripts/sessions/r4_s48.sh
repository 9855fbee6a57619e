#!/usr/bin/env bash
# Round 4 session 48: does the plain 1-GPU step (no RCCL group) also gain from running the model's
# kernels once at batch 1 before the real model is built?  Interleaved A/B.
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step base 200 python bench.py
step base_pw 200 python bench.py --prewarm layer1
step base_b 200 python bench.py
step base_pw_b 200 python bench.py --prewarm layer1
echo done
