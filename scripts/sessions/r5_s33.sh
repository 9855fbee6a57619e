#!/usr/bin/env bash
# Round 5 session 33: what makes eager --async-wgrad degrade step by step (10 steps each)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step aw_base 200 python -u bench.py --async-wgrad on --steps 10 --warmup 1
DTD_KEEP_HW_QUEUES=1 GPU_MAX_HW_QUEUES=4 step aw_hwq4 200 python -u bench.py --async-wgrad on --steps 10 --warmup 1
GPU_MAX_HW_QUEUES=16 step aw_hwq16 200 python -u bench.py --async-wgrad on --steps 10 --warmup 1
step aw_nooptov 200 python -u bench.py --async-wgrad on --opt-overlap off --steps 10 --warmup 1
echo done
