#!/usr/bin/env bash
# Round 4 session 27: hardware queues per process (GPU_MAX_HW_QUEUES, box default 4) vs the number
# of streams the step uses -- async weight gradients, default, and the N>1 path (force collectives)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
GPU_MAX_HW_QUEUES=8 step async_q8 240 python bench.py --async-wgrad on --steps 10 --warmup 3
GPU_MAX_HW_QUEUES=16 step async_q16 240 python bench.py --async-wgrad on --steps 10 --warmup 3
step base_q4 240 python bench.py
GPU_MAX_HW_QUEUES=8 step base_q8 240 python bench.py
step fc_q4 240 python bench.py --force-collectives
GPU_MAX_HW_QUEUES=8 step fc_q8 240 python bench.py --force-collectives
GPU_MAX_HW_QUEUES=16 step fc_q16 240 python bench.py --force-collectives
echo done
