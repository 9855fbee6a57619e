#!/usr/bin/env bash
# Round 4 session 29: what is left of the N>1 path's cost with 8 hardware queues -- kernel trace of
# bench.py --force-collectives, and RCCL channel caps (does a narrower all-reduce kernel disturb
# the co-running backward less at world 1?)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
step fc_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s29_fc -o run -- python bench.py --force-collectives --steps 5 --warmup 3
step fc_base 200 python bench.py --force-collectives
NCCL_MAX_NCHANNELS=4 step fc_ch4 200 python bench.py --force-collectives
NCCL_MAX_NCHANNELS=16 step fc_ch16 200 python bench.py --force-collectives
step fc_base2 200 python bench.py --force-collectives
echo done
