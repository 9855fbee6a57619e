#!/usr/bin/env bash
# Round 4 session 30: why the small memory-bound backward kernels (split-K reduce, column-sum
# finalize) run ~4x longer in most steps of the N>1 path at world 1 while nothing else runs on the
# GPU (profiles/r4_s29_fc_q8_kernels.txt) -- copy-engine traffic?  the staged optimizer?  clocks?
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step fc_copytrace 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/s30_fc -o run -- python bench.py --force-collectives --steps 8 --warmup 3
step base_trace 300 rocprofv3 --kernel-trace -d gpurun_out/s30_base -o run -- python bench.py --steps 8 --warmup 3
step fc_nooverlap 200 python bench.py --force-collectives --opt-overlap off
step base_nooverlap 200 python bench.py --opt-overlap off
HSA_ENABLE_SDMA=0 step fc_nosdma 200 python bench.py --force-collectives
TORCH_NCCL_ENABLE_MONITORING=0 step fc_nomon 200 python bench.py --force-collectives
step fc 200 python bench.py --force-collectives
echo done
