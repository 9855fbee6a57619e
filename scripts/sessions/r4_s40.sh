#!/usr/bin/env bash
# Round 4 session 40: shader clock and L2 / HBM traffic of the small kernels with and without an
# initialised RCCL communicator (counters only: --pmc with --kernel-trace, no other trace domains)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
P="GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
step pmc_base 300 timeout -s KILL 280 rocprofv3 --kernel-trace --pmc $P -d gpurun_out/s40_base -o run --output-format csv -- python bench.py --steps 3 --warmup 2
python scripts/diag/pmc_small_kernels.py gpurun_out/s40_base/run_counter_collection.csv base > gpurun_out/s40_pmc.jsonl
step pmc_rccl 300 timeout -s KILL 280 rocprofv3 --kernel-trace --pmc $P -d gpurun_out/s40_rccl -o run --output-format csv -- python bench.py --comm-init rccl --steps 3 --warmup 2
python scripts/diag/pmc_small_kernels.py gpurun_out/s40_rccl/run_counter_collection.csv rccl >> gpurun_out/s40_pmc.jsonl
rm -rf gpurun_out/s40_base gpurun_out/s40_rccl
echo done
