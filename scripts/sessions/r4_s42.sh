#!/usr/bin/env bash
# Round 4 session 42: standalone GEMM / copy rates do not change across RCCL init (s41), so is it
# the memory allocated after the communicator?  Init after the model / data, after the warm-up.
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step rccl_late 200 python bench.py --comm-init rccl-late
step rccl_after_warmup 200 python bench.py --comm-init rccl-after-warmup
step rccl 200 python bench.py --comm-init rccl
step base 200 python bench.py
echo done
