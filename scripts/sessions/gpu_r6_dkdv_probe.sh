#!/bin/bash
# (ran against the DTD_ATTN_DKDV_SB variants of commit cea4e37, reverted after this measurement)
# Round 6: price of the keep-mask handling in the dK/dV kernel: per-kernel times with dropout on /
# off, and the load-placement variants (DTD_ATTN_DKDV_SB), under a kernel trace.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
for v in "P=0.1 SB=0" "P=0.0 SB=0" "P=0.1 SB=1" "P=0.1 SB=2" "P=0.1 SB=0"; do
  set -- $v
  tag="${1#P=}_${2#SB=}"
  env $1 B=256 DTD_ATTN_DKDV_SB=${2#SB=} timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r6_dkdv/$tag -o run -- \
    python scripts/bench_attn.py 3,2,3 > gpurun_out/r6_dkdv_$tag.log 2>&1 || exit 1
done
