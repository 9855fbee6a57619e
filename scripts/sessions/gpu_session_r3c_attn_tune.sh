#!/usr/bin/env bash
# Attention launch-form re-tune after the SGPR keep-mask change: every existing instantiation
# (occupancy, dK/dV query tile, dQ key tile, packed-fp32 and pipelined forward) timed at the
# BERT-base b256 shape with dropout, two rounds in alternating order.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp B=256 P=0.1
rm -f gpurun_out/session.log
for r in 1 2; do
  step occ_$r 200 python -u scripts/bench_attn.py 3,2,3 2,2,3 3,1,3 3,2,2 1,1,1
  step bm64_$r 120 env DTD_ATTN_DKDV_BM=64 python -u scripts/bench_attn.py 3,2,3 3,1,3
  step dq128_$r 120 env DTD_ATTN_TILE=64,128 python -u scripts/bench_attn.py 3,2,3
  step pk_$r 120 env DTD_ATTN_FWD_PK=1 python -u scripts/bench_attn.py 3,2,3
  step pipe_$r 120 env DTD_ATTN_FWD=pipe python -u scripts/bench_attn.py 3,2,3
done
echo done
