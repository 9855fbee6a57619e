#!/usr/bin/env bash
# Round 5 session 65: elementwise / LayerNorm knobs re-checked at the b1024 default (tuned at b256):
# DTD_LN_BWD_PREFETCH=1 (software-pipelined LN backward, 3 waves/SIMD) and DTD_EW_MODE=1 (no
# non-temporal hints on the streaming passes), 2 interleaved rounds
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
for r in 1 2; do
  step base_$r 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
  step lnpf_$r 400 env DTD_LN_BWD_PREFETCH=1 python -u bench.py --gpus 1 --steps 20 --warmup 5
  step ew1_$r 400 env DTD_EW_MODE=1 python -u bench.py --gpus 1 --steps 20 --warmup 5
done
echo done
