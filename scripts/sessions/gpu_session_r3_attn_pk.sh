#!/usr/bin/env bash
# Packed-fp32 softmax forms of the attention forward and dQ kernels: numerics, timings, A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step attn_tests 400 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread
step bench_single 300 env B=256 python scripts/bench_attn.py 3,2,3
step bench_pk 300 env B=256 DTD_ATTN_FWD_PK=1 python scripts/bench_attn.py 3,2,3
step bench_single2 300 env B=256 python scripts/bench_attn.py 3,2,3
step bench_pk2 300 env B=256 DTD_ATTN_FWD_PK=1 python scripts/bench_attn.py 3,2,3
step ab 900 python scripts/ab.py base attn_pk wgrad_s8 --rounds 3
echo done
