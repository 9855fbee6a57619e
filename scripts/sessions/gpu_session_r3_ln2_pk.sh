#!/usr/bin/env bash
# LayerNorm from-output backward with LDS-staged constants + packed-fp32 softmax forms of the
# attention forward / dQ kernels: tests, kernel timings, whole-step A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step ln_tests 300 python -u -m pytest tests/test_kernels_gpu.py -k "layernorm" -x -q --timeout 120 --timeout-method thread
step attn_tests 400 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread
step bench_ln 300 python scripts/bench_ln.py
step bench_single 300 env B=256 python scripts/bench_attn.py 3,2,3
step bench_pk 300 env B=256 DTD_ATTN_FWD_PK=1 python scripts/bench_attn.py 3,2,3
step bench_single2 300 env B=256 python scripts/bench_attn.py 3,2,3
step bench_pk2 300 env B=256 DTD_ATTN_FWD_PK=1 python scripts/bench_attn.py 3,2,3
step bench_occ313 300 env B=256 DTD_ATTN_OCC=3,1,3 python scripts/bench_attn.py 3,1,3
step ab 900 python scripts/ab.py base attn_pk ln_memeff_off --rounds 3
echo done
