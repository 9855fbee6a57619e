#!/usr/bin/env bash
# Round 4 session 23: keep-mask generator with two interleaved xorshift chains per lane (ILP 2)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
DTD_ATTN_MASK_ILP=2 step tests_mask_ilp2 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_attention_gpu.py
step attn_ilp1 200 python -u scripts/bench_attn.py 3,2,3
DTD_ATTN_MASK_ILP=2 step attn_ilp2 200 python -u scripts/bench_attn.py 3,2,3
step ab_ilp 900 python scripts/ab.py base mask_ilp2 --rounds 3
echo done
