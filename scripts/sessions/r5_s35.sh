#!/usr/bin/env bash
# Round 5 session 35: attention.hip without SLP vectorization (no packed per-score f32) and the
# scalar dK/dV form, vs the round-4 code generation (attnslp library + DTD_ATTN_DKDV_PK=1)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
SO=$PWD/distributed_training_and_deepspeed_amd/ops/_dtd_kernels_attnslp.so
step attn_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py
B=256 step battn_new1 200 python -u scripts/bench_attn.py 3,2,3
B=256 DTD_KERNELS_SO=$SO DTD_ATTN_DKDV_PK=1 step battn_slp1 200 python -u scripts/bench_attn.py 3,2,3
B=256 step battn_new2 200 python -u scripts/bench_attn.py 3,2,3
B=256 DTD_KERNELS_SO=$SO DTD_ATTN_DKDV_PK=1 step battn_slp2 200 python -u scripts/bench_attn.py 3,2,3
step ab_slp 900 python -u scripts/ab.py base attnslp_so --rounds 3
echo done
