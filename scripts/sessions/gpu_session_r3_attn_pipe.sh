#!/usr/bin/env bash
# Pipelined attention forward (S(t+1) MFMAs under softmax(t)): numerics + bitwise check, kernel
# timings single vs pipe, whole-step A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step attn_tests 400 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread
step bench_single 300 env B=256 python scripts/bench_attn.py 3,2,3
step bench_pipe 300 env B=256 DTD_ATTN_FWD=pipe python scripts/bench_attn.py 3,2,3
step bench_single2 300 env B=256 python scripts/bench_attn.py 3,2,3
step bench_pipe2 300 env B=256 DTD_ATTN_FWD=pipe python scripts/bench_attn.py 3,2,3
step ab 900 python scripts/ab.py base attn_fwd_pipe wgrad_s4 wgrad_s1 --rounds 2
echo done
