#!/usr/bin/env bash
# Attention-dropout mask generator: transpose variant vs ballot/writelane variant, bits + time.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step tests 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/tests.log && ! grep -q "failed" gpurun_out/tests.log || exit 1
step mask_t 120 python -u scripts/bench_mask.py
DTD_ATTN_MASK=0 step mask_b 120 python -u scripts/bench_mask.py
S=200 B=64 step mask_t2 120 python -u scripts/bench_mask.py
S=200 B=64 DTD_ATTN_MASK=0 step mask_b2 120 python -u scripts/bench_mask.py
step ab 900 python -u scripts/ab.py base mask_ballot --rounds 4
echo done
