#!/usr/bin/env bash
# qkv bias gradient from the attention-backward epilogues: tests, kernel times, bench A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step tests 400 python -u -m pytest tests/test_attention_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/tests.log && ! grep -q "failed" gpurun_out/tests.log || exit 1
B=256 step attn_new 300 python -u scripts/bench_attn.py 3,2,3
step ab 900 python -u scripts/ab.py base no_qkv_bias_fused --rounds 4
echo done
