#!/usr/bin/env bash
# attention kernel change: tests + kernel times vs the saved base .so (no bench A/B).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step tests 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/tests.log && ! grep -q "failed" gpurun_out/tests.log || exit 1
B=256 step attn_new 300 python -u scripts/bench_attn.py 3,2,3
B=256 DTD_KERNELS_SO=$PWD/distributed_training_and_deepspeed_amd/ops/_dtd_kernels_base.so step attn_old 300 python -u scripts/bench_attn.py 3,2,3
B=256 step attn_new2 300 python -u scripts/bench_attn.py 3,2,3
echo done
