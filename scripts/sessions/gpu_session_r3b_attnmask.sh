#!/usr/bin/env bash
# Attention forward keep masks as scalar-loaded 64-bit lane masks (one v_cndmask per score):
# tests under the default (v2: first block's masks loaded before the softmax) and v1 (loads just
# before the selects), bench_attn base / v2 / v1, whole-step A/B against the base build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
OPS=$PWD/distributed_training_and_deepspeed_amd/ops
step pytest_attn 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread
step pytest_attn_v1 300 env DTD_KERNELS_SO=$OPS/_dtd_kernels_attnv1.so python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread
for r in 1 2; do
  step attn_base_$r 200 env B=256 DTD_KERNELS_SO=$OPS/_dtd_kernels_base.so python -u scripts/bench_attn.py 3,2,3
  step attn_v2_$r 200 env B=256 python -u scripts/bench_attn.py 3,2,3
  step attn_v1_$r 200 env B=256 DTD_KERNELS_SO=$OPS/_dtd_kernels_attnv1.so python -u scripts/bench_attn.py 3,2,3
done
step pytest_model 600 python -u -m pytest tests/test_model_gpu.py tests/test_graph_gpu.py -x -q --timeout 200 --timeout-method thread
step ab 900 python -u scripts/ab.py base_so base --rounds 3 -- --steps 12 --warmup 4
echo done
