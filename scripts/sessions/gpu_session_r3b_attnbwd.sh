#!/usr/bin/env bash
# dQ / dK-dV keep masks as scalar-loaded 64-bit lane masks: attention + model tests, bench_attn
# base (forward-only change) vs new, whole-step A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
OPS=$PWD/distributed_training_and_deepspeed_amd/ops
step pytest_attn 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread
for r in 1 2; do
  step attn_base_$r 200 env B=256 DTD_KERNELS_SO=$OPS/_dtd_kernels_base.so python -u scripts/bench_attn.py 3,2,3
  step attn_new_$r 200 env B=256 python -u scripts/bench_attn.py 3,2,3
done
step pytest_model 600 python -u -m pytest tests/test_model_gpu.py tests/test_graph_gpu.py -x -q --timeout 200 --timeout-method thread
step ab 900 python -u scripts/ab.py base_so base --rounds 3 -- --steps 12 --warmup 4
echo done
