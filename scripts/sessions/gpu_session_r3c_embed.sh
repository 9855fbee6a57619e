#!/usr/bin/env bash
# Embedding backward with 8 rows in flight per serial chunk step: per-kernel timing + bit-identity
# against the previous library (base_so), GPU kernel/model tests, whole-step A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
rm -f gpurun_out/session.log
OPS=$PWD/distributed_training_and_deepspeed_amd/ops
for r in 1 2; do
  step emb_new_$r 120 env T=131072 python -u scripts/bench_embed.py
  step emb_base_$r 120 env T=131072 DTD_KERNELS_SO=$OPS/_dtd_kernels_base.so python -u scripts/bench_embed.py
done
step tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py
step ab 800 python -u scripts/ab.py base base_so --rounds 3
echo done
