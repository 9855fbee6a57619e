#!/usr/bin/env bash
# Round 6: fused FFN kernels only from one 256x256 tile per CU (small batches on hipBLASLt + the
# activation kernel) vs always fused (DTD_GEMM_FFN_MIN_TILES=1): b4 graph bench and bloom-560m
# ZeRO-3 b1, interleaved; then the model GPU tests.
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
for r in 1 2; do
  for m in 1 0; do
    DTD_GEMM_FFN_MIN_TILES=$m step b4g_m${m}_r$r 300 python bench.py --batch-size 4 --graph on --steps 200 --warmup 20
    DTD_GEMM_FFN_MIN_TILES=$m MASTER_PORT=293$r$m step bloom_m${m}_r$r 300 python zero_dp_training.py --stage 3 --quiet --no-memstats
  done
done
step model_tests 600 python -u -m pytest tests/test_model_gpu.py tests/test_graph_gpu.py -x -q --timeout 200 --timeout-method thread
echo done
