#!/usr/bin/env bash
# Round 6: wgrad.hip below 8192 tokens (DTD_WGRAD_MIN_T) at the reference's small batches: b4
# graph bench and bloom-560m ZeRO-3 b1, interleaved.
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
for r in 1 2; do
  for t in 8192 512; do
    DTD_WGRAD_MIN_T=$t step wm_b4g_${t}_r$r 300 python bench.py --batch-size 4 --graph on --steps 200 --warmup 20
    DTD_WGRAD_MIN_T=$t MASTER_PORT=295$r${t:0:1} step wm_bloom_${t}_r$r 300 python zero_dp_training.py --stage 3 --quiet --no-memstats
  done
done
DTD_WGRAD_MIN_T=512 step wm_tests 300 python -u -m pytest tests/test_model_gpu.py -x -q -k "matches_reference or bitwise" --timeout 200 --timeout-method thread
echo done
