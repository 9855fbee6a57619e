#!/usr/bin/env bash
# Round 6: batched gradient finalizes -- GPU suite, then b4 graph / bloom b1 / b1024 with batching
# off (DTD_FINALIZE_BATCH=0) and on, interleaved.
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
step gpu_suite 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
for r in 1 2; do
  for fb in 0 1; do
    DTD_FINALIZE_BATCH=$fb step fb_b4g_${fb}_r$r 300 python bench.py --batch-size 4 --graph on --steps 200 --warmup 20
    DTD_FINALIZE_BATCH=$fb MASTER_PORT=294$r$fb step fb_bloom_${fb}_r$r 300 python zero_dp_training.py --stage 3 --quiet --no-memstats
  done
done
for fb in 0 1; do
  DTD_FINALIZE_BATCH=$fb step fb_b1024_$fb 300 python bench.py --steps 10 --warmup 3
done
echo done
