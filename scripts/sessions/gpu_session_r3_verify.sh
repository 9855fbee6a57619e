#!/usr/bin/env bash
# Round-3 verification: GPU tests (ZeRO graphs at every stage, deferred-finalize no_sync), smoke,
# bench, N=8 rehearsal, ZeRO refresh overlap trace, reference ZeRO config with graphs, MP loss A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 300 python bench.py
step bench_zero2 300 python bench.py --zero-stage 2
step n8_rehearsal 600 python scripts/n8_rehearsal.py
step zero2_trace 300 rocprofv3 --kernel-trace -d gpurun_out/zero2_trace -o run --output-format csv -- python bench.py --zero-stage 2 --steps 3 --warmup 2
step zero_bloom_s2_graph 400 python zero_dp_training.py --stage 2 --training-steps 60 --no-memstats --quiet
step zero_bloom_s2_eager 400 python zero_dp_training.py --stage 2 --training-steps 60 --no-memstats --quiet --graph off
step zero_bloom_s3_graph 400 python zero_dp_training.py --stage 3 --training-steps 60 --no-memstats --quiet
step mp_fused 400 python model_parallel_training.py --training-steps 40 --devices cuda:0,cuda:0
step mp_torch 400 python model_parallel_training.py --training-steps 40 --devices cuda:0,cuda:0 --loss torch
echo done
