#!/usr/bin/env bash
# Round 6: stage-3 world-1 aliasing of the persistent buckets (bloom-560m's tied embedding) --
# ZeRO GPU tests, the reference's default ZeRO config before/after, and the LM-head split-K probe.
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
step zero_tests 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_parallel_gpu.py tests/test_graph_gpu.py -k "zero"
MASTER_PORT=29321 step bloom_z3_alias_r1 300 python zero_dp_training.py --stage 3 --quiet --no-memstats
MASTER_PORT=29322 step bloom_z3_alias_r2 300 python zero_dp_training.py --stage 3 --quiet --no-memstats
step splitk_test 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_head_splitk_gpu.py
MASTER_PORT=29323 DTD_HEAD_SPLITK=8 step bloom_z3_sk8_r1 300 python zero_dp_training.py --stage 3 --quiet --no-memstats
MASTER_PORT=29324 DTD_HEAD_SPLITK=16 step bloom_z3_sk16_r1 300 python zero_dp_training.py --stage 3 --quiet --no-memstats
MASTER_PORT=29325 DTD_HEAD_SPLITK=8 step bloom_z3_sk8_r2 300 python zero_dp_training.py --stage 3 --quiet --no-memstats
step splitk_head 240 python scripts/bench_splitk_head.py gpurun_out/splitk_head.json
echo done
