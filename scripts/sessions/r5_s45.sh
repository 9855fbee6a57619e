#!/usr/bin/env bash
# Round 5 session 45: weight-gradient kernel LDS-DMA placement (groups 0-3 / odd groups / groups 4-7)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step wg_tests 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py -k "wgrad"
step wg_dpl 400 env ROUNDS=7 VARIANTS=44,46,48 python -u scripts/bench_wgrad.py
echo done
