#!/usr/bin/env bash
# LayerNorm from-output backward with LDS-staged constants: tests, kernel timings, whole-step A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step ln_tests 300 python -u -m pytest tests/test_kernels_gpu.py -k "layernorm" -x -q --timeout 120 --timeout-method thread
step bench_ln 300 python scripts/bench_ln.py
step ab_ln 900 python scripts/ab.py base ln_memeff_off --rounds 3
echo done
