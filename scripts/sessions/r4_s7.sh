#!/usr/bin/env bash
# Round 4 session 7: ZeRO RCCL-at-world-1 tests; same-box A/B of the per-GPU batch and the dK/dV
# occupancy after the dS' rewrite.
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step tests_zero_rccl 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_parallel_gpu.py -k "rccl_collectives_at_world1"
step ab 900 python scripts/ab.py base b320 b384 dkdv_occ1 --rounds 2
echo done
