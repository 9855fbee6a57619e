#!/usr/bin/env bash
# Tune the NT-form input-gradient GEMM shapes missing from the TunableOp table, then A/B the
# merged table against the current one on the whole step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
rm -f gpurun_out/session.log
step tune 600 python -u scripts/dgrad_tune.py
step ab 700 python -u scripts/ab.py base dgrad_table --rounds 3
echo done
