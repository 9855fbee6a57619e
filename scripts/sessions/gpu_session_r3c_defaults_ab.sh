#!/usr/bin/env bash
# Re-validate long-standing defaults against the round-3 kernels: same-box A/B, 3 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
rm -f gpurun_out/session.log
step ab 1150 python -u scripts/ab.py base gemm_wgrad no_defer_finalize opt_overlap_off ln_bwd_prefetch gemm_sched_static --rounds 3
echo done
