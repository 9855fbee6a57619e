#!/usr/bin/env bash
# Round 4 session 14: re-check the step's knobs against the round-4 kernels (same box, interleaved)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step tests_new 300 python -u -m pytest -v --timeout 180 --timeout-method thread tests/test_parallel_gpu.py -k "share_one_gpu or rccl_bucket"
step ab_knobs 1100 python scripts/ab.py base async_wgrad wgrad_s8 wgrad_s4 ln_bwd_prefetch gemm_sched_static no_defer_finalize attn_fwd_pipe attn_pk gemm_stagger2 --rounds 2
echo done
