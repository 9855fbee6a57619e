#!/usr/bin/env bash
# Round 4 session 13: captured ZeRO-2/3 steps with RCCL collectives vs eager; DDP RCCL + optimizer
# overlap vs the local path; two ranks on one GPU in the bench configuration; then the step's
# knobs re-checked against the round-4 kernels (same box, interleaved)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step tests_rccl 600 python -u -m pytest -v --timeout 180 --timeout-method thread tests/test_graph_gpu.py tests/test_parallel_gpu.py -k "rccl or share_one_gpu"
step ab_knobs 1100 python scripts/ab.py base async_wgrad wgrad_s8 wgrad_s4 ln_bwd_prefetch gemm_sched_static no_defer_finalize attn_fwd_pipe attn_pk gemm_stagger2 --rounds 2
echo done
