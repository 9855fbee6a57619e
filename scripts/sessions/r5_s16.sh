#!/usr/bin/env bash
# Round 5 session 16: bit-plane keep-mask generator (tests, isolated timing vs the round-4 form,
# whole-step A/B); mask over-read slack (S = 64); stage-per-process pipeline entry script
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step attn_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py
step mask_new 120 python -u scripts/bench_mask.py
DTD_KERNELS_SO=$PWD/distributed_training_and_deepspeed_amd/ops/_dtd_kernels_oldmask.so step mask_old 120 python -u scripts/bench_mask.py
DTD_DEBUG_SYNC=1 step stage_pipe 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_stage_pipeline_gpu.py
step ab_mask 1200 python -u scripts/ab.py base oldmask_so --rounds 3
echo done
