#!/usr/bin/env bash
# Round 5 session 18: run-to-run determinism of the fused step (the staged-Adam bit-identity test
# failed in s17): base, staged optimizer, hand GEMMs off, round-4 mask generator
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step det_base 200 env VARIANT=base python -u scripts/diag/determinism.py
step det_overlap 200 env VARIANT=overlap OVERLAP=1 python -u scripts/diag/determinism.py
step det_nogemm 200 env VARIANT=nogemm DTD_GEMM=0 python -u scripts/diag/determinism.py
step det_oldmask 200 env VARIANT=oldmask DTD_KERNELS_SO=$PWD/distributed_training_and_deepspeed_amd/ops/_dtd_kernels_oldmask.so python -u scripts/diag/determinism.py
step det_nodrop 200 env VARIANT=base_b8 B=8 python -u scripts/diag/determinism.py
step staged_test 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_model_gpu.py -k staged_adam
echo done
