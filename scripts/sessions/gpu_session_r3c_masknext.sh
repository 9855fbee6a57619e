#!/usr/bin/env bash
# Next step's attention keep masks generated under this step's backward (DTD_MASK_NEXT=1):
# bit-identity tests, then whole-step A/B against front-loading at the forward start.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
rm -f gpurun_out/session.log
step next_tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_mask_prefetch_gpu.py
step model_tests 300 env DTD_MASK_NEXT=1 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_model_gpu.py tests/test_graph_gpu.py
step ab 900 python -u scripts/ab.py base mask_next --rounds 4
echo done
