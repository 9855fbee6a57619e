#!/usr/bin/env bash
# Round 5 session 43: wgrad size guard per K-range (b768 was refused); batches 512 / 768 / 1024
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step wgrad_tests 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py -k "wgrad or tn"
step c512 300 python -u bench.py --steps 8 --warmup 3
step c768 300 python -u bench.py --steps 8 --warmup 3 --batch-size 768
step c1024 400 python -u bench.py --steps 6 --warmup 2 --batch-size 1024
echo done
