#!/usr/bin/env bash
# Round 4 session 9: fused projection + LayerNorm kernel -- numerics, then the standalone A/B
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step tests_gemm_ln 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_ln_gpu.py
DTD_GEMM_LN_PIPE=0 step bench_gemm_ln_p0 300 python -u scripts/bench_gemm_ln.py 131072 7
step bench_gemm_ln_p1 300 python -u scripts/bench_gemm_ln.py 131072 7
DTD_GEMM_LN_PIPE=0 DTD_GEMM_LN=1 step tests_gemm_ln_p0 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_ln_gpu.py -k "fp32 or unfused"
step ab_gemm_ln 600 python scripts/ab.py base gemm_ln gemm_ln_p0 --rounds 2
step capcoll 300 python -u scripts/diag/capture_collectives.py side_stream_rs autograd_rs autograd_side_stream_rs
step zerobisect 400 python -u scripts/diag/zero_capture_bisect.py s1_fwd_bwd_nostream s1_step_only_nostream s2_nostream
echo done
