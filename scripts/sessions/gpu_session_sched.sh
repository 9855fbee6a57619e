cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step gemm_tests 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread
step sched_bench 300 python -u scripts/bench_gemm_sched.py
step b_dyn1 200 python bench.py
step b_sta1 200 env DTD_GEMM_SCHED=static python bench.py
step b_dyn2 200 python bench.py
step b_sta2 200 env DTD_GEMM_SCHED=static python bench.py
echo done
