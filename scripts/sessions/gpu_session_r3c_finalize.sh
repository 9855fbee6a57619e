#!/usr/bin/env bash
# Column-sum finalize with 8 independent row chains per thread: kernel/model tests, per-kernel
# times (rocprofv3 --stats) new vs previous library, whole-step A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
rm -f gpurun_out/session.log
OPS=$PWD/distributed_training_and_deepspeed_amd/ops
step tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_graph_gpu.py
step prof_new 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fin_prof_new -o run --output-format csv -- python bench.py --steps 3 --warmup 1
( export DTD_KERNELS_SO=$OPS/_dtd_kernels_base.so; step prof_base 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fin_prof_base -o run --output-format csv -- python bench.py --steps 3 --warmup 1 ) || exit 99
step ab 800 python -u scripts/ab.py base base_so --rounds 3
echo done
