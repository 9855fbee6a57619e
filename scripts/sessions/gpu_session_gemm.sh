#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
step build 300 python -c "import __graft_entry__ as g; g.build()"
step pytest_gpu 900 python -m pytest tests -m gpu -q -x
step bench_gemm 400 python scripts/bench_gemm.py
step bench_b32 300 python bench.py --steps 10 --warmup 3 --batch-size 32
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results%d.csv PYTORCH_TUNABLEOP_VERBOSE=1
step bench_b32_tune 900 python bench.py --steps 10 --warmup 3 --batch-size 32
export PYTORCH_TUNABLEOP_TUNING=0
step bench_b32_tuned 300 python bench.py --steps 10 --warmup 3 --batch-size 32
echo done
