#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
DBIAS=0 step bench_attn_nobias 300 python scripts/bench_attn.py 2,2,2
DBIAS=1 step bench_attn_bias 300 python scripts/bench_attn.py 2,2,2
DBIAS=1 step prof_attn 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_attn -o run --output-format csv -- python scripts/bench_attn.py 2,2,2
echo done
