#!/usr/bin/env bash
# Per-kernel times of the word-embedding backward, new vs previous library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
rm -f gpurun_out/session.log
OPS=$PWD/distributed_training_and_deepspeed_amd/ops
step prof_new 120 rocprofv3 --kernel-trace --stats -d gpurun_out/emb_prof_new -o run --output-format csv -- python scripts/bench_embed.py
export DTD_KERNELS_SO=$OPS/_dtd_kernels_base.so
step prof_base 120 rocprofv3 --kernel-trace --stats -d gpurun_out/emb_prof_base -o run --output-format csv -- python scripts/bench_embed.py
echo done
