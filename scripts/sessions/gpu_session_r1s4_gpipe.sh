#!/usr/bin/env bash
# GPipe on 288 GB: recompute (torch Pipe's except_last) vs keeping every micro-batch's activations.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
for m in bert-base-cased bert-large-cased; do
  for ck in except_last never; do
    step gpipe_${m}_${ck} 300 python model_parallel_training.py --model $m --devices cuda:0,cuda:0 --training-steps 60 --pipeline --checkpoint $ck
  done
  step gpipe_${m}_1f1b 300 python model_parallel_training.py --model $m --devices cuda:0,cuda:0 --training-steps 60 --pipeline --checkpoint never --schedule 1f1b
done
step prof_gpipe_never 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gpipe_never -o run --output-format csv -- python model_parallel_training.py --model bert-large-cased --devices cuda:0,cuda:0 --training-steps 10 --pipeline --checkpoint never
echo done
