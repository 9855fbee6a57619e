#!/usr/bin/env bash
# Round 5 session 32: weight gradients on a parallel branch inside a captured step (the eager
# --async-wgrad degrades step by step: 91 -> 203 -> 794 ms/step at 2 / 10 / 20 steps, s31)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step ab_graph_async 900 python -u scripts/ab.py base graph graph_async_wgrad --rounds 2
echo done
