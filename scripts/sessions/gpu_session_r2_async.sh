#!/usr/bin/env bash
# async weight-gradient stream vs single stream on the current kernels (default bench).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step ab 900 python -u scripts/ab.py base async_wgrad --rounds 4
echo done
