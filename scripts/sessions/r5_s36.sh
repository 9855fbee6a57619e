#!/usr/bin/env bash
# Round 5 session 36: post-communicator kernel probe (ops/csrc/probe.hip) in bench.py's N > 1 path
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step probe_fc 300 python -u bench.py --force-collectives --steps 5 --warmup 2
step probe_fc_noprewarm 300 python -u bench.py --force-collectives --prewarm none --steps 5 --warmup 2
echo done
