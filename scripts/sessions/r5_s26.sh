#!/usr/bin/env bash
# Round 5 session 26: the captured-DDP-with-RCCL replay segfault: the case alone, then the failing
# subset with AMD_LOG_LEVEL=3 (tail kept) to name the last HIP call
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp

AMD_LOG_LEVEL=3 timeout -k 10 400 python -u -m pytest -s -x -v --timeout 200 --timeout-method thread tests/test_graph_gpu.py -k "rccl or zero" > gpurun_out/amdlog_full.txt 2>&1
echo "rc=$?" >> gpurun_out/session.log
tail -n 4000 gpurun_out/amdlog_full.txt > gpurun_out/amdlog_tail.txt
grep -n "PASSED\|FAILED\|Fatal" gpurun_out/amdlog_full.txt > gpurun_out/amdlog_tests.txt || true
rm -f gpurun_out/amdlog_full.txt
echo done
