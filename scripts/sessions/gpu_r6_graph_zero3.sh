#!/bin/bash
# Round 6: (1) the RCCL capture tests in ONE process (thread_local capture mode, no watchdog sleep),
# (2) the max-params ZeRO-3 step with a kernel trace (only when (1) ended normally: pass or fail).
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
DTD_RCCL_CAPTURE_INPROC=1 timeout -k 10 600 python -u -m pytest tests/test_graph_gpu.py -v -k "rccl or zero" \
  --timeout 240 --timeout-method thread > gpurun_out/r6_graph_inproc.log 2>&1
rc=$?
echo "graph_inproc_rc=$rc" >> gpurun_out/r6_graph_inproc.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/r6_mp3 -o run -- \
  python bench/max_params.py --measure --stage 3 --steps 3 > gpurun_out/r6_mp3.log 2>&1
echo "mp3_rc=$?" >> gpurun_out/r6_mp3.log
