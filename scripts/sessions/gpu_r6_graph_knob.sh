#!/bin/bash
# Round 6: in-process RCCL capture crash -- HIP error log (level 2) and an optional env knob ($1)
cd "$(dirname "$0")/../.."
tag=${1:-base}
env $2 DTD_SEGV_BT=1 AMD_LOG_LEVEL=2 DTD_RCCL_CAPTURE_INPROC=1 timeout -k 10 600 \
  python -u -m pytest tests/test_graph_gpu.py -v -s -k "rccl or zero" -p no:faulthandler \
  --timeout 240 --timeout-method thread > /tmp/g.out 2> /tmp/g.err
rc=$?
{ echo "rc=$rc knob=$2"; grep -E "PASSED|FAILED" /tmp/g.out; grep -nE "Failed|parallel|segv_bt|rror" /tmp/g.err | head -50; } > gpurun_out/r6_graph_$tag.txt
exit $rc
