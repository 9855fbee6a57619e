#!/bin/bash
# Round 6: the in-process RCCL capture crash with a native backtrace and the HIP API log of the
# graph / capture / host-function calls (filtered on the box).
cd "$(dirname "$0")/../.."
DTD_SEGV_BT=1 AMD_LOG_LEVEL=3 DTD_RCCL_CAPTURE_INPROC=1 timeout -k 10 600 \
  python -u -m pytest tests/test_graph_gpu.py -v -s -k "rccl or zero" -p no:faulthandler \
  --timeout 240 --timeout-method thread > /tmp/graph_bt.out 2> /tmp/graph_bt.err
rc=$?
echo "rc=$rc" > gpurun_out/r6_graph_bt.txt
grep -E "PASSED|FAILED|segv_bt|^\[|\(\+0x|\) \[0x" /tmp/graph_bt.out >> gpurun_out/r6_graph_bt.txt
grep -E "segv_bt|\(\+0x|\) \[0x|Segmentation" /tmp/graph_bt.err >> gpurun_out/r6_graph_bt.txt
cat /tmp/graph_bt.out /tmp/graph_bt.err | grep -nE "Graph|Capture|HostFunc|UserObject|segv_bt|Segmentation" | tail -4000 > gpurun_out/r6_graph_api.txt
wc -l /tmp/graph_bt.err /tmp/graph_bt.out >> gpurun_out/r6_graph_bt.txt
tail -c 20000 /tmp/graph_bt.err > gpurun_out/r6_graph_err_tail.txt
exit $rc
