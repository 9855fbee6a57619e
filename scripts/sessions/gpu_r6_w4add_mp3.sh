#!/bin/bash
# Round 6: gemm_w4 EPI_ADD (asm-prefetched residual rows) tests + bench, then the max-params ZeRO-3
# step under a kernel trace.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemm_w4_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/w4_test.log 2>&1 || exit 1
ONLY=dgrad_qkv_add,dgrad_fc1,fwd_qkv ROUNDS=3 timeout -k 10 300 python -u scripts/bench_gemm_w4.py > gpurun_out/r6_w4add.log 2>&1 || exit 1
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/r6_mp3 -o run -- \
  python bench/max_params.py --measure --stage 3 --steps 3 > gpurun_out/r6_mp3.log 2>&1
echo "mp3_rc=$?" >> gpurun_out/r6_mp3.log
