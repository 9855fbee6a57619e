#!/bin/bash
# Round 6: ZeRO optimizer-under-backward: GPU bit-identity tests, then the max-params ZeRO-3 step
# with the overlap off / on, and a kernel trace of the overlapped step.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_parallel_gpu.py -x -q -k "overlapped or stages_on_gpu" --timeout 120 --timeout-method thread > gpurun_out/r6_zero_overlap_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench/max_params.py --measure --stage 3 --steps 4 --overlap-optimizer off > gpurun_out/r6_mp3_off.log 2>&1 || exit 1
timeout -k 10 300 python -u bench/max_params.py --measure --stage 3 --steps 4 --overlap-optimizer on > gpurun_out/r6_mp3_on.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r6_mp3ov -o run -- \
  python bench/max_params.py --measure --stage 3 --steps 2 > gpurun_out/r6_mp3ov_prof.log 2>&1
echo "prof_rc=$?" >> gpurun_out/r6_mp3ov_prof.log
