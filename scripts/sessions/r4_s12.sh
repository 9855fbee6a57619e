#!/usr/bin/env bash
# Round 4 session 12: closing verification on the committed tree -- full GPU suite, smoke, the
# default bench, a kernel-trace summary of the default step, bloom-560m ZeRO 0/3 at the reference
# defaults; last, the ZeRO capture bisect with collectives on the capture stream.
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step pytest_gpu 1000 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 300 python bench.py
step prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s12 -o run -- python bench.py --steps 5 --warmup 2
export MASTER_ADDR=127.0.0.1
MASTER_PORT=29901 step bloom_z0 300 python zero_dp_training.py --stage 0 --quiet --no-memstats
MASTER_PORT=29902 step bloom_z3 300 python zero_dp_training.py --stage 3 --quiet --no-memstats
step zerobisect 600 python -u scripts/diag/zero_capture_bisect.py s1_fwd_only s1_fwd_bwd_only s1_step_only s1 s2 s3 s2_no_overlap_comm s2_one_bucket
echo done
