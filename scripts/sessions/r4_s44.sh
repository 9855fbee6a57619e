#!/usr/bin/env bash
# Round 4 session 44: comm.init now loads the framework's code objects before creating the RCCL
# communicator (comm.prewarm_device_code).  N>1 path at world 1 with it / without it / with only a
# torch kernel loaded first; ZeRO-2 with collectives; the GPU tests that create RCCL groups.
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step fc 200 python bench.py --force-collectives
DTD_COMM_PREWARM=0 step fc_noprewarm 200 python bench.py --force-collectives
DTD_COMM_PREWARM=torch step fc_torchonly 200 python bench.py --force-collectives
step z2fc 200 python bench.py --zero-stage 2 --force-collectives
step base 200 python bench.py
step fc2 200 python bench.py --force-collectives
step tests 600 python -u -m pytest tests/test_parallel_gpu.py tests/test_graph_gpu.py -q -x --timeout 180 --timeout-method thread
echo done
