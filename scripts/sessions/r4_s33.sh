#!/usr/bin/env bash
# Round 4 session 33: an initialised RCCL group alone costs the step ~10 % (s32).  Which part:
# the communicator (lazy group: none is created), sticky state (group destroyed before the model is
# built), or any process group (gloo)?
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step base 200 python bench.py
step rccl 200 python bench.py --comm-init rccl
step rccl_lazy 200 python bench.py --comm-init rccl-lazy
step rccl_destroy 200 python bench.py --comm-init rccl-destroy
step gloo 200 python bench.py --comm-init gloo
DTD_RCCL_HIGH_PRIORITY=0 step rccl_hp0 200 python bench.py --comm-init rccl
step base2 200 python bench.py
echo done
