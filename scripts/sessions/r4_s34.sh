#!/usr/bin/env bash
# Round 4 session 34: the RCCL communicator's creation slows every later kernel of the process
# (s33: lazy group fast, created-then-destroyed still slow).  Which RCCL init feature: its VMM
# allocator, MSCCL / MSCCL++, P2P setup?  NCCL_DEBUG=INFO log of the init.
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,ALLOC,ENV step rccl_info 200 python bench.py --comm-init rccl --steps 5 --warmup 2
NCCL_CUMEM_ENABLE=0 step rccl_nocumem 200 python bench.py --comm-init rccl
RCCL_MSCCL_ENABLE=0 RCCL_MSCCLPP_ENABLE=0 step rccl_nomsccl 200 python bench.py --comm-init rccl
NCCL_P2P_DISABLE=1 NCCL_SHM_DISABLE=1 step rccl_nop2p 200 python bench.py --comm-init rccl
step rccl 200 python bench.py --comm-init rccl
step base 200 python bench.py
echo done
