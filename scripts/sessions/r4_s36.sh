#!/usr/bin/env bash
# Round 4 session 36: which allocation of RCCL's init slows the later kernels -- its 512 MB uncached
# device buffer (flags 3 in the s34 log), a fine-grained one, or pinned host memory?
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step uncached 200 python bench.py --comm-init uncached
step finegrained 200 python bench.py --comm-init finegrained
step hostmem 200 python bench.py --comm-init hostmem
step base 200 python bench.py
step rccl 200 python bench.py --comm-init rccl
echo done
