#!/usr/bin/env bash
# Round 5 session 63: long-run stability at the b1024 default -- 20-step vs 200-step driver bench
# (a progressive slowdown or allocator growth would show as a lower long-run rate / higher peak),
# and the N > 1 data path (--force-collectives, real RCCL all-reduces at world 1) for 100 steps
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step bench20 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench200 600 python -u bench.py --gpus 1 --steps 200 --warmup 5
step fc100 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --steps 100 --warmup 5 --force-collectives
echo done
