#!/usr/bin/env python
"""All-reduce demo (parity with the reference's pytorch_allreduce.py).

Each rank builds an int64[3] tensor (rank 0 [1,2,3], rank 1 [10,20,30], rank 2 [4,5,6]; extra
ranks r use [r, 2r, 3r]) and sums it across ranks with one all-reduce -- RCCL over xGMI on
MI355X (torch backend "nccl"), gloo on CPU or when there are more ranks than GPUs.  With the
reference's 3 ranks every rank ends with [15, 27, 39].

  python pytorch_allreduce.py [--world-size 3] [--backend rccl|gloo]
"""
import argparse
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_training_and_deepspeed_amd import comm  # noqa: E402
from distributed_training_and_deepspeed_amd.launch import launch  # noqa: E402

INIT = {0: [1, 2, 3], 1: [10, 20, 30], 2: [4, 5, 6]}


def rank_tensor(rank: int) -> torch.Tensor:
    return torch.tensor(INIT.get(rank, [rank, 2 * rank, 3 * rank]))


def all_reduce_example(rank: int, world_size: int, backend: str | None = None):
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() and torch.cuda.device_count() >= world_size else "gloo"
    comm.init(rank=rank, world_size=world_size, backend=backend, local_rank=rank)
    device = torch.device("cuda", rank) if backend == "nccl" else torch.device("cpu")
    tensor = rank_tensor(rank).to(device)
    print("Before AllReduce: Rank ", rank, " has data ", tensor, flush=True)
    dist.all_reduce(tensor, op=dist.ReduceOp.SUM)
    print("After AllReduce:  Rank ", rank, " has data ", tensor, flush=True)
    comm.destroy()
    return tensor.cpu()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world-size", type=int, default=3)
    ap.add_argument("--backend", default=None, choices=[None, "rccl", "nccl", "gloo"])
    a = ap.parse_args()
    backend = "nccl" if a.backend == "rccl" else a.backend
    launch(all_reduce_example, args=(backend,), nprocs=a.world_size)


if __name__ == "__main__":
    main()
