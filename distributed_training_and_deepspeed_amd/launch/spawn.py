"""Single-node process launch (``torch.multiprocessing.spawn`` parity + torchrun compatibility).

Reference: ``mp.spawn(train, args=(...), nprocs=device_count, join=True)``
(data_parallel_training.py:76-81, pytorch_allreduce.py:36-38).  Two entry modes:

* ``launch(fn, args, nprocs)`` from a plain ``python script.py``: spawns one process per GPU,
  exporting the torchrun env contract (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT)
  so every rank initialises identically; ``join=True`` propagates the first child failure and
  terminates the siblings (fail-fast).
* under ``torchrun`` / the multinode launcher (env already present): ``fn`` runs in-process as
  rank ``RANK`` -- the same script works either way.
"""
from __future__ import annotations

import os
import socket

import torch.multiprocessing as mp


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _child(local_rank: int, fn, world: int, master_addr: str, master_port: int, args: tuple):
    os.environ.update({"RANK": str(local_rank), "LOCAL_RANK": str(local_rank), "WORLD_SIZE": str(world),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": master_addr, "MASTER_PORT": str(master_port)})
    fn(local_rank, world, *args)


def under_launcher() -> bool:
    return "RANK" in os.environ and "WORLD_SIZE" in os.environ and "MASTER_ADDR" in os.environ


def launch(fn, args: tuple = (), nprocs: int = 1, master_addr: str = "127.0.0.1", master_port: int | None = None,
           join: bool = True):
    """Run ``fn(rank, world_size, *args)`` on ``nprocs`` local ranks (or in-process under torchrun)."""
    if under_launcher():
        return fn(int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), *args)
    port = master_port or int(os.environ.get("MASTER_PORT", 0)) or free_port()
    if nprocs == 1:
        return _child(0, fn, 1, master_addr, port, args)
    return mp.spawn(_child, args=(fn, nprocs, master_addr, port, args), nprocs=nprocs, join=join)
