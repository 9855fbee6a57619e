#!/usr/bin/env python
"""RCCL bus-bandwidth sweep over xGMI (nccl-tests style) + DDP bucket-size recommendation.

SURVEY.md 5.8 / 7.1 step 10: one ring of an 8x MI355X node is bound by ONE xGMI link
(~153 GB/s); full-mesh algorithms and enough channels reach several links.  The right DDP /
ZeRO bucket size is the knee of the busbw-vs-size curve on THIS fabric, not NVSwitch's or the
reference's PCIe T4 box (25 MiB default, data_parallel_training.py:71).

For each op (all_reduce, reduce_scatter_tensor, all_gather_into_tensor, all_to_all_single) and
each message size (powers of two between --min-bytes and --max-bytes) it runs --warmup untimed
and --iters timed collectives back to back on the current stream, timed with HIP events, takes
the MAX over ranks, and reports latency, algbw = bytes/t and busbw (all_reduce x 2(n-1)/n,
reduce_scatter / all_gather / all_to_all x (n-1)/n).  ``--recommend`` prints the smallest
all_reduce size that reaches 90% of the best busbw -- the bucket size to pass to
``data_parallel_training.py --bucket-size`` / ``bench.py --bucket-mb``.

  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench/comm_sweep.py --recommend
  python bench/comm_sweep.py --nproc 2 --backend gloo --max-bytes 1048576      # CPU rehearsal
Output: a table on rank 0 plus one JSON line per (op, size) with --json.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_training_and_deepspeed_amd import comm  # noqa: E402
from distributed_training_and_deepspeed_amd.launch import launch  # noqa: E402

OPS = ("all_reduce", "reduce_scatter_tensor", "all_gather_into_tensor", "all_to_all_single")
DTYPES = {"bf16": torch.bfloat16, "fp32": torch.float32}


def busbw_factor(op: str, n: int) -> float:
    if n <= 1:
        return 1.0
    return 2.0 * (n - 1) / n if op == "all_reduce" else (n - 1) / n


def sizes(lo: int, hi: int) -> list[int]:
    out, s = [], lo
    while s <= hi:
        out.append(s)
        s *= 2
    return out


def _run_op(op: str, buf: torch.Tensor, out: torch.Tensor | None):
    if op == "all_reduce":
        dist.all_reduce(buf)
    elif op == "reduce_scatter_tensor":
        dist.reduce_scatter_tensor(out, buf)
    elif op == "all_gather_into_tensor":
        dist.all_gather_into_tensor(out, buf)
    elif op == "all_to_all_single":
        dist.all_to_all_single(out, buf)
    else:
        raise ValueError(op)


def measure(op: str, nbytes: int, dtype: torch.dtype, device: torch.device, warmup: int, iters: int) -> dict:
    """Time ``iters`` back-to-back collectives of an ``nbytes`` message (the nccl-tests 'size':
    the full per-rank input for all_reduce / reduce_scatter / all_to_all, the gathered output
    for all_gather).  Returns the max-over-ranks per-op latency in ms and the bandwidths."""
    n = dist.get_world_size()
    es = torch.tensor([], dtype=dtype).element_size()
    numel = max(n, nbytes // es // n * n)
    if op == "all_gather_into_tensor":
        buf = torch.ones(numel // n, dtype=dtype, device=device)
        out = torch.empty(numel, dtype=dtype, device=device)
    elif op == "reduce_scatter_tensor":
        buf = torch.ones(numel, dtype=dtype, device=device)
        out = torch.empty(numel // n, dtype=dtype, device=device)
    elif op == "all_to_all_single":
        buf = torch.ones(numel, dtype=dtype, device=device)
        out = torch.empty(numel, dtype=dtype, device=device)
    else:
        buf, out = torch.ones(numel, dtype=dtype, device=device), None
    for _ in range(warmup):
        _run_op(op, buf, out)
    dist.barrier()
    cuda = device.type == "cuda"
    if cuda:
        torch.cuda.synchronize(device)
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
    else:
        start = time.perf_counter()
    for _ in range(iters):
        _run_op(op, buf, out)
    if cuda:
        t1.record()
        t1.synchronize()
        ms = t0.elapsed_time(t1) / iters
    else:
        ms = (time.perf_counter() - start) * 1e3 / iters
    t = torch.tensor([ms], dtype=torch.float64, device=device if cuda else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ms = t.item()
    size = numel * es
    algbw = size / (ms * 1e-3) / 1e9
    return {"op": op, "bytes": size, "dtype": str(dtype).replace("torch.", ""), "world": n, "ms": ms,
            "algbw_GBps": algbw, "busbw_GBps": algbw * busbw_factor(op, n)}


def recommend_bucket(rows: list[dict], frac: float = 0.9) -> dict | None:
    ar = sorted((r for r in rows if r["op"] == "all_reduce"), key=lambda r: r["bytes"])
    if not ar:
        return None
    best = max(r["busbw_GBps"] for r in ar)
    for r in ar:
        if r["busbw_GBps"] >= frac * best:
            return {"bucket_bytes": r["bytes"], "bucket_mb": r["bytes"] / 2 ** 20, "busbw_GBps": r["busbw_GBps"],
                    "peak_busbw_GBps": best, "fraction": frac}
    return None


def run(rank: int, world: int, a: argparse.Namespace):
    comm.init(rank=rank, world_size=world, backend=a.backend)
    cuda = dist.get_backend() == "nccl"
    device = torch.device("cuda", torch.cuda.current_device()) if cuda else torch.device("cpu")
    rows = []
    for op in a.ops.split(","):
        for sz in sizes(a.min_bytes, a.max_bytes):
            r = measure(op, sz, DTYPES[a.dtype], device, a.warmup, a.iters)
            rows.append(r)
            if rank == 0:
                if a.json:
                    print(json.dumps(r), flush=True)
                else:
                    print(f"{op:>24s} {r['bytes']:>12d} B  {r['ms'] * 1e3:10.1f} us  algbw {r['algbw_GBps']:8.2f} GB/s"
                          f"  busbw {r['busbw_GBps']:8.2f} GB/s", flush=True)
    if rank == 0 and a.recommend:
        rec = recommend_bucket(rows)
        print(json.dumps({"recommended_bucket": rec}), flush=True)
    if rank == 0 and a.out:
        with open(a.out, "w") as f:
            json.dump({"rows": rows, "recommended_bucket": recommend_bucket(rows)}, f, indent=1)
    comm.destroy()
    return rows


def parse(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--ops", default=",".join(OPS))
    p.add_argument("--dtype", choices=list(DTYPES), default="bf16")
    p.add_argument("--min-bytes", type=int, default=1 << 10)
    p.add_argument("--max-bytes", type=int, default=512 << 20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--backend", default=None, help="nccl (=RCCL) on GPUs, gloo on CPU")
    p.add_argument("--nproc", type=int, default=None, help="spawn this many local ranks (no torchrun)")
    p.add_argument("--recommend", action="store_true")
    p.add_argument("--json", action="store_true")
    p.add_argument("--out", default="")
    return p.parse_args(argv)


def main(argv=None):
    a = parse(argv)
    n = a.nproc or (torch.cuda.device_count() if torch.cuda.is_available() else 1)
    launch(run, args=(a,), nprocs=n)


if __name__ == "__main__":
    main()
