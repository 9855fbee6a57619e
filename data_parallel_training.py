#!/usr/bin/env python
"""BERT masked-LM data-parallel training (parity with the reference's data_parallel_training.py).

Reference behaviour kept: argparse flags and defaults
(--batch-size 4, --training-steps 1000, --device-count all GPUs, --bucket-size 25 MiB,
--model base|large), one process per device via spawn, a fixed dataset of
batch_size * training_steps samples sharded by DistributedSampler (strong scaling: each rank
runs training_steps / world batches), transformers.AdamW(lr=5e-5) hyper-parameters, and the
final "Total Training Time: X.XX seconds" line.

MI355X-first differences: synthetic MLM data with the HF masking law (no network), random
init, bf16 compute with fp32 master weights by default (--dtype fp32 for the reference's
numerics), the framework's fused HIP model and flat-bucket DDP over RCCL/xGMI, and a
tokens/s summary.  Runs on CPU/gloo too (use --model tiny).
"""
import argparse
import json
import os

# HIP hardware queues per process: the box default (4) is fewer than the streams of the N > 1
# step (compute, keep-mask, optimizer, finalize and RCCL's own); streams sharing a queue
# serialise their cross-stream waits.  Set to 8 before anything initialises HIP
# (docs/PERFORMANCE.md, "Hardware queues").
# The MI355X boxes export GPU_MAX_HW_QUEUES=4 themselves, so a value below 8 is raised (with a note
# on stderr) unless DTD_KEEP_HW_QUEUES=1 asks to keep it (A/B runs); the value in effect is logged.
# Keeping the boxes' 4 costs the N > 1 data path 17 % (profiles/r5_s12_results.jsonl).
_HWQ = os.environ.get("GPU_MAX_HW_QUEUES", "")
if os.environ.get("DTD_KEEP_HW_QUEUES") != "1" and (not _HWQ.isdigit() or int(_HWQ) < 8):
    if _HWQ:
        print(f"[dtd] GPU_MAX_HW_QUEUES={_HWQ} raised to 8 (DTD_KEEP_HW_QUEUES=1 keeps it)", file=__import__("sys").stderr)
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_training_and_deepspeed_amd import comm  # noqa: E402
from distributed_training_and_deepspeed_amd.data import DeviceBatchLoader, DistributedSampler, load_synthetic  # noqa: E402
from distributed_training_and_deepspeed_amd.launch import launch  # noqa: E402
from distributed_training_and_deepspeed_amd.models import build_model, get_config  # noqa: E402
from distributed_training_and_deepspeed_amd.optim import hf_adamw  # noqa: E402
from distributed_training_and_deepspeed_amd.parallel import DistributedDataParallel  # noqa: E402
from distributed_training_and_deepspeed_amd.utils import get_device_count  # noqa: E402
from distributed_training_and_deepspeed_amd.utils.checkpoint import load_checkpoint, save_checkpoint  # noqa: E402
from distributed_training_and_deepspeed_amd.utils.prewarm import prewarm_enabled, prewarm_model_kernels  # noqa: E402
from distributed_training_and_deepspeed_amd.utils.tracing import StepTimer, enable_markers, marker  # noqa: E402


def train(rank, world_size, batch_size, training_steps, bucket_size, model_name, opts):
    backend = opts.backend or ("nccl" if torch.cuda.is_available() else "gloo")
    if torch.cuda.is_available():
        from distributed_training_and_deepspeed_amd.utils.tuning import maybe_use_tuned_gemms
        maybe_use_tuned_gemms()   # measured hipBLASLt solutions (incl. this script's default shapes)
    if backend == "nccl" and prewarm_enabled():
        # the step's kernels run once before the RCCL communicator exists: kernels first launched
        # after it run 5-25 % slower for the life of the process (utils/prewarm.py)
        local = rank % max(1, get_device_count())
        torch.cuda.set_device(local)
        prewarm_model_kernels({"base": "bert-base-cased", "large": "bert-large-cased"}.get(model_name, model_name),
                              torch.device("cuda", local), dtype={"bf16": torch.bfloat16, "fp32": torch.float32}[opts.dtype],
                              impl=opts.impl, seq_len=opts.seq_len)
    comm.init(rank=rank, world_size=world_size, backend=backend, local_rank=rank % max(1, get_device_count()))
    cuda = backend == "nccl"
    device = torch.device("cuda", torch.cuda.current_device()) if cuda else torch.device("cpu")
    dtype = {"bf16": torch.bfloat16, "fp32": torch.float32}[opts.dtype]
    name = {"base": "bert-base-cased", "large": "bert-large-cased"}.get(model_name, model_name)
    cfg = get_config(name)
    model = build_model(name, dtype=dtype, device=device, seed=0, impl=opts.impl)
    model.train()
    model.rt.rng.reseed(rank)   # independent dropout masks per replica (parameters are broadcast)
    ddp = DistributedDataParallel(model, bucket_cap_mb=bucket_size,
                                  grad_dtype={"bf16": torch.bfloat16, "fp32": torch.float32}.get(opts.grad_dtype, dtype),
                                  force_collectives=opts.force_collectives)
    optimizer = hf_adamw(ddp.parameters(), lr=5e-5)
    if opts.resume:
        meta = load_checkpoint(opts.resume, model, optimizer)
        if rank == 0:
            print(f"resumed from {opts.resume} (step {meta['step']})")

    dataset = load_synthetic(cfg, batch_size * training_steps, seq_len=opts.seq_len, seed=0)
    sampler = DistributedSampler(dataset, num_replicas=world_size, rank=rank)
    loader = DeviceBatchLoader(dataset, batch_size=batch_size, sampler=sampler, device=device)

    progress = None
    if rank == 0 and not opts.quiet:
        try:
            from tqdm import tqdm
            progress = tqdm(range(training_steps))
        except ImportError:
            pass
    if opts.markers:
        enable_markers()
    def step(input_ids, labels):
        with marker("forward"):
            out = ddp(input_ids, labels=labels)
        with marker("backward+allreduce"):
            out.loss.backward()
        with marker("optimizer"):
            optimizer.step()
            optimizer.zero_grad()
            model.rt.rng.advance()
        return out.loss.detach()

    graphed, batches, warm, loss = None, iter(loader), [], None
    if opts.graph == "auto":
        # small per-GPU batches are host-launch bound: replay the whole step.  Only at world 1 by
        # default: a captured step with the bucket all-reduces inside it has been checked against
        # eager on one rank (tests/test_graph_gpu.py, force_collectives) but not yet replayed in
        # lockstep across ranks on a multi-GPU node; `--graph on` opts in at world > 1.
        opts.graph = "on" if (cuda and world_size == 1 and batch_size <= 32 and not opts.markers) else "off"
    if opts.graph == "on" and cuda:
        # whole step (forward, backward + bucket all-reduces, optimizer, RNG advance) replayed as
        # one hipGraph: the reference's 4 x 512-token batches are host-launch bound otherwise
        from distributed_training_and_deepspeed_amd.utils.graphs import CapturedStep, mlm_capacity
        model.rt.mlm_capacity = mlm_capacity(batch_size * opts.seq_len)
        warm = [b for _, b in zip(range(min(3, training_steps)), batches)]
        graphed = None if not warm else CapturedStep(step, warm[0], warmup_batches=warm, runtime=model.rt)
        loss = graphed.warmup_losses[-1] if graphed is not None else None
        if progress is not None:
            progress.update(len(warm))

    if opts.opt_overlap and graphed is None and cuda and hasattr(model, "zero3_units"):
        # eager steps: the Adam update of later stages overlaps the next forward (bit-identical);
        # opt-in: see the parameter-access contract of FusedAdam.overlap_with_forward
        optimizer.overlap_with_forward(model.zero3_units(), root=model)
    timer = StepTimer(batch_size * opts.seq_len, world_size)
    start = time.time()
    n = 0  # timed steps (graph warm-up steps trained before the clock started)
    for batch in batches:
        timer.start()
        if graphed is not None and batch["input_ids"].shape == graphed.static["input_ids"].shape:
            loss = graphed(input_ids=batch["input_ids"], labels=batch["labels"])
        else:
            loss = step(batch["input_ids"], batch["labels"])
        timer.stop()
        n += 1
        if progress is not None:
            progress.update(1)
    if cuda:
        torch.cuda.synchronize()
    elapsed = time.time() - start
    if graphed is not None:
        graphed.check()
    if opts.save_dir:
        save_checkpoint(os.path.join(opts.save_dir, "ddp_checkpoint.pt"), model, optimizer, step=n + len(warm))
    print(f"\nTotal Training Time: {elapsed:.2f} seconds")
    if rank == 0:
        tokens = n * batch_size * opts.seq_len * world_size
        print(json.dumps({"tokens_per_s": round(tokens / max(elapsed, 1e-9), 1), "steps_per_rank": n + len(warm), "timed_steps": n,
                          "world_size": world_size, "final_loss": round(float(loss.detach()), 4) if loss is not None else None}))
        if opts.metrics_json:
            timer.write(opts.metrics_json, {"model": name, "per_gpu_batch": batch_size, "seq_len": opts.seq_len,
                                            "bucket_mb": bucket_size, "world_size": world_size})
    comm.destroy()


if __name__ == "__main__":
    parser = argparse.ArgumentParser()
    parser.add_argument("--batch-size", type=int, default=4)
    parser.add_argument("--training-steps", type=int, default=1000)
    parser.add_argument("--device-count", type=int, default=None)
    parser.add_argument("--bucket-size", type=float, default=25)
    parser.add_argument("--model", type=str, default="base", help="base | large | tiny (or any preset)")
    parser.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    parser.add_argument("--grad-dtype", default=None, choices=[None, "bf16", "fp32"])
    parser.add_argument("--seq-len", type=int, default=512)
    parser.add_argument("--backend", default=None, choices=[None, "nccl", "gloo"])
    parser.add_argument("--impl", default="auto", choices=["auto", "fused", "reference"])
    parser.add_argument("--quiet", action="store_true")
    parser.add_argument("--force-collectives", action="store_true",
                        help="bucket all-reduces through RCCL even on one GPU (the N > 1 data path)")
    parser.add_argument("--metrics-json", default="", help="write tokens/s, step-time percentiles, peak HBM here")
    parser.add_argument("--markers", action="store_true", help="roctx ranges per phase (rocprofv3 --marker-trace)")
    parser.add_argument("--save-dir", default="", help="write <dir>/ddp_checkpoint.pt at the end")
    parser.add_argument("--resume", default="", help="checkpoint file to resume from")
    parser.add_argument("--opt-overlap", action="store_true",
                        help="stage the Adam update under the next forward (FusedAdam.overlap_with_forward)")
    parser.add_argument("--graph", nargs="?", const="on", default="auto", choices=["auto", "on", "off"],
                        help="capture the whole training step (bucket all-reduces included) in a hipGraph and "
                             "replay it (auto: on at <= 32 sequences per GPU, where the step is host-launch bound)")
    args = parser.parse_args()

    device_count = args.device_count or get_device_count()
    launch(train, args=(args.batch_size, args.training_steps, args.bucket_size, args.model, args),
           nprocs=device_count)
