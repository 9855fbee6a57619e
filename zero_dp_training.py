#!/usr/bin/env python
"""ZeRO stage 0-3 causal-LM training (parity with the reference's zero_dp_training.py).

Reference behaviour kept: flags --model-name (bigscience/bloom-560m),
--batch-size 1, --training-steps 100, --stage 0, unknown args tolerated (parse_known_args
swallows launcher-injected --local_rank); rank/world from LOCAL_RANK / WORLD_SIZE; the inline
DeepSpeed config (micro-batch, Adam lr 1.5e-4, comms_logger prof_all, zero_optimization
{stage, reduce_bucket_size 5e6}); the prints "Device r - ZeRO Stage: s", "Device r -
Optimizer: lr=..; betas=..; eps=..; parameter count=N" (N = local partition), per-step rank-0
MEMSTATS, "Total Training Time", the comms summary table and "Total Communication Latency".

MI355X-first: the framework's ZeRO engine (flat-buffer reduce-scatter / all-gather over RCCL
on a side stream, one fused-Adam launch per rank), fused HIP model kernels, bf16 by default,
synthetic causal-LM data (labels = input_ids, pads included, as util.py:54-58), random init.
Latency is reported in milliseconds (the reference's "seconds" label sums DeepSpeed's ms
values, quirk 12).

  torchrun --nproc-per-node 8 zero_dp_training.py --stage 2
  python zero_dp_training.py --num-gpus 2 --stage 3 --model-name facebook/opt-125m
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
from distributed_training_and_deepspeed_amd.comm import logger as dist_log  # noqa: E402
from distributed_training_and_deepspeed_amd.data import DeviceBatchLoader, DistributedSampler, load_synthetic  # noqa: E402
from distributed_training_and_deepspeed_amd.launch import launch  # noqa: E402
from distributed_training_and_deepspeed_amd.models import build_model, get_config  # noqa: E402
from distributed_training_and_deepspeed_amd.parallel.zero import initialize  # noqa: E402
from distributed_training_and_deepspeed_amd.profiling import memory_status  # noqa: E402
from distributed_training_and_deepspeed_amd.utils.prewarm import prewarm_enabled, prewarm_model_kernels  # noqa: E402


def train(model_name, batch_size, training_steps, stage, opts):
    rank = int(os.getenv("LOCAL_RANK", "0"))
    world_size = int(os.getenv("WORLD_SIZE", "1"))
    backend = opts.backend or ("nccl" if torch.cuda.is_available() else "gloo")
    if torch.cuda.is_available():
        from distributed_training_and_deepspeed_amd.utils.tuning import maybe_use_tuned_gemms
        maybe_use_tuned_gemms()   # measured hipBLASLt solutions (incl. this script's default shapes)
    if backend == "nccl" and prewarm_enabled():
        # the step's kernels run once before the RCCL communicator exists: kernels first launched
        # after it run 5-25 % slower for the life of the process (utils/prewarm.py)
        torch.cuda.set_device(rank)
        prewarm_model_kernels(model_name, torch.device("cuda", rank),
                              dtype={"bf16": torch.bfloat16, "fp32": torch.float32}[opts.dtype], impl=opts.impl,
                              seq_len=opts.seq_len, static_mlm=False)
    comm.init(backend=backend)
    cuda = backend == "nccl"
    device = torch.device("cuda", rank) if cuda else torch.device("cpu")
    dtype = {"bf16": torch.bfloat16, "fp32": torch.float32}[opts.dtype]
    cfg = get_config(model_name)
    model = build_model(model_name, dtype=dtype, device=device, seed=0, impl=opts.impl)

    if opts.graph == "auto":
        # at world > 1 eager by default: the run's comm-latency report (the comms logger times each
        # collective) is the script's output; --graph on captures the collectives too (untimed)
        opts.graph = "on" if (cuda and world_size == 1) else "off"
    # every stage is capturable: stage-2/3 gradient landing regions and stage-3 gathered units
    # live in persistent ring arenas (parallel/zero.py _Arena), so replays reuse one address set
    graph = opts.graph == "on" and cuda
    ds_config = {
        "train_micro_batch_size_per_gpu": batch_size,
        "optimizer": {"type": "Adam", "params": {"lr": 0.00015}},
        # per-collective event timing is not meaningful inside a replayed graph
        "comms_logger": {"enabled": not graph, "verbose": False, "prof_all": True, "debug": False},
        "zero_optimization": {"stage": stage, "reduce_bucket_size": opts.reduce_bucket_size},
        "bf16": {"enabled": dtype == torch.bfloat16},
    }
    model_engine, optimizer, _, _ = initialize(model=model, model_parameters=model.parameters(), config=ds_config)
    print(f"Device {rank} - ZeRO Stage: {model_engine.zero_optimization_stage()}")
    optimizer_state = optimizer.param_groups[0]
    print(f"Device {rank} - Optimizer: lr={optimizer_state['lr']}; "
          f"betas={optimizer_state['betas']}; eps={optimizer_state['eps']}; "
          f"parameter count={sum([torch.numel(p) for p in optimizer_state['params']]):,}")

    dataset = load_synthetic(cfg, batch_size * training_steps, seq_len=opts.seq_len, mlm=False, seed=0)
    sampler = DistributedSampler(dataset, num_replicas=world_size, rank=int(os.getenv("RANK", rank)))
    loader = DeviceBatchLoader(dataset, batch_size=batch_size, sampler=sampler, device=device)
    model_engine.train()
    dist_log.comms_logger.reset()  # only the training loop's collectives are summed below

    def train_step(input_ids, labels):
        outputs = model_engine(input_ids, labels=labels)
        model_engine.backward(outputs.loss)
        model_engine.step()
        return outputs.loss.detach()

    graphed, batches, warm = None, iter(loader), []
    if graph:
        # whole step (forward, backward + gradient reduction, fused Adam, parameter refresh,
        # dropout-RNG advance) replayed as one hipGraph: batch 1 x 512 is host-launch bound.
        # Captured before the clock starts (3 eager warm-up steps on the first batch, like
        # data_parallel_training.py --graph)
        from distributed_training_and_deepspeed_amd.utils.graphs import CapturedStep
        rt = getattr(model, "rt", None)
        if rt is not None and cfg.family == "bert":
            # the sparse MLM head gathers its labelled rows; the causal-LM data here (mlm=False)
            # labels every position, so a static gather of all of them keeps the step capturable
            rt.mlm_capacity = batch_size * opts.seq_len
        warm = [b for _, b in zip(range(min(3, training_steps)), batches)]
        graphed = None if not warm else CapturedStep(train_step, warm[0], warmup_batches=warm, runtime=getattr(model, "rt", None))
        loss = graphed.warmup_losses[-1] if graphed is not None else None
    start = time.time()
    progress = None
    if rank == 0 and not opts.quiet:
        try:
            from tqdm import tqdm
            progress = tqdm(range(training_steps))
            progress.update(len(warm))
        except ImportError:
            pass
    n = 0  # timed steps (graph warm-up steps trained before the clock started)
    for batch in batches:
        if graphed is not None and batch["input_ids"].shape == graphed.static["input_ids"].shape:
            loss = graphed(input_ids=batch["input_ids"], labels=batch["labels"])
        else:
            loss = train_step(batch["input_ids"], batch["labels"])
        n += 1
        if rank == 0:
            if not opts.no_memstats:
                memory_status("Memory stats after training step:")
            if progress is not None:
                progress.update(1)
    if cuda:
        torch.cuda.synchronize()
    elapsed = time.time() - start
    if rank == 0:
        print(f"\nTotal Training Time: {elapsed:.2f} seconds")
    total_comms_latency = dist_log.comms_logger.total_latency_ms()
    dist_log.log_summary()
    if rank == 0:
        print(f"\nTotal Communication Latency: {total_comms_latency:.2f} ms")
        tokens = n * batch_size * opts.seq_len * world_size
        print(json.dumps({"tokens_per_s": round(tokens / max(elapsed, 1e-9), 1), "stage": stage,
                          "partition_numel": model_engine.partition_numel(),
                          "final_loss": round(float(loss.detach()), 4), "hip_graph": graphed is not None}))
    comm.destroy()


def _spawned(rank, world, args):
    os.environ["LOCAL_RANK"] = str(rank)
    train(args.model_name, args.batch_size, args.training_steps, args.stage, args)


if __name__ == "__main__":
    parser = argparse.ArgumentParser()
    parser.add_argument("--model-name", type=str, default="bigscience/bloom-560m")
    parser.add_argument("--batch-size", type=int, default=1)
    parser.add_argument("--training-steps", type=int, default=100)
    parser.add_argument("--stage", type=int, default=0)
    parser.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    parser.add_argument("--seq-len", type=int, default=512)
    parser.add_argument("--reduce-bucket-size", type=float, default=5e6)
    parser.add_argument("--backend", default=None, choices=[None, "nccl", "gloo"])
    parser.add_argument("--impl", default="auto", choices=["auto", "fused", "reference"])
    parser.add_argument("--num-gpus", type=int, default=None, help="spawn locally (like `deepspeed --num_gpus`)")
    parser.add_argument("--no-memstats", action="store_true")
    parser.add_argument("--graph", nargs="?", const="on", default="auto", choices=["auto", "on", "off"],
                        help="capture the whole training step in a hipGraph and replay it, at any ZeRO stage "
                             "(auto: on for one GPU, where batch-1 steps are host-launch bound)")
    parser.add_argument("--quiet", action="store_true")
    args, extra_args = parser.parse_known_args()
    if args.num_gpus and "WORLD_SIZE" not in os.environ:
        launch(_spawned, args=(args,), nprocs=args.num_gpus)
    else:
        train(args.model_name, args.batch_size, args.training_steps, args.stage, args)
