#!/usr/bin/env python
"""BERT model-parallel / GPipe training (parity with the reference's model_parallel_training.py).

Reference behaviour kept: flags --pipeline, --verbose,
--batch-size 16, --training-steps 250, --device-count (all GPUs), --micro-batch-count 4;
single process driving several GPUs; BertModelWithMP (bert-base-cased config, random init,
untied MLM head) placed with the np.array_split law; ``to_pipeline(chunks)`` for GPipe;
AdamW(lr=5e-5) with torch defaults (eps 1e-8, wd 0.01); CrossEntropyLoss over [-1, vocab]
on the head device; shuffled batches; "Total Training Time" and the fancy_grid table
"Average Idle Time per Device".

MI355X-first: activations cross devices on copy streams over xGMI, idle time is measured
with HIP events on each device's stream (``--timing host`` for the reference's host clocks),
fused HIP layers, bf16 by default, synthetic MLM data.  ``--devices cuda:0,cuda:0`` runs two
pipeline stages on one GPU (schedule check on a single-GPU machine).
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

from distributed_training_and_deepspeed_amd.data import DeviceBatchLoader, load_synthetic  # noqa: E402
from distributed_training_and_deepspeed_amd.models import get_config  # noqa: E402
from distributed_training_and_deepspeed_amd.models.bert_mp import BertModelWithMP  # noqa: E402
from distributed_training_and_deepspeed_amd.ops import functional as Fx  # noqa: E402
from distributed_training_and_deepspeed_amd.optim import PerDeviceOptimizer, torch_adamw  # noqa: E402


def _flat(logits: torch.Tensor, upcast: bool) -> torch.Tensor:
    out = logits.view(-1, logits.shape[-1])
    return out.float() if upcast else out


def summarize_idle_time(bert: BertModelWithMP, training_steps: int):
    rows = bert.tracker.table(training_steps)
    try:
        from tabulate import tabulate
        print(tabulate(rows, headers="firstrow", floatfmt=".2f", tablefmt="fancy_grid"))
    except ImportError:
        for r in rows:
            print(*r, sep="\t")
    return rows


def main():
    parser = argparse.ArgumentParser()
    parser.add_argument("--pipeline", action="store_true")
    parser.add_argument("--verbose", action="store_true")
    parser.add_argument("--batch-size", type=int, default=16)
    parser.add_argument("--training-steps", type=int, default=250)
    parser.add_argument("--device-count", type=int, default=None)
    parser.add_argument("--micro-batch-count", type=int, default=4)
    parser.add_argument("--model", default="bert-base-cased")
    parser.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    parser.add_argument("--seq-len", type=int, default=512)
    parser.add_argument("--devices", default=None, help="explicit stage devices, e.g. cuda:0,cuda:1")
    parser.add_argument("--timing", default="device", choices=["device", "host"])
    parser.add_argument("--checkpoint", default="auto", choices=["auto", "except_last", "always", "never"],
                        help="GPipe activation recompute. auto: 'never' when every stage device has >= 64 GB "
                             "(MI355X: 288 GB holds all micro-batches' activations; recompute cost +50%% step "
                             "time, profiles/r1_gpipe_recompute.jsonl), else torch Pipe's 'except_last'")
    parser.add_argument("--impl", default="auto", choices=["auto", "fused", "reference"])
    parser.add_argument("--schedule", default="gpipe", choices=["gpipe", "1f1b"],
                        help="pipeline schedule: torch-Pipe fill-drain (reference) or 1F1B (S live micro-batches)")
    parser.add_argument("--loss", default="fused", choices=["fused", "torch"],
                        help="fused: bf16 softmax-CE kernel; torch: CrossEntropyLoss on fp32-upcast logits")
    parser.add_argument("--graph", nargs="?", const="on", default="auto", choices=["auto", "on", "off"],
                        help="replay the whole step (every stage's micro-batch forwards and backwards, loss, "
                             "optimizer) as one hipGraph when all stages share one GPU; auto: on then, unless "
                             "--verbose (whose per-hook prints need eager steps)")
    parser.add_argument("--pipe-overlap", default="on", choices=["on", "off"],
                        help="stage-per-process: off = the blocking send/recv form (a GPipe measurement baseline)")
    parser.add_argument("--pipe-backend", default="auto", choices=["auto", "rccl", "gloo"],
                        help="stage-per-process mode (launched with several ranks): the point-to-point "
                             "transport; auto = RCCL on GPUs, gloo on CPU")
    args = parser.parse_args()
    if torch.cuda.is_available():
        from distributed_training_and_deepspeed_amd.utils.tuning import maybe_use_tuned_gemms
        maybe_use_tuned_gemms()   # measured hipBLASLt solutions
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        return main_stage_per_process(args)

    config = get_config(args.model)
    dtype = {"bf16": torch.bfloat16, "fp32": torch.float32}[args.dtype]
    devices = args.devices.split(",") if args.devices else None
    bert = BertModelWithMP(config=config, device_count=args.device_count, verbose=args.verbose, devices=devices,
                           dtype=dtype, impl=args.impl, timing=args.timing)
    if args.checkpoint == "auto":
        big = all(d.type == "cuda" and torch.cuda.get_device_properties(d).total_memory >= 64 * 2 ** 30
                  for d in bert.group_devices)
        args.checkpoint = "never" if big else "except_last"
    model = bert.to_pipeline(chunks=args.micro_batch_count, checkpoint=args.checkpoint) if args.pipeline else bert

    optimizer = PerDeviceOptimizer(model.parameters(), torch_adamw, lr=5e-5)
    # fused softmax-CE on the head stage's bf16 logits (ops/csrc/xent.hip): no fp32 up-cast of the
    # [b*s, vocab] logits (the reference's CrossEntropyLoss over .float() logits: 950 MB at b16)
    loss_fn = Fx.CrossEntropyLoss() if args.loss == "fused" else torch.nn.CrossEntropyLoss().to(bert.head_device)
    upcast = args.loss != "fused"
    dataset = load_synthetic(config, args.batch_size * args.training_steps, seq_len=args.seq_len, seed=0)
    g = torch.Generator().manual_seed(0)
    sampler = torch.randperm(len(dataset), generator=g).tolist()  # DataLoader(shuffle=True)
    loader = DeviceBatchLoader(dataset, batch_size=args.batch_size, sampler=sampler, device=bert.embedding_device)
    model.train()

    def step(input_ids, labels):
        if args.pipeline and args.schedule == "1f1b":
            loss = model.train_step(input_ids, labels, lambda out, t: loss_fn(_flat(out, upcast), t.view(-1)),
                                    schedule="1f1b")
        else:
            outputs = model(input_ids)
            loss = loss_fn(_flat(outputs, upcast), labels.to(bert.head_device).view(-1))
            loss.backward()
        optimizer.step()
        optimizer.zero_grad()
        bert.advance_rng()
        return loss.detach()

    # One GPU holding every stage (virtual stages): the step is a fixed sequence of kernels on one
    # device, so it is captured once and replayed -- the b16 / 4-micro-batch step is otherwise bound
    # by the host issuing ~10^4 small launches.  Stages on distinct GPUs stay eager.
    one_gpu = len({str(d) for d in bert.group_devices}) == 1 and bert.group_devices[0].type == "cuda"
    if args.graph == "auto":
        args.graph = "on" if one_gpu and not args.verbose else "off"
    if args.graph == "on" and not one_gpu:
        print("--graph: stages on several devices of one process run eagerly; launch one process per "
              "stage (torchrun --nproc-per-node S) for a hipGraph per stage")
        args.graph = "off"
    batches = iter(loader)
    graphed, warm, n, loss = None, [], 0, None
    if args.graph == "on":
        from distributed_training_and_deepspeed_amd.utils.graphs import CapturedStep
        bert.tracker.enabled = False
        warm = [b for _, b in zip(range(min(3, args.training_steps)), batches)]
        if warm:
            graphed = CapturedStep(step, {"input_ids": warm[0]["input_ids"], "labels": warm[0]["labels"]},
                                   warmup_batches=[{"input_ids": b["input_ids"], "labels": b["labels"]}
                                                   for b in warm])
            loss = graphed.warmup_losses[-1]

    start = time.time()
    progress = None
    if not args.verbose:
        try:
            from tqdm import tqdm
            progress = tqdm(range(args.training_steps))
        except ImportError:
            pass
    if progress is not None and warm:
        progress.update(len(warm))
    for batch in batches:
        if graphed is not None and batch["input_ids"].shape == graphed.static["input_ids"].shape:
            loss = graphed(input_ids=batch["input_ids"], labels=batch["labels"])
        else:
            loss = step(batch["input_ids"], batch["labels"])
        bert.step_boundary()
        n += 1
        if progress is not None:
            progress.update(1)
    for d in set(bert.group_devices):
        if d.type == "cuda":
            torch.cuda.synchronize(d)
    elapsed = time.time() - start
    print(f"\nTotal Training Time: {elapsed:.2f} seconds")
    print("\nAverage Idle Time per Device:")
    if graphed is not None:
        # a replayed graph records no per-stage activity marks: the idle time is not measured
        print("(hipGraph replay: the stages' kernels run back to back on one device; no per-stage idle events)")
        rows = [["Device", "Avg Idle Time (ms)"]] + [[i, "n/a (graph)"] for i in range(len(bert.group_devices))]
        print("\n".join(f"{r[0]}\t{r[1]}" for r in rows))
    else:
        rows = summarize_idle_time(bert, max(n, 1))
    print(json.dumps({"tokens_per_s": round(n * args.batch_size * args.seq_len / max(elapsed, 1e-9), 1),
                      "timed_steps": n, "graph": graphed is not None,
                      "pipeline": args.pipeline, "stages": len(bert.group_devices),
                      "checkpoint": args.checkpoint if args.pipeline else None,
                      "idle_ms_per_step": [None if isinstance(r[1], str) else round(r[1], 3) for r in rows[1:]],
                      "loss_impl": args.loss,
                      "peak_hbm_gb": [round(torch.cuda.max_memory_allocated(d) / 1e9, 3)
                                      for d in sorted({d for d in bert.group_devices if d.type == "cuda"},
                                                      key=str)],
                      "final_loss": round(float(loss.detach()), 4) if loss is not None else None}))


def main_stage_per_process(args):
    """One pipeline stage per rank (``torchrun --nproc-per-node S model_parallel_training.py ...``):
    rank s owns BertModelWithMP's s-th np.array_split module group on its own GPU, activations and
    gradients go between ranks as RCCL send/recv (parallel/stage_pipeline.py).  Every rank issues
    only its stage's kernels, so the step is not host-issue-bound the way one thread driving every
    GPU is; ``--graph on`` replays each rank's whole step (sends and receives included) as one
    hipGraph.  The idle table reports each stage's device idle time between its activities."""
    from distributed_training_and_deepspeed_amd import comm
    from distributed_training_and_deepspeed_amd.parallel.stage_pipeline import StagePipeline, bert_stage
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    cuda = torch.cuda.is_available()
    backend = {"auto": "nccl" if cuda else "gloo", "rccl": "nccl", "gloo": "gloo"}[args.pipe_backend]
    if cuda:
        torch.cuda.set_device(local % torch.cuda.device_count())
    device = torch.device("cuda", torch.cuda.current_device()) if cuda else torch.device("cpu")
    comm.init(rank=rank, world_size=world, backend=backend, local_rank=local % max(1, torch.cuda.device_count()))
    config = get_config(args.model)
    dtype = {"bf16": torch.bfloat16, "fp32": torch.float32}[args.dtype]
    owner, mods = bert_stage(config, rank, world, device, dtype=dtype, impl=args.impl, seed=0)
    chunks = args.micro_batch_count if args.pipeline else 1
    loss_fn = Fx.CrossEntropyLoss() if args.loss == "fused" else torch.nn.CrossEntropyLoss()
    upcast = args.loss != "fused"
    ck = args.checkpoint
    if ck == "auto":   # as the single-process form: recompute only where HBM is small
        ck = "never" if not cuda or torch.cuda.get_device_properties(device).total_memory >= 64 * 2 ** 30 \
            else "except_last"
    pipe = StagePipeline(mods, rank, world, device, act_shape=lambda mb: (mb, args.seq_len, config.hidden_size),
                         act_dtype=dtype, loss_fn=lambda out, t: loss_fn(_flat(out, upcast), t.reshape(-1)),
                         chunks=chunks, schedule=args.schedule, set_micro=lambda m: setattr(owner.rt.rng, "micro", m),
                         checkpoint=ck if args.pipeline else "never", overlap=args.pipe_overlap == "on")
    optimizer = torch_adamw([p for p in pipe.parameters() if p.requires_grad], lr=5e-5)
    dataset = load_synthetic(config, args.batch_size * args.training_steps, seq_len=args.seq_len, seed=0)
    g = torch.Generator().manual_seed(0)
    sampler = torch.randperm(len(dataset), generator=g).tolist()  # every rank walks the same batches
    loader = DeviceBatchLoader(dataset, batch_size=args.batch_size, sampler=sampler, device=device)
    pipe.train()

    def step(input_ids, labels):
        loss = pipe.train_step(input_ids if rank == 0 else None, labels if rank == world - 1 else None,
                               rows=input_ids.shape[0])
        optimizer.step()
        optimizer.zero_grad()
        owner.rt.rng.advance()
        return loss.detach() if loss is not None else torch.zeros((), device=device)

    batches = iter(loader)
    graphed, warm, loss = None, [], None
    if args.graph == "on" and backend != "nccl":
        if rank == 0:
            print("--graph: gloo stages messages through host memory (not capturable); running eagerly")
        args.graph = "off"
    if args.graph == "on" and cuda:
        from distributed_training_and_deepspeed_amd.utils.graphs import CapturedStep
        owner.tracker.enabled = False
        warm = [b for _, b in zip(range(min(3, args.training_steps)), batches)]
        if warm:
            graphed = CapturedStep(step, {"input_ids": warm[0]["input_ids"], "labels": warm[0]["labels"]},
                                   warmup_batches=[{"input_ids": b["input_ids"], "labels": b["labels"]} for b in warm])
            loss = graphed.warmup_losses[-1]
    comm.barrier()
    start = time.time()
    n = 0
    for batch in batches:
        if graphed is not None and batch["input_ids"].shape == graphed.static["input_ids"].shape:
            loss = graphed(input_ids=batch["input_ids"], labels=batch["labels"])
        else:
            loss = step(batch["input_ids"], batch["labels"])
        owner.step_boundary()
        n += 1
    if cuda:
        torch.cuda.synchronize()
    comm.barrier()
    elapsed = time.time() - start
    # a replayed graph has no host-side activity marks: its idle time is not measured
    idle = owner.tracker.table(max(n, 1))[1 + rank][1] if graphed is None else None
    idle_all = [None] * world
    torch.distributed.all_gather_object(idle_all, idle)
    loss_all = [None] * world
    torch.distributed.all_gather_object(loss_all, float(loss) if loss is not None else None)
    if rank == 0:
        print(f"\nTotal Training Time: {elapsed:.2f} seconds")
        print("\nAverage Idle Time per Device:")
        rows = [["Device", "Average Idle Time (ms)"]] + [[i, "n/a (graph)" if v is None else v]
                                                         for i, v in enumerate(idle_all)]
        try:
            from tabulate import tabulate
            print(tabulate(rows, headers="firstrow", floatfmt=".2f", tablefmt="fancy_grid"))
        except ImportError:
            for r in rows:
                print(*r, sep="\t")
        print(json.dumps({"tokens_per_s": round(n * args.batch_size * args.seq_len / max(elapsed, 1e-9), 1),
                          "timed_steps": n, "graph": graphed is not None, "pipeline": args.pipeline,
                          "schedule": args.schedule if args.pipeline else None, "stages": world,
                          "mode": "stage-per-process", "transport": backend, "overlap": args.pipe_overlap,
                          "checkpoint": ck if args.pipeline else None,
                          "idle_ms_per_step": [None if v is None else round(v, 3) for v in idle_all],
                          "final_loss": loss_all[-1]}))
    comm.destroy()


if __name__ == "__main__":
    main()
