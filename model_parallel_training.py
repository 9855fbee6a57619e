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
    args = parser.parse_args()

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

    start = time.time()
    progress = None
    if not args.verbose:
        try:
            from tqdm import tqdm
            progress = tqdm(range(args.training_steps))
        except ImportError:
            pass
    n, loss = 0, None
    for batch in loader:
        input_ids = batch["input_ids"]
        if args.pipeline and args.schedule == "1f1b":
            loss = model.train_step(input_ids, batch["labels"],
                                    lambda out, t: loss_fn(_flat(out, upcast), t.view(-1)),
                                    schedule="1f1b")
        else:
            outputs = model(input_ids)
            labels = batch["labels"].to(bert.head_device)
            loss = loss_fn(_flat(outputs, upcast), labels.view(-1))
            loss.backward()
        optimizer.step()
        optimizer.zero_grad()
        bert.advance_rng()
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
    rows = summarize_idle_time(bert, args.training_steps)
    print(json.dumps({"tokens_per_s": round(n * args.batch_size * args.seq_len / max(elapsed, 1e-9), 1),
                      "pipeline": args.pipeline, "stages": len(bert.group_devices),
                      "checkpoint": args.checkpoint if args.pipeline else None,
                      "idle_ms_per_step": [round(r[1], 3) for r in rows[1:]],
                      "loss_impl": args.loss,
                      "peak_hbm_gb": [round(torch.cuda.max_memory_allocated(d) / 1e9, 3)
                                      for d in sorted({d for d in bert.group_devices if d.type == "cuda"},
                                                      key=str)],
                      "final_loss": round(float(loss.detach()), 4) if loss is not None else None}))


if __name__ == "__main__":
    main()
