#!/usr/bin/env python
"""Projected vs measured training memory of one transformer block, re-derived for MI355X.

Parity with the reference estimate_transformer_memory.py: builds the
instrumented OPT-style block (h=9216, a=72, ffn=36864, s=512, b=4 by default), prints
"Projected total memory usage", then measures on the device, each with a "Percent difference":
model memory (allocator delta vs parameter bytes), activation memory (allocator delta of the
forward vs the forward-hook byte count), gradient memory (after backward(retain_graph=True) vs
parameter bytes), optimizer memory (after torch Adam(lr=1e-3).step() vs 8 B/param), and the
actual total.  Labels follow the reference (its "Optimizer + Gradient" line measures the
optimizer delta only -- quirk 4).

MI355X additions (``--mi355x-report``): the 288 GB capacity view -- projections for fp32 (the
reference formula), bf16 mixed precision with the flash-attention activation path, and ZeRO
stages 1-3 over N GPUs, plus the largest block hidden size that fits 288 GB.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_training_and_deepspeed_amd.memory import (ActivationCounter, get_model_memory,  # noqa: E402
                                                           get_optimizer_memory, max_hidden_for_capacity,
                                                           project_training_memory, project_transformer_memory,
                                                           register_hooks_recursive)
from distributed_training_and_deepspeed_amd.models.transformer_block import BlockConfig, TransformerBlock  # noqa: E402
from distributed_training_and_deepspeed_amd.utils import format_size, get_device  # noqa: E402


def get_current_memory_allocation(device):
    if device == "mps":
        return torch.mps.current_allocated_memory()
    if device == "cuda":
        return torch.cuda.memory_allocated()
    raise ValueError(f"Unsupported device: {device} (allocator statistics need a GPU)")


def pct(a, b):
    return abs(a - b) / b * 100 if b else 0.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hidden-size", type=int, default=9216)
    ap.add_argument("--heads", type=int, default=72)
    ap.add_argument("--ffn-dim", type=int, default=36864)
    ap.add_argument("--seq-len", type=int, default=512)
    ap.add_argument("--batch-size", type=int, default=4)
    ap.add_argument("--mi355x-report", action="store_true")
    ap.add_argument("--project-only", action="store_true")
    args = ap.parse_args()

    b, s = args.batch_size, args.seq_len
    config = BlockConfig(hidden_size=args.hidden_size, num_attention_heads=args.heads, ffn_dim=args.ffn_dim,
                         max_position_embeddings=s, dropout=0.1, enable_bias=True)
    with torch.device("meta"):
        meta_block = TransformerBlock(config)
    n_params = sum(p.numel() for p in meta_block.parameters())
    projected = project_transformer_memory(1, config.hidden_size, config.num_attention_heads, b, s,
                                           optimizer_bytes_per_param=8, num_params=n_params)
    print(f"Projected total memory usage: {format_size(projected)}")
    print("-" * 80)
    result = {"projected_bytes": projected, "params": n_params}
    if args.mi355x_report:
        rep = {}
        for prec in ("fp32", "bf16"):
            for stage in (0, 1, 2, 3):
                p = project_training_memory(1, config.hidden_size, config.num_attention_heads, b, s, config.ffn_dim,
                                            precision=prec, flash_attention=(prec == "bf16"), zero_stage=stage,
                                            world_size=8 if stage else 1)
                rep[f"{prec}_zero{stage}"] = format_size(p.total)
        rep["max_hidden_fp32_reference_formula_288GB"] = max_hidden_for_capacity(fp32_reference=True)
        rep["max_hidden_bf16_flash_288GB"] = max_hidden_for_capacity(fp32_reference=False)
        print(json.dumps(rep, indent=1))
        result["mi355x"] = rep
    if args.project_only:
        return result

    device = get_device()
    model = TransformerBlock(config)
    model.to(device)
    with_model = get_current_memory_allocation(device)
    est_model = get_model_memory(model)
    print(f"Measured Model Memory: {format_size(with_model)}")
    print(f"Estimated Model Memory: {format_size(est_model)}")
    print(f"Percent difference: {pct(with_model, est_model):.2f}%")
    print("-" * 80)

    counter = ActivationCounter()
    register_hooks_recursive(model, counter)
    inputs = torch.randn(b, s, config.hidden_size).to(device)
    outputs = model(inputs)
    counter.add_activations(inputs)
    fwd = get_current_memory_allocation(device) - with_model
    print(f"Consumed Activation Memory: {format_size(fwd)}")
    print(f"Estimated Activation Memory: {format_size(counter.activation_bytes)}")
    print(f"Percent difference: {pct(fwd, counter.activation_bytes):.2f}%")
    print("-" * 80)

    loss_fn = torch.nn.MSELoss()
    labels = torch.randn_like(outputs).to(device)
    loss = loss_fn(outputs, labels)
    loss.backward(retain_graph=True)
    grads = get_current_memory_allocation(device) - with_model - fwd
    print(f"Consumed Gradient Memory: {format_size(grads)}")
    print(f"Estimated Gradient Memory: {format_size(est_model)}")
    print(f"Percent difference: {pct(grads, est_model):.2f}%")
    print("-" * 80)

    optimizer = torch.optim.Adam(model.parameters(), lr=1e-3)
    optimizer.step()
    post = get_current_memory_allocation(device) - with_model - fwd - grads
    est_opt = get_optimizer_memory(model, optimizer)
    print(f"Consumed Optimizer + Gradient Memory: {format_size(post)}")
    print(f"Estimated Optimizer + Gradient Memory: {format_size(est_opt)}")
    print(f"Percent difference: {pct(post, est_opt):.2f}%")
    print("-" * 80)
    total = get_current_memory_allocation(device)
    print(f"Actual total memory usage: {format_size(total)}")
    result.update({"model": [with_model, est_model], "activations": [fwd, counter.activation_bytes],
                   "grads": [grads, est_model], "optimizer": [post, est_opt], "total": total})
    print(json.dumps({k: v for k, v in result.items() if k != "mi355x"}))
    return result


if __name__ == "__main__":
    main()
