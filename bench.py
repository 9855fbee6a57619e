#!/usr/bin/env python
"""Headline benchmark: BERT-base masked-LM DDP training throughput (tokens/s, whole job).

BASELINE.json metric: "tokens/sec (whole node) BERT-base DDP at 1/2/4/8 MI355X".  The step
timed here is the full training step of the reference's ``data_parallel_training.py``
(forward with MLM labels -> backward with bucketed gradient all-reduce -> Adam step), on
bert-base-cased geometry (108.3 M parameters, random init), seq 512, synthetic MLM batches
with the reference masking law, bf16 compute with fp32 master weights.  Per-GPU batch is
fixed as N grows (weak scaling); the default 256 x 512 tokens per GPU (the reference ran 4 on a
16 GB T4) peaks at ~47 GB of the 288 GB HBM, runs the GEMMs at their large-M efficiency
(1.0-1.4 PF/s, TunableOp table measured at this shape) and amortises the per-step gradient
all-reduce over a ~100 ms step (b256 vs b128: +2.1 % tokens/s same box; b384/b512 add < 1 %).
Each rank draws its own dropout masks (seed offset by rank).

  python bench.py --gpus N --steps K --warmup W
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Other BASELINE configs through the same timing contract: ``--model large`` (BERT-large DDP),
``--zero-stage 2`` (BERT-base through the ZeRO engine of zero_dp_training.py), ``--model
gpt2-medium --zero-stage 3``.

Rank 0 prints ONE JSON line; ``value`` = total tokens/s over all ranks, computed from the
MAX step time over ranks.
"""
from __future__ import annotations

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
import torch.distributed as dist


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="base")
    ap.add_argument("--batch-size", type=int, default=int(os.environ.get("DTD_BENCH_BATCH", "1024")),
                    help="per-GPU micro-batch (sequences); 1024 x 512 tokens use 161 GB of the 288 GB "
                         "(same box: 256 / 512 / 768 / 1024 -> 1.471 / 1.498 / 1.506 / 1.510 M tokens/s, "
                         "profiles/r5_s39_batch.jsonl)")
    ap.add_argument("--seq-len", type=int, default=512)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--grad-dtype", default=None, choices=[None, "bf16", "fp32"])
    ap.add_argument("--bucket-mb", type=float, default=float(os.environ.get("DTD_BUCKET_MB", "64")))
    ap.add_argument("--impl", default="fused", choices=["fused", "reference"])
    ap.add_argument("--graph", default="off", choices=["on", "off"],
                    help="capture the whole training step in a hipGraph and replay it")
    ap.add_argument("--small-bucket-allreduce", default="rccl", choices=["rccl", "xgmi"],
                    help="xgmi: buckets <= 4 MiB use the native peer-mapped all-reduce kernel")
    ap.add_argument("--async-wgrad", default="off", choices=["on", "off"],
                    help="weight-gradient GEMMs on a side stream, concurrent with the dgrad chain")
    ap.add_argument("--zero-stage", type=int, default=None, choices=[0, 1, 2, 3],
                    help="train through the ZeRO engine (zero_dp_training.py's path) instead of DDP")
    ap.add_argument("--reduce-bucket", type=float, default=2.5e7,
                    help="ZeRO reduce_bucket_size (elements) for --zero-stage")
    ap.add_argument("--dense-mlm-head", action="store_true")
    ap.add_argument("--mlm-capacity", default="static", choices=["static", "dynamic"],
                    help="sparse MLM head rows: a fixed capacity (mean + 8 sigma of the 15%% law, rounded "
                         "to 256; constant GEMM shapes, no per-step host sync; overflow raises) or the exact "
                         "labelled-row count per batch")
    ap.add_argument("--opt-overlap", default=os.environ.get("DTD_OPT_OVERLAP", "on"), choices=["on", "off"],
                    help="DDP: the Adam update runs stage by stage on a side stream and the next forward "
                         "waits per stage (FusedAdam.overlap_with_forward; bit-identical results)")
    ap.add_argument("--force-collectives", action="store_true",
                    help="issue the DDP bucket all-reduces / ZeRO reduce-scatters and all-gathers through RCCL "
                         "even at world size 1 (the N > 1 data path on one GPU)")
    ap.add_argument("--comm-init", default="none", choices=["none", "rccl", "rccl-lazy", "rccl-destroy", "rccl-late", "rccl-after-warmup", "gloo", "uncached",
                             "finegrained", "hostmem"],
                    help="diagnostic: initialise a process group even when no collective runs (rccl: "
                         "comm.init; rccl-lazy: no device_id, so no communicator is created; "
                         "rccl-destroy: comm.init then destroy before the model is built; rccl-late / "
                         "rccl-after-warmup: comm.init after the model and data are allocated / after "
                         "the warm-up steps; gloo; "
                         "uncached / finegrained / hostmem: only the 512 MB uncached, fine-grained "
                         "device or 4 MB pinned host buffer RCCL's init allocates)")
    ap.add_argument("--ddp-overlap", default="on", choices=["on", "off"],
                    help="diagnostic: off launches every bucket collective after the backward")
    ap.add_argument("--prewarm", default="auto", choices=["auto", "none", "layer1", "layer1-batch", "tiny", "full",
                                                          "blas", "reserve", "custom"],
                    help="one forward+backward of a throwaway copy of the model before the RCCL group is "
                         "created (auto: a 1-layer copy at batch 1 whenever a group is created; layer1-batch: "
                         "1 layer at the bench batch; tiny: full depth, batch 1; full: full depth at the bench "
                         "batch; utils/prewarm.py).  Bisect arms: blas (one hipBLASLt GEMM only), reserve (only "
                         "an allocator reservation of --reserve-gb), custom (the 1-layer step with the products "
                         "on the hand-written GEMMs, no hipBLASLt where they tile)")
    ap.add_argument("--reserve-gb", type=float, default=48.0, help="--prewarm reserve: bytes to reserve")
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("--no-tuned-gemms", action="store_true", help="skip the measured hipBLASLt solution table")
    return ap.parse_args()


def _hand_gemm_config() -> dict:
    """Which products the hand-written GEMMs take in this run (ops/gemm.py dispatch rules)."""
    from distributed_training_and_deepspeed_amd.ops import gemm as G
    from distributed_training_and_deepspeed_amd.ops import functional as Fx
    from distributed_training_and_deepspeed_amd.ops import grad as GR
    return {"proj_w4": G.w4_enabled(), "proj_w4_max_k": G._W4_MAX_K[0], "proj_w4_min_tiles": G.w4_min_tiles(),
            "proj_w4_residual_add": G._W4_ADD[0], "ffn_fused": G.ffn_fwd_enabled(),
            "ffn_min_tiles": G._FFN_MIN_TILES[0] or "cus", "wgrad": G.wgrad_enabled(),
            "wgrad_min_tokens": GR._WGRAD_MIN_T[0], "finalize_batch": Fx._BATCH[0]}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from distributed_training_and_deepspeed_amd import comm
    from distributed_training_and_deepspeed_amd.data import SyntheticLMDataset
    from distributed_training_and_deepspeed_amd.models import build_model, get_config
    from distributed_training_and_deepspeed_amd.optim import hf_adamw
    from distributed_training_and_deepspeed_amd.parallel import DistributedDataParallel
    from distributed_training_and_deepspeed_amd.utils.prewarm import prewarm_enabled, prewarm_model_kernels

    cuda = torch.cuda.is_available()
    tuned = False
    if cuda:
        torch.cuda.set_device(local)
        if not args.no_tuned_gemms and "PYTORCH_TUNABLEOP_ENABLED" not in os.environ:
            from distributed_training_and_deepspeed_amd.utils.tuning import use_tuned_gemms
            tuned = use_tuned_gemms()
    device = torch.device("cuda", local) if cuda else torch.device("cpu")
    group = world > 1 or args.zero_stage is not None or args.force_collectives or args.comm_init != "none"
    if cuda and args.prewarm in ("blas", "reserve"):
        from distributed_training_and_deepspeed_amd.utils.prewarm import prewarm_blas, prewarm_reserve
        if args.prewarm == "blas":
            prewarm_blas(device)
        else:
            prewarm_reserve(device, int(args.reserve_gb * 1e9))
    elif cuda and args.prewarm != "none" and (args.prewarm != "auto" or (group and prewarm_enabled())):
        # the step's kernels run once before the RCCL communicator exists (utils/prewarm.py:
        # kernels first launched after it run 5-25 % slower for the life of the process)
        prewarm_model_kernels(args.model, device, dtype=torch.bfloat16 if args.dtype == "bf16" else torch.float32,
                              impl=args.impl, seq_len=args.seq_len,
                              layers=None if args.prewarm in ("tiny", "full") else 1,
                              batch=args.batch_size if args.prewarm in ("full", "layer1-batch") else 1,
                              static_mlm=not args.dense_mlm_head and args.mlm_capacity == "static",
                              library_gemms=args.prewarm != "custom",
                              **({"sparse_mlm_head": not args.dense_mlm_head} if get_config(args.model).family == "bert" else {}))
    real_group = world > 1 or args.zero_stage is not None or args.force_collectives   # ZeRO always runs on a group
    if real_group:
        comm.init(rank=rank, world_size=world, local_rank=local)
    elif args.comm_init != "none":   # diagnostic process-group / allocation forms (world 1 only)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29561")
        if args.comm_init in ("uncached", "finegrained", "hostmem"):
            import ctypes
            # the HIP runtime torch already loaded (a second copy would be a second runtime)
            hip = ctypes.CDLL(next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln))
            buf = ctypes.c_void_p()
            if args.comm_init == "hostmem":
                rc = hip.hipHostMalloc(ctypes.byref(buf), ctypes.c_size_t(4 << 20), ctypes.c_uint(0))
            else:
                rc = hip.hipExtMallocWithFlags(ctypes.byref(buf), ctypes.c_size_t(512 << 20),
                                               ctypes.c_uint(3 if args.comm_init == "uncached" else 1))
            if rc != 0:
                raise RuntimeError(f"diagnostic allocation failed: hip error {rc}")
        elif args.comm_init in ("rccl-late", "rccl-after-warmup"):
            pass   # below
        elif args.comm_init in ("rccl", "rccl-destroy"):
            comm.init(rank=rank, world_size=world, local_rank=local)
            if args.comm_init == "rccl-destroy":
                comm.destroy()
        else:
            dist.init_process_group(backend="nccl" if args.comm_init == "rccl-lazy" else "gloo", rank=rank,
                                    world_size=world)
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    cfg = get_config(args.model)
    mlm = cfg.family == "bert"
    model = build_model(args.model, impl=args.impl, dtype=dtype, device=device, seed=1234,
                        **({"sparse_mlm_head": not args.dense_mlm_head} if mlm else {}))
    if args.impl == "reference":
        model.rt.exact_dropout = False  # torch-eager baseline: ATen dropout, HF-style eager ops
    model.train()
    model.rt.rng.reseed(1234 + rank)   # independent dropout masks per data-parallel replica
    gdt = {"bf16": torch.bfloat16, "fp32": torch.float32}.get(args.grad_dtype, dtype)
    zero = args.zero_stage is not None
    if zero:
        from distributed_training_and_deepspeed_amd.parallel.zero import initialize
        # zero_dp_training.py's DeepSpeed config (Adam lr 1.5e-4), larger reduce buckets
        zcfg = {"train_micro_batch_size_per_gpu": args.batch_size,
                "optimizer": {"type": "Adam", "params": {"lr": 1.5e-4}},
                # the partitioned data flow even at world 1 (the path every rank runs at N > 1)
                "zero_optimization": {"stage": args.zero_stage, "reduce_bucket_size": args.reduce_bucket,
                                      "world1_replicated": False,
                                      "force_collectives": args.force_collectives},
                "bf16": {"enabled": dtype == torch.bfloat16}}
        engine, _, _, _ = initialize(model=model, model_parameters=model.parameters(), config=zcfg)
        gdt = engine.grad_dtype
    else:
        ddp = DistributedDataParallel(model, bucket_cap_mb=args.bucket_mb, grad_dtype=gdt,
                                      small_bucket_allreduce=args.small_bucket_allreduce,
                                      async_wgrad=args.async_wgrad == "on",
                                      force_collectives=args.force_collectives,
                                      overlap=args.ddp_overlap == "on")
        opt = hf_adamw(ddp.parameters(), lr=5e-5)

    B, S = args.batch_size, args.seq_len
    nb = args.warmup + args.steps
    ds = SyntheticLMDataset(cfg, num_samples=B * min(nb, 8), seq_len=S, seed=100 + rank)
    ids = ds.input_ids.view(-1, B, S).to(device)
    labels = ds.labels.view(-1, B, S).to(device)
    nbuf = ids.shape[0]

    def train_step(input_ids, labels):
        if zero:
            out = engine(input_ids, labels=labels)
            engine.backward(out.loss)
            engine.step()                # advances the dropout RNG step itself
            return out.loss.detach()
        out = ddp(input_ids, labels=labels)
        out.loss.backward()
        opt.step()
        model.rt.rng.advance()
        return out.loss.detach()

    static_mlm = mlm and not args.dense_mlm_head and cuda and (args.graph == "on" or args.mlm_capacity == "static")
    if static_mlm:
        # fixed labelled-row capacity: padding rows carry label -100 (zero loss and gradient), so
        # loss and gradients equal the exact-count head's; rt.mlm_overflow flags a batch that
        # would not fit (checked after the timed steps)
        from distributed_training_and_deepspeed_amd.utils.graphs import mlm_capacity
        model.rt.mlm_capacity = -(-mlm_capacity(B * S) // 256) * 256
        model.rt.mlm_overflow = torch.zeros((), dtype=torch.bool, device=device)
    opt_overlap = (not zero and cuda and args.graph != "on" and args.opt_overlap == "on"
                   and hasattr(opt, "overlap_with_forward") and hasattr(model, "zero3_units"))
    if opt_overlap:
        opt.overlap_with_forward(model.zero3_units(), root=model)
    graphed = None
    if args.graph == "on" and cuda and not zero:
        # one hipGraph replay per step (host-launch-bound small batches); static-size MLM head
        from distributed_training_and_deepspeed_amd.utils.graphs import CapturedStep
        graphed = CapturedStep(train_step, {"input_ids": ids[0], "labels": labels[0]}, warmup=3, runtime=model.rt)

    def step(i):
        if graphed is not None:
            return graphed(input_ids=ids[i % nbuf], labels=labels[i % nbuf])
        return train_step(ids[i % nbuf], labels[i % nbuf])

    def sync():
        if cuda:
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    if args.comm_init == "rccl-late":
        comm.init(rank=rank, world_size=world, local_rank=local)
    for i in range(args.warmup):
        loss = step(i)
    sync()
    if args.comm_init == "rccl-after-warmup":
        comm.init(rank=rank, world_size=world, local_rank=local)
    first_loss = float(loss.detach()) if args.warmup else float("nan")
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step(args.warmup + i)
    sync()
    dt = time.perf_counter() - t0
    if graphed is not None:
        graphed.check()
    if static_mlm and bool(model.rt.mlm_overflow):
        raise RuntimeError("a batch had more labelled rows than the static MLM capacity: use --mlm-capacity dynamic")
    if world > 1:
        t = torch.tensor([dt], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    tokens = world * B * S * args.steps
    value = tokens / dt
    if rank == 0:
        engine_name = f"ZeRO-{args.zero_stage}" if zero else "DDP"
        res = {
            "metric": "tokens/sec (whole node) BERT-base DDP" if cfg.name == "bert-base-cased" and not zero
                      else f"tokens/sec (whole node) {cfg.name} {engine_name}",
            "value": round(value, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": ("synthetic (random token ids, HF MLM 15%/80/10/10 masking; random-init weights; "
                     "batches pre-staged on device)" if mlm
                     else "synthetic (random token ids, causal labels = input_ids; random-init weights; "
                          "batches pre-staged on device)"),
            "config": {
                "model": cfg.name,
                "params": sum(p.numel() for p in model.parameters()),
                "global_batch": B * world,
                "per_gpu_batch": B,
                "seq_len": S,
                "parallelism": f"zero{args.zero_stage}-dp{world}" if zero else f"dp{world}",
                "bucket_mb": args.reduce_bucket * 2 / 2 ** 20 if zero else args.bucket_mb,
                "grad_dtype": str(gdt).replace("torch.", ""),
                "impl": args.impl,
                "mlm_head": (None if not mlm else "dense" if args.dense_mlm_head
                             else "sparse (labelled rows only, static capacity %d; identical loss/grads)"
                             % model.rt.mlm_capacity if static_mlm
                             else "sparse (labelled rows only; identical loss/grads)"),
                "optimizer": ("fused Adam on the ZeRO shard (zero_dp_training.py config, lr 1.5e-4)" if zero
                              else "fused AdamW (transformers.AdamW hyper-params, lr 5e-5)"),
                "tuned_gemms": tuned,
                "hand_gemms": _hand_gemm_config() if cuda else None,
                "hip_graph": graphed is not None,
                "force_collectives": args.force_collectives,
                "prewarm": args.prewarm,
                "async_wgrad": args.async_wgrad == "on",
                "opt_overlap": opt_overlap,
                "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 1e9, 1) if cuda else None,
                "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
            },
            "loss_first": round(first_loss, 4),
            "loss_last": round(float(loss.detach()), 4),
        }
        print(json.dumps(res), flush=True)
    if world > 1 or zero or args.force_collectives or dist.is_initialized():
        comm.destroy()


if __name__ == "__main__":
    main()
