"""GPU tests of the parallel engines on one MI355X (RCCL at world 1, gloo for world 2 on one card)."""
import os

import pytest
import torch
import torch.multiprocessing as mp

from distributed_training_and_deepspeed_amd import comm
from distributed_training_and_deepspeed_amd.data import SyntheticLMDataset
from distributed_training_and_deepspeed_amd.models import build_model
from distributed_training_and_deepspeed_amd.models import config as C

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rccl_world1():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(29000 + os.getpid() % 1000)
    comm.init(rank=0, world_size=1, backend="nccl", local_rank=0)
    yield
    comm.destroy()


def _zero_run(stage, steps=4, replicated=True, force=False, overlap_opt=False):
    from distributed_training_and_deepspeed_amd.parallel.zero import initialize
    model = build_model("causal-tiny", dtype=torch.bfloat16, device="cuda", seed=3)
    cfg = {"optimizer": {"type": "Adam", "params": {"lr": 1e-3}}, "comms_logger": {"enabled": True},
           "zero_optimization": {"stage": stage, "reduce_bucket_size": 100000, "world1_replicated": replicated,
                                 "force_collectives": force, "overlap_optimizer_step": overlap_opt}}
    eng, opt, _, _ = initialize(model=model, model_parameters=model.parameters(), config=cfg)
    ds = SyntheticLMDataset(model.cfg, 4 * steps, seq_len=128, mlm=False, seed=1)
    ids, lab = ds.input_ids.view(steps, 4, 128).cuda(), ds.labels.view(steps, 4, 128).cuda()
    losses = []
    eng.started_in_backward = []
    for i in range(steps):
        loss = eng(ids[i], labels=lab[i]).loss
        eng.backward(loss)
        eng.started_in_backward.append(eng._opt_started)
        eng.step()
        losses.append(loss.item())
    torch.cuda.synchronize()
    return losses, eng.master.detach().float().clone(), eng


@pytest.mark.parametrize("stage,replicated", [(1, False), (2, False), (3, False), (1, True), (2, True), (3, True)])
def test_zero_stages_on_gpu_match_stage0(rccl_world1, stage, replicated):
    """Stages 1-3 train like stage 0 on one GPU, through the partitioned data flow (landing
    arena, reduce-scatter / refresh stand-ins, overlapped refresh) and through the world-1
    replicated layout (stages 1/2 alias the flat buffers)."""
    l0, m0, _ = _zero_run(0)
    ls, ms, eng = _zero_run(stage, replicated=replicated)
    assert eng.replicated == (replicated and stage <= 2) and eng.alias_units == (replicated and stage == 3)
    assert all(torch.isfinite(torch.tensor(ls)))
    assert abs(l0[-1] - ls[-1]) < 5e-3, (l0, ls)
    # world 1: every layout holds the same parameter set (different order for stage 3 units)
    assert abs(m0.sum().item() - ms.sum().item()) < 1e-2 * m0.abs().sum().item() / m0.numel() * 100 + 1e-3


@pytest.mark.parametrize("stage", [1, 2, 3])
def test_zero_rccl_collectives_at_world1_match_local_path(rccl_world1, stage):
    """force_collectives: the partitioned engine issues its real RCCL reduce-scatters and refresh /
    stage-3 all-gathers (on its comm stream, overlapped with backward) at world 1 -- and trains
    exactly like the same engine's local stand-ins for them."""
    ll, ml, el = _zero_run(stage, replicated=False)
    lf, mf, ef = _zero_run(stage, replicated=False, force=True)
    assert ef.collect and not el.collect
    assert ll == lf, (ll, lf)
    assert torch.equal(ml, mf)


@pytest.mark.parametrize("stage,replicated,force", [(0, True, False), (1, False, False), (2, False, False),
                                                    (2, False, True), (3, True, False), (3, False, False),
                                                    (3, False, True)])
def test_zero_optimizer_overlapped_with_backward_is_bit_identical(rccl_world1, stage, replicated, force):
    """overlap_optimizer_step: each segment's Adam update launched on a side stream once the
    backward is past it (stage-3 units one unit late, so a layer's own input-gradient GEMM has read
    its weights) -- the same kernel per element, so losses and master weights are bit-identical to
    the single launch in step(), and the update really started inside the backward."""
    lo, mo, eo = _zero_run(stage, replicated=replicated, force=force)
    import os as _os
    os_prev = _os.environ.pop("DTD_ZERO_OPT_OVERLAP", None)
    try:
        lv, mv, ev = _zero_run(stage, replicated=replicated, force=force, overlap_opt=True)
    finally:
        if os_prev is not None:
            _os.environ["DTD_ZERO_OPT_OVERLAP"] = os_prev
    assert ev.overlap_opt and not eo.overlap_opt
    assert all(ev.started_in_backward) and not any(eo.started_in_backward)
    assert ev.optimizer.step_count == eo.optimizer.step_count == 4
    assert lo == lv, (lo, lv)
    assert torch.equal(mo, mv)


def _ddp_run(force, steps=4, overlap=True):
    """bench.py's data path at small scale: fused BERT, DDP buckets (shaped tail buckets), fused
    AdamW with the stage-by-stage update overlapped with the next forward."""
    from distributed_training_and_deepspeed_amd.optim import hf_adamw
    from distributed_training_and_deepspeed_amd.parallel import DistributedDataParallel
    model = build_model("tiny", dtype=torch.bfloat16, device="cuda", seed=3)
    ddp = DistributedDataParallel(model, bucket_cap_mb=0.25, force_collectives=force)
    opt = hf_adamw(ddp.parameters(), lr=1e-3)
    if overlap:
        opt.overlap_with_forward(model.zero3_units(), root=model)
    ds = SyntheticLMDataset(model.cfg, 4 * steps, seq_len=128, seed=1)
    ids, lab = ds.input_ids.view(steps, 4, 128).cuda(), ds.labels.view(steps, 4, 128).cuda()
    losses = []
    for i in range(steps):
        out = ddp(ids[i], labels=lab[i])
        out.loss.backward()
        opt.step()
        model.rt.rng.advance()
        losses.append(out.loss.detach())
    opt.synchronize()
    torch.cuda.synchronize()
    return [x.item() for x in losses], [p.detach().clone() for p in model.parameters()], ddp


def test_ddp_rccl_bucket_allreduce_with_optimizer_overlap_matches_local_path(rccl_world1):
    """The N > 1 step of bench.py on one GPU: every bucket's RCCL all-reduce (AVG over one rank
    is exact) issued from the autograd thread, the optimizer's stage-by-stage update on its side
    stream under the next forward -- bitwise equal to the same step without collectives."""
    ll, pl, dl = _ddp_run(False)
    lf, pf, df = _ddp_run(True)
    assert df.collectives and not dl.collectives and len(df.buckets) > 2
    assert ll == lf, (ll, lf)
    for a, b in zip(pl, pf):
        assert torch.equal(a, b)


def test_gpipe_two_stages_one_gpu_recompute_is_exact():
    from distributed_training_and_deepspeed_amd.models.bert_mp import BertModelWithMP
    cfg = C.BERT_TINY
    a = BertModelWithMP(cfg, devices=["cuda:0", "cuda:0"], dtype=torch.bfloat16, seed=5)
    ds = SyntheticLMDataset(cfg, 8, seq_len=128, seed=2)
    ids, lab = ds.input_ids.cuda(), ds.labels.cuda()
    grads = []
    for ck in ("never", "always"):
        a.zero_grad(set_to_none=True)
        out = a.to_pipeline(chunks=4, checkpoint=ck)(ids)
        torch.nn.functional.cross_entropy(out.view(-1, cfg.vocab_size).float(), lab.view(-1)).backward()
        grads.append({n: p.grad.float().clone() for n, p in a.named_parameters()})
    for n in grads[0]:
        assert torch.equal(grads[0][n], grads[1][n]), n
    rows = a.tracker.table(2)
    assert len(rows) == 3


def test_estimator_matches_allocator_on_gpu():
    """Run the estimator in a fresh process (its allocator deltas assume an empty device)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(root, "estimate_transformer_memory.py"), "--hidden-size", "2048",
                          "--heads", "16", "--ffn-dim", "8192"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    res = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    for k in ("model", "optimizer"):
        got, est = res[k]
        assert abs(got - est) / est < 0.05, (k, got, est)
    # the allocator delta after backward(retain_graph=True) also holds autograd temporaries
    # (the reference's measurement has the same bias; 5.7% at its h=9216 block on MI355X)
    got, est = res["grads"]
    assert 0.95 * est <= got <= 1.7 * est, (got, est)


def _ddp_gloo_gpu(rank, world, port, out, bench_like=False):
    from distributed_training_and_deepspeed_amd.optim import hf_adamw
    from distributed_training_and_deepspeed_amd.parallel import DistributedDataParallel
    comm.init(rank=rank, world_size=world, backend="gloo", init_method=f"file://{out}/rdzv")
    torch.cuda.set_device(0)
    dt = torch.bfloat16 if bench_like else torch.float32
    model = build_model("tiny", dtype=dt, device="cuda:0", seed=3)
    ddp = DistributedDataParallel(model, bucket_cap_mb=0.5)
    opt = hf_adamw(ddp.parameters(), lr=1e-3)
    if bench_like:   # bench.py's N > 1 step: bf16, the optimizer staged under the next forward
        opt.overlap_with_forward(model.zero3_units(), root=model)
    ds = SyntheticLMDataset(model.cfg, 4, seq_len=64, seed=10 + rank)
    for _ in range(3 if bench_like else 2):
        ddp(ds.input_ids.cuda(), labels=ds.labels.cuda()).loss.backward()
        opt.step()
        model.rt.rng.advance()
    if bench_like:
        opt.synchronize()
    torch.save([p.detach().cpu() for p in model.parameters()], os.path.join(out, f"p{rank}.pt"))
    comm.destroy()


@pytest.mark.parametrize("bench_like", [False, True])
def test_ddp_two_ranks_share_one_gpu_stay_in_sync(tmp_path, free_port, bench_like):
    """Two processes share cuda:0 over gloo with different batches: after the gradient all-reduce
    every parameter is identical on both ranks (an optimizer that read a gradient before its
    bucket's reduction finished -- e.g. the side-stream staged update -- would diverge)."""
    mp.spawn(_ddp_gloo_gpu, args=(2, free_port, str(tmp_path), bench_like), nprocs=2, join=True)
    a = torch.load(tmp_path / "p0.pt", weights_only=True)
    b = torch.load(tmp_path / "p1.pt", weights_only=True)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


def _zero_gloo_gpu(rank, world, port, out, stage):
    """ZeRO on real HIP streams with a real peer: two processes share cuda:0 over gloo, bf16
    fused model, gradient accumulation 2 -- exercises the landing arena's event-guarded reuse,
    release events and the gather / compute ordering (stage 3) with async comm streams."""
    from distributed_training_and_deepspeed_amd.parallel.zero import initialize
    comm.init(rank=rank, world_size=world, backend="gloo", init_method=f"file://{out}/rdzv{stage}")
    torch.cuda.set_device(0)
    model = build_model("causal-tiny", dtype=torch.bfloat16, device="cuda:0", seed=3)
    cfg = {"gradient_accumulation_steps": 2, "optimizer": {"type": "Adam", "params": {"lr": 1e-3}},
           "zero_optimization": {"stage": stage, "reduce_bucket_size": 20000, "allgather_bucket_size": 40000,
                                 "stage3_prefetch_bucket_size": 30000}}
    eng, _, _, _ = initialize(model=model, model_parameters=model.parameters(), config=cfg)
    ds = SyntheticLMDataset(model.cfg, 2 * 4 * 6, seq_len=128, mlm=False, seed=1)
    ids = ds.input_ids.view(6, 2, 4, 128)[:, rank].cuda()
    lab = ds.labels.view(6, 2, 4, 128)[:, rank].cuda()
    losses = []
    for i in range(6):
        loss = eng(ids[i], labels=lab[i]).loss
        eng.backward(loss)
        eng.step()
        losses.append(loss.item())
    torch.cuda.synchronize()
    # full fp32 master parameters by name, rebuilt from every rank's shard
    shard = eng.master.detach().float().cpu()
    shards = [torch.zeros_like(shard) for _ in range(world)]
    torch.distributed.all_gather(shards, shard)
    names = {id(p): n for n, p in model.named_parameters()}
    full = {}
    for s in eng.segments:
        w_s = world if (stage > 0) else 1
        seg = torch.cat([shards[r][s.shard_off:s.shard_off + s.chunk] for r in range(w_s)])
        for i, p in enumerate(s.params):
            full[names[id(p)]] = s.view(seg, i).clone()
    torch.save({"losses": losses, "params": full}, os.path.join(out, f"z{stage}_{rank}.pt"))
    comm.destroy()


@pytest.mark.parametrize("stage", [1, 2, 3])
def test_zero_two_ranks_share_one_gpu_match_stage0(tmp_path, free_port, stage):
    import math
    res = {}
    for st in (0, stage):
        mp.spawn(_zero_gloo_gpu, args=(2, free_port, str(tmp_path), st), nprocs=2, join=True)
        res[st] = [torch.load(tmp_path / f"z{st}_{r}.pt", weights_only=True) for r in range(2)]
    # same losses per rank (both engines see the same data and start from rank 0's weights)
    for r in range(2):
        a, b = res[0][r]["losses"], res[stage][r]["losses"]
        assert all(math.isfinite(x) for x in b)
        assert max(abs(x - y) for x, y in zip(a, b)) < 2e-2, (r, a, b)

    p0, ps = res[0][0]["params"], res[stage][0]["params"]
    assert p0.keys() == ps.keys()
    # compare the training UPDATES (final - initial): Adam moves every element by up to ~lr per step
    # whatever its gradient's size, so elements whose tiny gradients differ by reduction order can
    # flip direction -- bound each element by 2 lr per step and the update's relative norm by 5 %
    init = {n: p.detach().to(torch.bfloat16).float() for n, p in build_model("causal-tiny", seed=3).named_parameters()}
    for n in p0:
        assert torch.isfinite(ps[n]).all(), n
        d0, ds = p0[n] - init[n], ps[n] - init[n]
        assert (d0 - ds).abs().max().item() <= 2 * 1e-3 * 3 + 1e-4, (stage, n, (d0 - ds).abs().max().item())
        # relative norm only where it is statistically stable: in a 128-element LayerNorm gain a
        # handful of sign flips of near-zero gradients moves it by several percent
        if d0.numel() >= 4096:
            rel = ((d0 - ds).norm() / (d0.norm() + 1e-12)).item()
            assert rel < 0.05, (stage, n, rel)


def test_rccl_bf16_avg_collectives_used_by_ddp_and_zero(rccl_world1):
    """The exact RCCL calls the DDP / ZeRO reducers issue (bf16 AVG all-reduce from a side stream,
    reduce-scatter, all-gather) are accepted by this torch+RCCL build (world 1 on one GPU)."""
    import torch.distributed as dist
    from distributed_training_and_deepspeed_amd.comm import logger as clog
    x = torch.randn(1 << 20, device="cuda").bfloat16()
    ref = x.clone()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        w = clog.all_reduce(x, op=dist.ReduceOp.AVG, async_op=True)
    w.wait()
    torch.cuda.synchronize()
    assert torch.equal(x, ref)
    out = torch.empty_like(x)
    clog.reduce_scatter_tensor(out, x, op=dist.ReduceOp.AVG, async_op=False)
    gat = torch.empty_like(x)
    clog.all_gather_into_tensor(gat, out, async_op=False)
    torch.cuda.synchronize()
    assert torch.equal(gat, ref)


def test_rccl_streams_are_high_priority(rccl_world1):
    """comm.init creates RCCL's internal streams with high priority (DTD_RCCL_HIGH_PRIORITY
    default), so backward-overlapped collectives get freed CUs first; a collective still works."""
    import torch.distributed as dist
    pg = dist.distributed_c10d._get_default_group()
    backend = pg._get_backend(torch.device("cuda", 0))
    assert backend.options.is_high_priority_stream
    t = torch.full((1024,), 2.0, device="cuda", dtype=torch.bfloat16)
    dist.all_reduce(t, op=dist.ReduceOp.AVG)
    torch.cuda.synchronize()
    assert torch.all(t == 2.0)


def test_ddp_deferred_finalize_no_sync_matches_inline(monkeypatch):
    """World 1 with DTD_DEFER_FINALIZE=1 (bias / LN finalizes on the side stream): a no_sync
    micro-step followed by a synced one accumulates exactly the gradients of the inline schedule
    (the no_sync backward joins its side-stream writes before returning)."""
    from distributed_training_and_deepspeed_amd.data import SyntheticLMDataset
    from distributed_training_and_deepspeed_amd.models import build_model
    from distributed_training_and_deepspeed_amd.ops.grad import _ASYNC
    from distributed_training_and_deepspeed_amd.parallel import DistributedDataParallel
    ds = SyntheticLMDataset(build_model("tiny").cfg, 4 * 3, seq_len=128, seed=5)
    ids = ds.input_ids.view(3, 4, 128).cuda()
    lab = ds.labels.view(3, 4, 128).cuda()
    grads = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("DTD_DEFER_FINALIZE", mode)
        model = build_model("tiny", dtype=torch.bfloat16, device="cuda", seed=3)
        ddp = DistributedDataParallel(model)
        assert ddp._defer_finalize == (mode == "1")
        with ddp.no_sync():
            ddp(ids[0], labels=lab[0]).loss.backward()
        assert not _ASYNC.defer_finalize          # the no_sync backward closed the deferral window
        ddp(ids[1], labels=lab[1]).loss.backward()
        torch.cuda.synchronize()
        grads[mode] = {n: p.main_grad.detach().clone() for n, p in model.named_parameters()}
        with torch.no_grad():                     # a grad-free forward opens no deferral window
            ddp(ids[2], labels=lab[2])
        assert not _ASYNC.defer_finalize
    for n in grads["0"]:
        assert torch.equal(grads["0"][n], grads["1"][n]), n
