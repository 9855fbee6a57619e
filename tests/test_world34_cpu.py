"""Multi-rank correctness at world sizes 3 and 4 on gloo (CPU), the reference's topologies:
3 ranks in pytorch_allreduce.py (/root/reference/pytorch_allreduce.py:36-38) and the 3-node
multi-node stack (/root/reference/aws/multi_node_training_stack.py:16-18), 4 GPUs of the
single-node g4dn.12xlarge (/root/reference/aws/training_stack.py:21).

* DDP with several buckets and a no_sync micro-step at world 3 and 4 vs the single-process
  average of every rank's gradients.
* ZeRO 1/2/3 at world 3 (segment padding to multiples of 3 x 64, not a power of two) agree with
  stage 0, with gradient clipping active so the partial squared norms are all-reduced
  (``_reduce_sqnorm``).
* A ZeRO checkpoint written at world 2 loads at world 3 (re-shard from the module state).
* bench.py through ``torch.distributed.run --nproc-per-node 4``: one JSON line, n_gpus 4.
"""
import torch
import torch.multiprocessing as mp
import pytest

from distributed_training_and_deepspeed_amd.models import build_model

from . import dist_workers as W
from .conftest import pick_free_port
from .test_bench_cpu import KEYS, _run
from .test_distributed_cpu import _full_params


def _spawn(fn, world, *args):
    mp.spawn(fn, args=(world,) + args, nprocs=world, join=True)


def _avg_grads(model, world, steps_idx, n_steps):
    g = {n: torch.zeros_like(p) for n, p in model.named_parameters()}
    for r in range(world):
        ids, lab = W._batches(model.cfg, r, world, n_steps)
        for i in steps_idx:
            model.zero_grad(set_to_none=True)
            model(ids[i], labels=lab[i]).loss.backward()
            for n, p in model.named_parameters():
                g[n] += p.grad / world
    return g


@pytest.mark.parametrize("world", [3, 4])
def test_ddp_buckets_world(tmp_path, world):
    _spawn(W.ddp_worker, world, pick_free_port(), str(tmp_path), "tiny", "fused", 2, 0.05)
    res = torch.load(tmp_path / "ddp.pt", weights_only=True)
    assert len(res["buckets"]) > 2
    model = build_model("tiny", impl="fused", seed=3)
    ref = _avg_grads(model, world, (0,), 2)
    for n, g in ref.items():
        err = (res["grads0"][n] - g).abs().max().item()
        assert err <= 1e-5 * (g.abs().max().item() + 1e-6), (world, n, err)


@pytest.mark.parametrize("world", [3, 4])
def test_ddp_no_sync_world(tmp_path, world):
    _spawn(W.ddp_nosync_worker, world, pick_free_port(), str(tmp_path), "fused")
    res = torch.load(tmp_path / "nosync.pt", weights_only=True)
    model = build_model("tiny", impl="fused", seed=3)
    for key, mbs in (("acc", (0, 1)), ("fresh", (2,))):
        ref = _avg_grads(model, world, mbs, 3)
        for n, g in ref.items():
            err = (res[key][n] - g).abs().max().item()
            assert err <= 1e-5 * (g.abs().max().item() + 1e-6), (world, key, n, err)


def _param_vector(res, world):
    vals = []
    for (unit, numel, chunk, off, shapes), full in zip(res["layout"], _full_params(res, world)):
        o = 0
        for shp in shapes:
            n = 1
            for d in shp:
                n *= d
            vals.append((tuple(shp), full[o:o + n].clone()))
            o += -(-n // 64) * 64
    vals.sort(key=lambda t: (t[0], t[1].sum().item()))
    return vals


def test_zero_stages_world3_with_clipping(tmp_path):
    world, steps, gas, clip = 3, 2, 2, 0.05
    res = {}
    for stage in (0, 1, 2, 3):
        _spawn(W.zero_worker, world, pick_free_port(), str(tmp_path), "causal-tiny", stage, steps, gas, clip, "c")
        res[stage] = torch.load(tmp_path / f"zero{stage}c.pt", weights_only=True)
    _spawn(W.zero_worker, world, pick_free_port(), str(tmp_path), "causal-tiny", 1, steps, gas, 0.0, "n")
    noclip = torch.load(tmp_path / "zero1n.pt", weights_only=True)
    for st in (1, 2, 3):   # 1/3 of the padded state per rank; padding to 3 x 64 element multiples
        assert res[st]["partition"] * world <= res[0]["partition"] + 64 * world * 40
        for unit, numel, chunk, off, shapes in res[st]["layout"]:
            assert numel % (world * 64) == 0 and chunk * world == numel
    ref = _param_vector(res[0], 1)
    for st in (1, 2, 3):
        got = _param_vector(res[st], world)
        assert len(got) == len(ref)
        for (s1, a), (s2, b) in zip(ref, got):
            assert s1 == s2
            assert torch.allclose(a, b, atol=3e-5, rtol=1e-4), (st, s1, (a - b).abs().max().item())
        assert "all_reduce" in res[st]["comms"]          # the clip norm's partial sums
    # clipping was active: the unclipped run ends elsewhere
    diff = max((a - b).abs().max().item() for (_, a), (_, b) in zip(_param_vector(noclip, world),
                                                                     _param_vector(res[1], world)))
    assert diff > 1e-5


@pytest.mark.parametrize("stage", [1, 2, 3])
def test_zero_checkpoint_world2_to_world3(tmp_path, stage):
    _spawn(W.zero_reshard_save_worker, 2, pick_free_port(), str(tmp_path), stage)
    _spawn(W.zero_reshard_load_worker, 3, pick_free_port(), str(tmp_path), stage)
    saved = torch.load(tmp_path / "saved_full.pt", weights_only=True)
    rs = [torch.load(tmp_path / f"reshard_r{r}.pt", weights_only=True) for r in range(3)]
    for r in rs:
        assert r["gs"] == 3
        for k in saved:
            assert torch.equal(saved[k], r["loaded"][k]), k
    for k in rs[0]["after"]:   # the ranks stay replicas after a training step at the new size
        assert torch.equal(rs[0]["after"][k], rs[1]["after"][k]) and torch.equal(rs[0]["after"][k], rs[2]["after"][k])
    assert any(not torch.equal(rs[0]["after"][k], saved[k]) for k in saved if saved[k].is_floating_point())


def test_bench_json_line_world4():
    r = _run(pick_free_port(), "--model", "tiny", nproc=4)
    assert KEYS <= set(r)
    assert r["n_gpus"] == 4 and r["config"]["global_batch"] == 8
    assert r["config"]["parallelism"] == "dp4"
    assert r["value"] == pytest.approx(8 * 64 / (r["ms_per_step"] / 1e3), rel=2e-3)
