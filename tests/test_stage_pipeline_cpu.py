"""One pipeline stage per process (parallel/stage_pipeline.py), CPU / gloo, world 2 and 3.

Every rank builds the same seeded BertModelWithMP, keeps its np.array_split module group and runs
GPipe (fill-drain) or 1F1B over 4 micro-batches with activations / gradients sent between
ranks (receives posted a micro-batch ahead, non-blocking sends), with and without activation
recompute.  The stage gradients and loss must equal the sequential model's for ONE
CrossEntropyLoss over the concatenated batch with real MLM labels (-100 on the unmasked tokens),
as the reference computes it, in fp32; the "mean" weighting must equal the mean of the
micro-batch means.  Reference: model/bert_mp.py:39-47,73-99, model_parallel_training.py:43-44,65-78.
"""
import os

import pytest
import torch
import torch.multiprocessing as mp

from .conftest import pick_free_port


def _cfg():
    from distributed_training_and_deepspeed_amd.models import get_config
    return get_config("bert-tiny").with_(hidden_dropout=0.0, attn_dropout=0.0, num_layers=4)


def _batch(cfg):
    from distributed_training_and_deepspeed_amd.data import SyntheticLMDataset
    ds = SyntheticLMDataset(cfg, 8, seq_len=32, seed=4)
    return ds.input_ids, ds.labels


def _loss(cfg):
    from distributed_training_and_deepspeed_amd.ops import functional as Fx
    ce = Fx.CrossEntropyLoss()
    return lambda out, t: ce(out.reshape(-1, cfg.vocab_size).float(), t.reshape(-1))


def _worker(rank, world, port, out_dir, schedule, device, impl="reference", checkpoint="never", weighting="tokens",
            overlap=True):
    import torch.distributed as dist
    from distributed_training_and_deepspeed_amd.parallel.stage_pipeline import StagePipeline, bert_stage
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = _cfg()
    dev = torch.device(device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    owner, mods = bert_stage(cfg, rank, world, dev, dtype=torch.float32, impl=impl, seed=7)
    ids, labels = _batch(cfg)
    pipe = StagePipeline(mods, rank, world, dev, act_shape=lambda mb: (mb, ids.shape[1], cfg.hidden_size),
                         act_dtype=torch.float32, loss_fn=_loss(cfg), chunks=4, schedule=schedule,
                         checkpoint=checkpoint, loss_weighting=weighting, overlap=overlap)
    loss = pipe.train_step(ids.to(dev) if rank == 0 else None, labels.to(dev) if rank == world - 1 else None,
                           rows=ids.shape[0])
    names = {id(p): n for n, p in owner.named_parameters()}
    grads = {names[id(p)]: p.grad.detach().cpu().clone() for p in pipe.parameters() if p.grad is not None}
    torch.save({"grads": grads, "loss": None if loss is None else loss.cpu()},
               os.path.join(out_dir, f"stage{rank}.pt"))
    dist.destroy_process_group()


def _sequential(weighting="tokens"):
    """The reference's loss: one CrossEntropyLoss over the concatenated batch ("tokens"), or the
    mean of the 4 micro-batch means ("mean")."""
    from distributed_training_and_deepspeed_amd.models.bert_mp import BertModelWithMP
    cfg = _cfg()
    model = BertModelWithMP(config=cfg, devices=["cpu"], dtype=torch.float32, impl="reference", timing="host", seed=7)
    ids, labels = _batch(cfg)
    loss_fn, total = _loss(cfg), 0.0
    if weighting == "tokens":
        loss = loss_fn(model(ids), labels)
        loss.backward()
        total = float(loss.detach())
    else:
        for x, t in zip(torch.chunk(ids, 4), torch.chunk(labels, 4)):
            loss = loss_fn(model(x), t) / 4
            loss.backward()
            total += float(loss.detach())
    return {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}, total


def test_batch_has_unequal_labelled_counts_per_micro_batch():
    """The check below is only meaningful when the micro-batches' labelled-token counts differ."""
    _, labels = _batch(_cfg())
    counts = [int((t != -100).sum()) for t in torch.chunk(labels, 4)]
    assert len(set(counts)) > 1 and 0 < min(counts), counts


def test_micro_loss_weights_sum_to_the_concatenated_loss():
    from distributed_training_and_deepspeed_amd.parallel.stage_pipeline import micro_loss_weights
    torch.manual_seed(0)
    logits = torch.randn(8, 16, 10)
    labels = torch.randint(0, 10, (8, 16))
    labels[torch.rand(8, 16) < 0.8] = -100
    ce = torch.nn.CrossEntropyLoss()
    w = micro_loss_weights(labels, 4)
    parts = sum(ce(x.reshape(-1, 10), t.reshape(-1)) * w[m]
                for m, (x, t) in enumerate(zip(torch.chunk(logits, 4), torch.chunk(labels, 4))))
    assert torch.allclose(parts, ce(logits.reshape(-1, 10), labels.reshape(-1)), rtol=1e-5)


@pytest.mark.parametrize("world,schedule,checkpoint,weighting,overlap", [
    (2, "gpipe", "never", "tokens", True), (2, "1f1b", "never", "tokens", True), (3, "gpipe", "never", "tokens", True),
    (3, "1f1b", "never", "tokens", True), (2, "gpipe", "except_last", "tokens", True),
    (3, "1f1b", "except_last", "tokens", True), (2, "1f1b", "always", "tokens", True),
    (2, "gpipe", "never", "mean", True), (3, "gpipe", "never", "tokens", False)])
def test_stage_per_process_matches_sequential(tmp_path, world, schedule, checkpoint, weighting, overlap):
    mp.spawn(_worker, args=(world, pick_free_port(), str(tmp_path), schedule, "cpu", "reference", checkpoint,
                            weighting, overlap), nprocs=world, join=True)
    ref, ref_loss = _sequential(weighting)
    seen = set()
    for r in range(world):
        res = torch.load(tmp_path / f"stage{r}.pt", weights_only=True)
        for n, g in res["grads"].items():
            assert torch.allclose(g, ref[n], rtol=1e-4, atol=1e-6), (schedule, checkpoint, r, n,
                                                                     (g - ref[n]).abs().max().item())
            seen.add(n)
        if r == world - 1:
            assert abs(float(res["loss"]) - ref_loss) < 1e-5
    assert seen == set(ref), set(ref) - seen          # every parameter lives on exactly one stage
