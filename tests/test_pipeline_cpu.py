"""Model-parallel / GPipe tests on CPU "devices" (schedule + recompute semantics)."""
import torch

from distributed_training_and_deepspeed_amd.data import SyntheticLMDataset
from distributed_training_and_deepspeed_amd.models import config as C
from distributed_training_and_deepspeed_amd.models.bert_mp import BertModelWithMP
from distributed_training_and_deepspeed_amd.parallel.pipeline import array_split_sizes


def _grads(model, owner, ids, lab, V):
    owner.zero_grad(set_to_none=True)
    out = model(ids)
    loss = torch.nn.functional.cross_entropy(out.view(-1, V).float(), lab.view(-1))
    loss.backward()
    return loss.item(), {n: p.grad.clone() for n, p in owner.named_parameters() if p.grad is not None}


def test_array_split_law():
    # np.array_split(14 modules, d): emb + 12 layers + head of the reference
    assert array_split_sizes(14, 4) == [4, 4, 3, 3]
    assert array_split_sizes(14, 3) == [5, 5, 4]
    assert sum(array_split_sizes(26, 8)) == 26


def test_untied_head_parameter_count():
    with torch.device("meta"):
        pass
    m = BertModelWithMP(C.BERT_TINY, devices=["cpu"], impl="reference")
    tied_delta = C.BERT_TINY.vocab_size * C.BERT_TINY.hidden_size
    from distributed_training_and_deepspeed_amd.models import build_model, count_parameters
    assert count_parameters(m) == count_parameters(build_model("tiny")) + tied_delta


def test_gpipe_matches_sequential_without_dropout():
    cfg = C.BERT_TINY.with_(hidden_dropout=0.0, attn_dropout=0.0)
    ds = SyntheticLMDataset(cfg, 8, seq_len=32, seed=1)
    a = BertModelWithMP(cfg, devices=["cpu", "cpu", "cpu"], impl="fused", seed=4)
    l1, g1 = _grads(a, a, ds.input_ids, ds.labels, cfg.vocab_size)
    pipe = a.to_pipeline(chunks=4)
    l2, g2 = _grads(pipe, a, ds.input_ids, ds.labels, cfg.vocab_size)
    assert abs(l1 - l2) < 1e-5
    for n in g1:
        assert torch.allclose(g1[n], g2[n], atol=1e-5, rtol=1e-4), n


def test_gpipe_recompute_reproduces_dropout_masks():
    """Checkpointed micro-batches are recomputed with the same counter-RNG masks, so
    checkpoint='always' and checkpoint='never' give identical gradients with dropout on."""
    cfg = C.BERT_TINY
    ds = SyntheticLMDataset(cfg, 8, seq_len=32, seed=2)
    a = BertModelWithMP(cfg, devices=["cpu", "cpu"], impl="fused", seed=5)
    _, g_never = _grads(a.to_pipeline(chunks=4, checkpoint="never"), a, ds.input_ids, ds.labels, cfg.vocab_size)
    _, g_always = _grads(a.to_pipeline(chunks=4, checkpoint="always"), a, ds.input_ids, ds.labels, cfg.vocab_size)
    for n in g_never:
        assert torch.allclose(g_never[n], g_always[n], atol=1e-6, rtol=1e-5), n


def test_idle_time_table_shape():
    cfg = C.BERT_TINY
    a = BertModelWithMP(cfg, devices=["cpu", "cpu"], impl="fused", timing="host")
    ds = SyntheticLMDataset(cfg, 4, seq_len=16, seed=3)
    out = a(ds.input_ids)
    out.float().sum().backward()
    rows = a.tracker.table(1)
    assert rows[0] == ["Device", "Average Idle Time (ms)"] and len(rows) == 3


def test_1f1b_schedule_matches_gpipe_with_dropout():
    """1F1B and fill-drain give the same gradients (same dropout masks per micro-batch)."""
    cfg = C.BERT_TINY
    ds = SyntheticLMDataset(cfg, 8, seq_len=32, seed=1)
    V = cfg.vocab_size

    def loss_fn(out, t):
        return torch.nn.functional.cross_entropy(out.reshape(-1, V).float(), t.reshape(-1))

    res = []
    for sched in ("gpipe", "1f1b"):
        a = BertModelWithMP(cfg, devices=["cpu", "cpu", "cpu"], impl="fused", seed=4)
        a.train()
        pipe = a.to_pipeline(chunks=4, checkpoint="never")
        loss = pipe.train_step(ds.input_ids, ds.labels, loss_fn, schedule=sched)
        res.append((loss.item(), {n: p.grad.clone() for n, p in a.named_parameters() if p.grad is not None}))
    assert abs(res[0][0] - res[1][0]) < 1e-6
    for n in res[0][1]:
        assert torch.allclose(res[0][1][n], res[1][1][n], atol=1e-6), n


def test_train_step_loss_equals_one_loss_over_the_concatenated_batch():
    """train_step's token-weighted micro-batch losses give the loss and gradients of the reference's
    single CrossEntropyLoss over the concatenated pipeline output (model_parallel_training.py:68-75),
    with MLM labels whose labelled count differs per micro-batch."""
    cfg = C.BERT_TINY
    ds = SyntheticLMDataset(cfg, 8, seq_len=32, seed=1)
    V = cfg.vocab_size

    def loss_fn(out, t):
        return torch.nn.functional.cross_entropy(out.reshape(-1, V).float(), t.reshape(-1))

    counts = [int((t != -100).sum()) for t in torch.chunk(ds.labels, 4)]
    assert len(set(counts)) > 1, counts
    res = []
    for mode in ("forward", "train_step"):
        a = BertModelWithMP(cfg, devices=["cpu", "cpu"], impl="fused", seed=4)
        a.train()
        pipe = a.to_pipeline(chunks=4, checkpoint="never")
        if mode == "forward":
            loss = loss_fn(pipe(ds.input_ids), ds.labels)
            loss.backward()
        else:
            loss = pipe.train_step(ds.input_ids, ds.labels, loss_fn, schedule="1f1b")
        res.append((loss.item(), {n: p.grad.clone() for n, p in a.named_parameters() if p.grad is not None}))
    assert abs(res[0][0] - res[1][0]) < 1e-5
    for n in res[0][1]:
        assert torch.allclose(res[0][1][n], res[1][1][n], atol=1e-6, rtol=1e-4), n
