"""Batched weight transposes (ops/gemm.py::prepare_transposes, gemm.hip transpose_many_kernel): one
launch at the start of a backward gives every NT input-gradient operand, bit-identical to the
per-weight transpose kernel, and training with it is bit-identical to training without it."""
import pytest
import torch

from distributed_training_and_deepspeed_amd.data import SyntheticLMDataset
from distributed_training_and_deepspeed_amd.models import build_model
from distributed_training_and_deepspeed_amd.ops import gemm as G
from distributed_training_and_deepspeed_amd.optim import hf_adamw

pytestmark = pytest.mark.gpu


def test_transpose_many_matches_transpose():
    torch.manual_seed(0)
    shapes = [(2304, 768), (768, 768), (3072, 768), (768, 3072), (72, 136), (8, 8)] * 12   # 72 > one launch
    ws = [torch.randn(r, c, device="cuda").to(torch.bfloat16) for r, c in shapes]
    G.clear_transposes()
    G.prepare_transposes(ws)
    for w in ws:
        got = G.transposed(w)
        assert got.shape == (w.shape[1], w.shape[0])
        assert torch.equal(got, w.t().contiguous())
        assert torch.equal(got, G.transpose(w))
    # a parameter moved to new storage misses the cache (fresh transpose)
    w = ws[0]
    w.data = w.data.clone() * 2
    assert torch.equal(G.transposed(w), w.t().contiguous())
    G.clear_transposes()


def test_transpose_many_skips_released_parameters():
    ws = [torch.randn(64, 64, device="cuda").to(torch.bfloat16), torch.empty(0, device="cuda", dtype=torch.bfloat16)]
    G.clear_transposes()
    G.prepare_transposes(ws)
    assert not G._WT_CACHE   # a partitioned (empty) weight in the set: no batch, per-call transposes
    G.clear_transposes()


def _train(batch: bool, name="tiny", steps=3):
    prev = G._WT_BATCH[0]
    G._WT_BATCH[0] = batch
    try:
        model = build_model(name, dtype=torch.bfloat16, device="cuda", seed=3)
        model.train()
        opt = hf_adamw(model.parameters(), lr=1e-3)
        ds = SyntheticLMDataset(build_model(name).cfg, 4 * steps, seq_len=128, mlm=name != "causal-tiny", seed=5)
        ids = ds.input_ids.view(steps, 4, 128).cuda()
        lab = ds.labels.view(steps, 4, 128).cuda()
        losses = []
        for i in range(steps):
            out = model(ids[i], labels=lab[i])
            out.loss.backward()
            opt.step()
            opt.zero_grad(set_to_none=True)
            model.rt.rng.advance()
            losses.append(out.loss.detach())
        torch.cuda.synchronize()
        return torch.stack(losses), [p.detach().clone() for p in model.parameters()]
    finally:
        G._WT_BATCH[0] = prev
        G.clear_transposes()


@pytest.mark.parametrize("name", ["tiny", "causal-tiny"])
def test_training_bit_identical_with_batched_transposes(name):
    la, pa = _train(False, name)
    lb, pb = _train(True, name)
    assert torch.equal(la, lb)
    for a, b in zip(pa, pb):
        assert torch.equal(a, b)
