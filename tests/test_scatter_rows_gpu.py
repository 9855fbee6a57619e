"""Sparse-MLM-head row gather with a one-pass scatter backward (models/layers.py::_GatherRows,
embed.hip scatter_rows_kernel): the input gradient equals index_select's autograd (zero fill +
index_add) bit for bit, for the exact-size gather and the static-capacity gather with padding."""
import pytest
import torch

from distributed_training_and_deepspeed_amd.models import layers as L

pytestmark = pytest.mark.gpu


def _ref_grad(x, idx, g):
    xr = x.detach().clone().requires_grad_(True)
    xr.index_select(0, idx).backward(g)
    return xr.grad


@pytest.mark.parametrize("row0_labelled", [True, False])
@pytest.mark.parametrize("static", [True, False])
def test_scatter_backward_matches_index_select(static, row0_labelled):
    torch.manual_seed(0)
    T, h = 4096, 768
    lab = torch.full((T,), -100, device="cuda", dtype=torch.int64)
    lab[torch.rand(T, device="cuda") < 0.15] = 7
    lab[0] = 7 if row0_labelled else -100
    valid = lab != -100
    x = torch.randn(T, h, device="cuda").to(torch.bfloat16).requires_grad_(True)
    if static:
        cap = int(valid.sum().item()) + 37            # padding entries (index 0) past the count
        idx = torch.nonzero_static(valid, size=cap, fill_value=0).squeeze(1)
        count = valid.sum()
    else:
        idx = valid.nonzero().squeeze(1)
        cap, count = idx.numel(), None
    y = L._gather_rows(x, idx, count, cap)
    assert torch.equal(y, x.detach().index_select(0, idx))
    g = torch.randn_like(y)
    n = int(valid.sum().item())
    g[n:] = 0                                          # padding rows carry no gradient (label -100)
    y.backward(g)
    assert torch.equal(x.grad, _ref_grad(x, idx, g))


def test_scatter_backward_capacity_overflow():
    """More labelled rows than the capacity: the first `cap` of them are gathered and scattered back."""
    T, h = 1024, 256
    valid = torch.rand(T, device="cuda") < 0.5
    cap = int(valid.sum().item()) // 2
    idx = torch.nonzero_static(valid, size=cap, fill_value=0).squeeze(1)
    x = torch.randn(T, h, device="cuda").to(torch.bfloat16).requires_grad_(True)
    y = L._gather_rows(x, idx, valid.sum(), cap)
    g = torch.randn_like(y)
    y.backward(g)
    assert torch.equal(x.grad, _ref_grad(x, idx, g))
