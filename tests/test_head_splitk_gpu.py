"""K-split input gradient of a big-vocabulary LM head (``ops/gemm.py`` head_dgrad): dLogits [M, V]
. E [V, h] as one strided-batch GEMM over vocabulary ranges with fp32 partials, vs fp32 PyTorch,
at bloom-560m's micro-batch-1 shape (M = 511, V = 250880, h = 1024) and a GPT-2-sized vocabulary."""
import pytest
import torch

from distributed_training_and_deepspeed_amd.ops import gemm as G

pytestmark = pytest.mark.gpu


@pytest.fixture
def splitk():
    prev = G._HEAD_SPLITK[0]
    yield
    G.set_head_splitk(prev)


@pytest.mark.parametrize("M,V,h,s", [(511, 250880, 1024, 8), (511, 250880, 1024, 16), (255, 50304, 768, 4)])
def test_head_dgrad_splitk_matches_fp32(splitk, M, V, h, s):
    g = torch.Generator(device="cuda").manual_seed(0)
    a = (torch.randn(M, V, device="cuda", generator=g) * 1e-2).bfloat16()
    w = torch.randn(V, h, device="cuda", generator=g).bfloat16()
    ref = a.float() @ w.float()
    G.set_head_splitk(s)
    out = G.head_dgrad(a, w)
    assert out.dtype == torch.bfloat16 and out.shape == (M, h)
    err = ((out.float() - ref).norm() / ref.norm()).item()
    assert err < 4e-3, err
    G.set_head_splitk(0)
    lib = G.head_dgrad(a, w)
    err_lib = ((lib.float() - ref).norm() / ref.norm()).item()
    assert err <= err_lib * 1.05 + 1e-4, (err, err_lib)   # fp32 partials: no worse than one pass
