"""Flash-attention HIP kernels (MFMA, gfx950) vs the fp32 math reference.

Covers BERT (non-causal, dropout), GPT/OPT (causal), BLOOM (causal + ALiBi), head_dim 64/128,
sequence lengths that are not multiples of the tile sizes, and dropout-mask regeneration in
the backward pass (the reference uses the same counter-RNG mask)."""
import pytest
import torch

from distributed_training_and_deepspeed_amd.ops import attention as A
from distributed_training_and_deepspeed_amd.ops.rng import RngState

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


CASES = [
    # B, S, H, D, causal, alibi, p
    (2, 512, 4, 64, False, False, 0.0),
    (2, 512, 4, 64, False, False, 0.1),
    (1, 256, 2, 64, True, False, 0.0),
    (1, 256, 4, 64, True, True, 0.0),
    (2, 100, 3, 64, False, False, 0.0),
    (1, 200, 2, 64, True, True, 0.1),
    (1, 256, 2, 128, False, False, 0.0),
    (1, 160, 2, 128, True, False, 0.1),
]


@pytest.mark.parametrize("B,S,H,D,causal,alibi,p", CASES)
def test_flash_attention_fwd_bwd(B, S, H, D, causal, alibi, p):
    torch.manual_seed(0)
    qkv = torch.randn(B * S, 3 * H * D).to(torch.bfloat16)
    dctx = torch.randn(B * S, H * D).to(torch.bfloat16)
    slopes = A.alibi_slopes(H) if alibi else None
    rg, rc = RngState(11, device="cuda"), RngState(11, device="cpu")
    assert A.kernel_supported(qkv.cuda(), D)
    ctx_g, lse_g, mk = A.attn_fwd(qkv.cuda(), B, S, H, D, causal, slopes, p, rg, 9)
    ctx_r, lse_r = A.attn_fwd_ref(qkv, B, S, H, D, causal, slopes, p, rc, 9)
    assert rel(ctx_g, ctx_r) < 1e-2, rel(ctx_g, ctx_r)
    assert (lse_g.cpu() - lse_r).abs().max().item() < 2e-2
    dq_g = A.attn_bwd(dctx.cuda(), qkv.cuda(), ctx_g, lse_g, B, S, H, D, causal, slopes, p, rg, 9, mk)
    dq_r = A.attn_bwd_ref(dctx, qkv, ctx_r, lse_r, B, S, H, D, causal, slopes, p, rc, 9)
    g = dq_g.view(B, S, 3, H, D).cpu()
    r = dq_r.view(B, S, 3, H, D)
    for i, name in enumerate("qkv"):
        e = rel(g[:, :, i], r[:, :, i])
        assert e < 2e-2, f"d{name} rel err {e}"


def test_side_stream_masks_match_inline_generation():
    B, S, H, D, p = 2, 256, 4, 64, 0.1
    torch.manual_seed(0)
    qkv = torch.randn(B * S, 3 * H * D, device="cuda").to(torch.bfloat16)
    rg = RngState(5, device="cuda")
    c1, l1, m1 = A.attn_fwd(qkv, B, S, H, D, False, None, p, rg, 4)
    pend = A.attn_masks_async(B, S, H, D, p, rg, 4, qkv.device)
    assert pend is not None
    c2, l2, m2 = A.attn_fwd(qkv, B, S, H, D, False, None, p, rg, 4, masks=pend)
    torch.cuda.synchronize()
    assert torch.equal(m1, m2) and torch.equal(c1, c2) and torch.equal(l1, l2)
