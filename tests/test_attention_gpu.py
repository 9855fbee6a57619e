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
    (2, 64, 2, 64, False, False, 0.1),     # S < one 128-query tile: waves past W clamp their mask rows
    (3, 96, 2, 64, False, False, 0.1),     # W = 3: the last key block's keep words clamp into the row
]


def _form(monkeypatch, fwd):
    """single: attn_fwd_kernel; pipe: attn_fwd_pipe_kernel; pk: packed-fp32 softmax forms of the
    forward and dQ kernels."""
    monkeypatch.setenv("DTD_ATTN_FWD", "pipe" if fwd == "pipe" else "single")
    monkeypatch.setenv("DTD_ATTN_FWD_PK", "1" if fwd == "pk" else "0")


@pytest.mark.parametrize("fwd", ["single", "pipe", "pk"])
@pytest.mark.parametrize("B,S,H,D,causal,alibi,p", CASES)
def test_flash_attention_fwd_bwd(B, S, H, D, causal, alibi, p, fwd, monkeypatch):
    _form(monkeypatch, fwd)
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
    # qkv bias gradient from the backward epilogues (column partials) == column sums of dqkv
    db = torch.full((3 * H * D,), 0.25, device="cuda", dtype=torch.float32)
    dq_b = A.attn_bwd(dctx.cuda(), qkv.cuda(), ctx_g, lse_g, B, S, H, D, causal, slopes, p, rg, 9, mk,
                      dbias=(db, True))
    assert torch.equal(dq_b, dq_g)
    ref_db = dq_g.float().sum(0)
    assert ((db - 0.25) - ref_db).abs().max().item() <= 1e-3 * (ref_db.abs().max().item() + 1.0)


@pytest.mark.parametrize("S,p", [(512, 0.1), (512, 0.0), (384, 0.1), (256, 0.0), (128, 0.1)])
def test_fused_backward_matches_reference_and_split(S, p):
    """attn_bwd_fused_kernel (one workgroup per (batch, head), dQ summed in LDS, no atomics) vs the
    fp32 math reference and vs the split dQ + dK/dV kernels; the qkv-bias column sums from its
    epilogues equal the column sums of the dqkv it wrote.  H = 3 so (batch, head) decoding and
    the bias rows of several heads are exercised."""
    if not A.fused_bwd_built():
        pytest.skip("the one-kernel backward is compiled only into experimental builds (DTD_BUILD_EXPERIMENTAL=1)")
    B, H, D = 2, 3, 64
    torch.manual_seed(1)
    qkv = torch.randn(B * S, 3 * H * D).to(torch.bfloat16)
    dctx = torch.randn(B * S, H * D).to(torch.bfloat16)
    rg, rc = RngState(5, device="cuda"), RngState(5, device="cpu")
    assert A.fused_bwd_applies(S, D, False, None)
    ctx_g, lse_g, mk = A.attn_fwd(qkv.cuda(), B, S, H, D, False, None, p, rg, 3)
    ctx_r, lse_r = A.attn_fwd_ref(qkv, B, S, H, D, False, None, p, rc, 3)
    dq_r = A.attn_bwd_ref(dctx, qkv, ctx_r, lse_r, B, S, H, D, False, None, p, rc, 3).view(B, S, 3, H, D)
    out = {}
    for form in ("split", "fused", "fused4"):
        prev = A.set_bwd_form(form)
        try:
            db = torch.zeros(3 * H * D, device="cuda", dtype=torch.float32)
            g = A.attn_bwd(dctx.cuda(), qkv.cuda(), ctx_g, lse_g, B, S, H, D, False, None, p, rg, 3, mk,
                           dbias=(db, True))
            torch.cuda.synchronize()
        finally:
            A.set_bwd_form(prev)
        out[form] = g
        gv = g.view(B, S, 3, H, D).cpu()
        for i, name in enumerate("qkv"):
            e = rel(gv[:, :, i], dq_r[:, :, i])
            assert e < 2e-2, f"{form} d{name} rel err {e}"
        ref_db = g.float().sum(0)
        assert (db - ref_db).abs().max().item() <= 1e-3 * (ref_db.abs().max().item() + 1.0), form
    assert rel(out["fused"], out["split"]) < 1e-2
    assert rel(out["fused4"], out["split"]) < 1e-2


@pytest.mark.parametrize("B,S,H,D,causal,alibi,p", [c for c in CASES if c[3] == 64] + [(4, 512, 12, 64, False, False, 0.1)])
def test_pipelined_forward_is_bitwise_the_single_stage_forward(B, S, H, D, causal, alibi, p, monkeypatch):
    """attn_fwd_pipe_kernel (next tile's score MFMAs under this tile's softmax) reorders issue,
    not arithmetic: output and LSE equal attn_fwd_kernel's bit for bit."""
    torch.manual_seed(3)
    qkv = torch.randn(B * S, 3 * H * D, device="cuda").to(torch.bfloat16)
    slopes = A.alibi_slopes(H).cuda() if alibi else None
    outs = {}
    for fwd in ("single", "pipe"):
        monkeypatch.setenv("DTD_ATTN_FWD", fwd)
        rg = RngState(17, device="cuda")
        outs[fwd] = A.attn_fwd(qkv, B, S, H, D, causal, slopes, p, rg, 2)
    torch.cuda.synchronize()
    assert torch.equal(outs["single"][0], outs["pipe"][0])
    assert torch.equal(outs["single"][1], outs["pipe"][1])


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


def _spiked_qkv(B, S, H, D, spikes):
    """Random q/k/v plus, in head 0, one query direction u shared by every query and keys
    set to c*u at chosen positions: the running max of each query row jumps by ~11.5*c log2
    units at those keys' tiles (c = 1 crosses the defer-max threshold, 0.5 stays under it)."""
    torch.manual_seed(1)
    x = (torch.randn(B, S, 3, H, D) * 0.5)
    u = torch.ones(D)
    x[:, :, 0, 0] = u
    for key, c in spikes:
        x[:, key, 1, 0] = c * u
    return x.reshape(B * S, 3 * H * D).to(torch.bfloat16)


def _fwd_fp64(qkv, B, S, H, D, causal):
    x = qkv.double().view(B, S, 3, H, D)
    q, k, v = (x[:, :, i].transpose(1, 2) for i in range(3))
    s = q @ k.transpose(-1, -2) / D ** 0.5
    if causal:
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool).triu(1), float("-inf"))
    lse = torch.logsumexp(s, -1)
    ctx = torch.softmax(s, -1) @ v
    return ctx.transpose(1, 2).reshape(B * S, H * D), lse


@pytest.mark.parametrize("fwd", ["single", "pipe", "pk"])
@pytest.mark.parametrize("causal", [False, True])
def test_defer_max_rescale_branch_forced(monkeypatch, causal, fwd):
    """SKILL rule 26: the defer-max rescale is data dependent.  Force it at chosen tiles (and a
    sub-threshold growth in between), check the FULL output against an fp64 host reference,
    and check that the shipped threshold and THR=0 (rescale on every growth) agree."""
    _form(monkeypatch, fwd)
    B, S, H, D = 2, 512, 2, 64
    qkv = _spiked_qkv(B, S, H, D, [(70, 1.0), (200, 1.5), (330, 2.5), (460, 2.6)])
    ref_ctx, ref_lse = _fwd_fp64(qkv, B, S, H, D, causal)
    outs = {}
    for thr in ("0", "8", "1000"):
        monkeypatch.setenv("DTD_ATTN_RESCALE_THR", thr)
        ctx, lse, _ = A.attn_fwd(qkv.cuda(), B, S, H, D, causal, None, 0.0, None, 0)
        torch.cuda.synchronize()
        outs[thr] = (ctx.double().cpu(), lse.double().cpu())
        assert torch.isfinite(outs[thr][0]).all()
        err = (outs[thr][0] - ref_ctx).abs().max().item()
        assert err < 3e-2, (thr, err)
        assert (outs[thr][1] - ref_lse).abs().max().item() < 2e-2, thr
    d = (outs["0"][0] - outs["8"][0]).abs().max().item()
    assert d < 2e-2, d


@pytest.mark.parametrize("S", [512, 200, 100, 64])
def test_mask_generator_matches_reference_bits(S):
    """Both keep-bit layouts written by the HIP generator decode to ops/rng.attn_keep_mask."""
    from distributed_training_and_deepspeed_amd.ops.rng import attn_keep_mask
    B, H, D, p = 2, 3, 64, 0.1
    rg = RngState(21, device="cuda")
    pend = A.attn_masks_async(B, S, H, D, p, rg, 6, torch.device("cuda"))
    torch.cuda.current_stream().wait_event(pend.event)
    a, b = A.decode_masks(pend.masks, B, H, S)   # [bh][q][key] from each layout
    ref = attn_keep_mask(B, H, S, p, 21, 0, 6).view(B * H, S, S).to(torch.int64)
    assert torch.equal(a, ref)
    assert torch.equal(b, ref)


@pytest.mark.parametrize("B,S,H,D,causal,alibi,p", CASES)
def test_f32_attention_kernels_match_fp64(B, S, H, D, causal, alibi, p):
    """Reference-precision path (ops/csrc/attention_f32.hip, exact f32 MFMA products): forward
    output / LSE and dQ, dK, dV against an fp64 evaluation of the same math (same dropout masks:
    the kernel takes the bits of the HIP generator, the reference regenerates them bit-identically)."""
    torch.manual_seed(1)
    qkv = torch.randn(B * S, 3 * H * D, dtype=torch.float32)
    dctx = torch.randn(B * S, H * D, dtype=torch.float32)
    slopes = A.alibi_slopes(H) if alibi else None
    rg, rc = RngState(13, device="cuda"), RngState(13, device="cpu")
    assert A.f32_kernel_supported(qkv.cuda(), D)
    ctx_g, lse_g, mk = A.attn_fwd(qkv.cuda(), B, S, H, D, causal, slopes, p, rg, 5)
    ctx_r, lse_r = A.attn_fwd_ref(qkv.double(), B, S, H, D, causal, slopes, p, rc, 5)
    assert ctx_g.dtype == torch.float32
    assert rel(ctx_g, ctx_r) < 2e-5, rel(ctx_g, ctx_r)
    assert (lse_g.cpu().double() - lse_r).abs().max().item() < 1e-4
    dq_g = A.attn_bwd(dctx.cuda(), qkv.cuda(), ctx_g, lse_g, B, S, H, D, causal, slopes, p, rg, 5, mk)
    dq_r = A.attn_bwd_ref(dctx.double(), qkv.double(), ctx_r, lse_r, B, S, H, D, causal, slopes, p, rc, 5)
    g = dq_g.view(B, S, 3, H, D).cpu().double()
    r = dq_r.view(B, S, 3, H, D)
    for i, name in enumerate("qkv"):
        e = rel(g[:, :, i], r[:, :, i])
        assert e < 5e-5, f"d{name} rel err {e}"


@pytest.mark.parametrize("S", [64, 96, 512])
def test_exact_size_mask_buffer(S):
    """The keep-bit buffer is exactly 2 x mask_words (no read slack): fwd + bwd with dropout on it
    match the reference, so every keep word the kernels use is inside it."""
    B, H, D, p = 2, 3, 64, 0.1
    masks = A.alloc_masks(B, H, S, torch.device("cuda"))
    assert masks.untyped_storage().nbytes() == 2 * A.mask_words(B, H, S) * 4
    torch.manual_seed(2)
    qkv = torch.randn(B * S, 3 * H * D).to(torch.bfloat16)
    dctx = torch.randn(B * S, H * D).to(torch.bfloat16)
    rg, rc = RngState(13, device="cuda"), RngState(13, device="cpu")
    ctx_g, lse_g, mk = A.attn_fwd(qkv.cuda(), B, S, H, D, False, None, p, rg, 3)
    assert mk.untyped_storage().nbytes() == 2 * A.mask_words(B, H, S) * 4
    ctx_r, lse_r = A.attn_fwd_ref(qkv, B, S, H, D, False, None, p, rc, 3)
    assert rel(ctx_g, ctx_r) < 1e-2
    dq_g = A.attn_bwd(dctx.cuda(), qkv.cuda(), ctx_g, lse_g, B, S, H, D, False, None, p, rg, 3, mk)
    dq_r = A.attn_bwd_ref(dctx, qkv, ctx_r, lse_r, B, S, H, D, False, None, p, rc, 3)
    assert rel(dq_g, dq_r) < 2e-2
