"""Projection GEMM + bias + hidden dropout + residual + LayerNorm in one kernel (ops/csrc/gemm_ln.hip)
against an fp32 PyTorch reference of the same op and against the unfused path it replaces
(hipBLASLt Linear, then ops.functional.ln_fwd)."""
import pytest
import torch

from distributed_training_and_deepspeed_amd.ops import functional as Fx
from distributed_training_and_deepspeed_amd.ops import gemm as G
from distributed_training_and_deepspeed_amd.ops.rng import RngState, keep_mask

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _experimental_build():
    if not G._lib.has("dtd_gemm_ln"):
        pytest.skip("gemm_ln.hip is compiled only into experimental builds (DTD_BUILD_EXPERIMENTAL=1)")


def _inputs(M, K, seed=0, bias=True):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = (torch.randn(M, K, device="cuda", generator=g) * 0.5).bfloat16()
    w = (torch.randn(768, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
    b = (torch.randn(768, device="cuda", generator=g) * 0.1).bfloat16() if bias else None
    r = torch.randn(M, 768, device="cuda", generator=g).bfloat16()
    gamma = (1 + 0.1 * torch.randn(768, device="cuda", generator=g)).bfloat16()
    beta = (0.1 * torch.randn(768, device="cuda", generator=g)).bfloat16()
    return x, w, b, r, gamma, beta


def _reference(x, w, b, r, gamma, beta, eps, p, rng, sid):
    """fp32 math with the kernel's two roundings: the projection output stored as bf16, and the
    keep bits of the counter RNG (ops/rng.py keep_mask, the law norm.hip regenerates)."""
    y = x.float() @ w.float().t()
    if b is not None:
        y = y + b.float()
    y = y.bfloat16().float()
    if p > 0:
        seed, step = (int(v) for v in rng.state.tolist())
        keep = keep_mask(y.numel(), p, seed, step, sid, device=y.device).view_as(y)
        y = y * keep / (1 - p)
    z = r.float() + y
    mean = z.mean(-1)
    var = z.var(-1, unbiased=False)
    rstd = torch.rsqrt(var + eps)
    out = (z - mean[:, None]) * rstd[:, None] * gamma.float() + beta.float()
    return z, out, mean, rstd


@pytest.mark.parametrize("M,K,p,bias", [(1024, 768, 0.0, True), (1024, 768, 0.1, True), (512, 3072, 0.1, True),
                                        (256, 768, 0.1, False), (128, 64, 0.0, True)])
def test_gemm_ln_matches_fp32_reference(M, K, p, bias):
    x, w, b, r, gamma, beta = _inputs(M, K, bias=bias)
    rng = RngState(7, device="cuda")
    assert G.linear_ln_supported(x, w, r, b, gamma, beta)
    z, out, mean, rstd = G.linear_ln(x, w, b, r, gamma, beta, 1e-12, p, rng, 3, store_z=True)
    torch.cuda.synchronize()
    zr, outr, meanr, rstdr = _reference(x, w, b, r, gamma, beta, 1e-12, p, rng, 3)
    # a projection output on a bf16 rounding boundary can round the other way (different
    # accumulation order): bound the share of such elements and the error everywhere else
    dz = (z.float() - zr).abs()
    assert (dz > 0.02 + 0.01 * zr.abs()).float().mean().item() < 1e-3
    err = (out.float() - outr).abs()
    assert err.max().item() < 0.15, err.max().item()
    assert err.mean().item() < 2e-3, err.mean().item()
    assert torch.allclose(mean, meanr, atol=2e-3, rtol=1e-3)
    assert torch.allclose(rstd, rstdr, atol=1e-3, rtol=2e-3)
    if p > 0:   # identical keep bits: a dropped element leaves exactly the residual
        dropped_k = z.float() == r.float()
        dropped_r = zr.bfloat16().float() == r.float()
        assert (dropped_k != dropped_r).float().mean().item() < 1e-3


def test_gemm_ln_matches_unfused_path():
    """Against what it replaces: hipBLASLt Linear (bf16 output) + ln_fwd."""
    M, K, p = 2048, 768, 0.1
    x, w, b, r, gamma, beta = _inputs(M, K, seed=1)
    rng = RngState(9, device="cuda")
    _, out, mean, rstd = G.linear_ln(x, w, b, r, gamma, beta, 1e-12, p, rng, 5)
    y = torch.nn.functional.linear(x, w, b)
    _, out_u, mean_u, rstd_u = Fx.ln_fwd(y, r, gamma, beta, 1e-12, p, rng, 5, store_z=False)
    torch.cuda.synchronize()
    err = (out.float() - out_u.float()).abs()
    assert err.mean().item() < 1e-3, err.mean().item()
    assert (err > 0.05).float().mean().item() < 1e-3
    assert torch.allclose(mean, mean_u, atol=1e-3, rtol=1e-3)
    assert torch.allclose(rstd, rstd_u, atol=1e-3, rtol=1e-3)


def test_gemm_ln_strided_operands_and_repeatability():
    """Row-strided views (the attention context is a view of a wider buffer) and bitwise-repeatable
    results across launches (no atomics, fixed reduction order)."""
    M, K = 512, 768
    x, w, b, r, gamma, beta = _inputs(M, K, seed=2)
    xw = torch.zeros(M, K + 64, device="cuda", dtype=torch.bfloat16)
    xw[:, :K] = x
    xv = xw[:, :K]
    rng = RngState(3, device="cuda")
    a = G.linear_ln(xv, w, b, r, gamma, beta, 1e-5, 0.1, rng, 1)
    c = G.linear_ln(x, w, b, r, gamma, beta, 1e-5, 0.1, rng, 1)
    torch.cuda.synchronize()
    for u, v in zip(a[1:], c[1:]):
        assert torch.equal(u, v)


def test_gemm_ln_rejects_unsupported_shapes():
    x, w, b, r, gamma, beta = _inputs(256, 768)
    assert not G.linear_ln_supported(x[:200], w, r[:200], b, gamma, beta)      # M % 128
    w2 = torch.randn(1024, 768, device="cuda").bfloat16()
    r2 = torch.randn(256, 1024, device="cuda").bfloat16()
    assert not G.linear_ln_supported(x, w2, r2, None, None, None)              # hidden 1024


def test_bert_base_step_with_fused_projection_ln_matches_unfused():
    """A BERT-base training step (dropout on) through the fused sublayer outputs (DTD_GEMM_LN path)
    against the Linear + LayerNorm pair: same loss and the same gradients up to the projection
    output's bf16 rounding."""
    from distributed_training_and_deepspeed_amd.data import SyntheticLMDataset
    from distributed_training_and_deepspeed_amd.models import build_model
    from distributed_training_and_deepspeed_amd.models.config import get_config
    ds = SyntheticLMDataset(get_config("base"), 4, seq_len=128, seed=3)
    ids, lab = ds.input_ids.view(4, 128).cuda(), ds.labels.view(4, 128).cuda()
    res = {}
    prev = G.ln_fused_enabled()
    try:
        for fused in (False, True):
            G.set_ln_fused(fused)
            model = build_model("base", dtype=torch.bfloat16, device="cuda", seed=11)
            model.train()
            out = model(ids, labels=lab)
            out.loss.backward()
            res[fused] = (out.loss.item(), {n: p.grad.float().clone() for n, p in model.named_parameters()
                                            if p.grad is not None})
    finally:
        G.set_ln_fused(prev)
    (la, ga), (lb, gb) = res[False], res[True]
    assert abs(la - lb) <= 2e-3 * abs(la), (la, lb)
    assert ga.keys() == gb.keys()
    for n in ga:
        if ga[n].numel() >= 4096:
            r = ((ga[n] - gb[n]).norm() / (ga[n].norm() + 1e-12)).item()
            assert r < 0.03, (n, r)
