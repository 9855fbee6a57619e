"""One-wave-per-SIMD projection GEMM (ops/csrc/gemm_w4.hip) vs fp32 PyTorch.

Every plain BERT-base product the step runs on it -- the qkv / o / fc2 forward with bias and the
qkv (residual add) / o / fc1 input gradients on the transposed weight -- at T = 16384 and at
T = 524288 tokens (the b1024 x 512 step's own token count is 524288), checked against
``a.float() @ b.float().t()``; plus small and uneven tile counts (workgroups with 0, 1 and several
tiles, K = 128, the cross-tile prefetch), an asymmetric operand pair that exposes a transposed or
permuted output map, and strided operands."""
import pytest
import torch

from distributed_training_and_deepspeed_amd.ops import gemm as G

pytestmark = pytest.mark.gpu

H, F = 768, 3072
# name: (N, K, bias, add)
SHAPES = {
    "fwd_qkv": (3 * H, H, True, False),
    "fwd_o": (H, H, True, False),
    "fwd_fc2": (H, F, True, False),
    "dgrad_qkv_add": (H, 3 * H, False, True),
    "dgrad_o": (H, H, False, False),
    "dgrad_fc1": (H, F, False, False),
}


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _run(T, N, K, bias, add, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    a = torch.randn(T, K, device="cuda", generator=g).bfloat16()
    b = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
    bv = torch.randn(N, device="cuda", generator=g).bfloat16() if bias else None
    c0 = torch.randn(T, N, device="cuda", generator=g).bfloat16() if add else None
    assert G.w4_supported(T, N, K, a, b)
    if add:
        c = c0.clone()
        G.gemm_w4(a, b, out=c)
    else:
        c = G.gemm_w4(a, b, bv)
    ref = a.float() @ b.float().t()
    if bias:
        ref += bv.float()
    if add:
        ref += c0.float()
    return c, ref


@pytest.mark.parametrize("T", [16384, 524288])
@pytest.mark.parametrize("name", list(SHAPES))
def test_w4_bert_products_match_fp32(name, T):
    N, K, bias, add = SHAPES[name]
    c, ref = _run(T, N, K, bias, add)
    err = rel(c, ref)
    # one bf16 rounding of an fp32-accumulated result: ~2^-9 relative
    assert err < 4e-3, (name, T, err)
    del c, ref
    torch.cuda.empty_cache()


@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (256, 512, 192), (512, 768, 768), (2304, 768, 3072),
                                   (8448, 768, 768), (16384, 2304, 256), (256 * 300, 256, 128)])
@pytest.mark.parametrize("add", [False, True])
def test_w4_tile_counts(M, N, K, add):
    c, ref = _run(M, N, K, not add, add, seed=1)
    assert rel(c, ref) < 4e-3, rel(c, ref)


def test_w4_asymmetric_operands_detect_transpose():
    """A = I: the product is exactly B^T, so a transposed or permuted output map shows up."""
    n = 512
    a = torch.eye(n, device="cuda").bfloat16()
    b = torch.arange(n * n, device="cuda").float().view(n, n).remainder(97).bfloat16()
    c = G.gemm_w4(a, b)
    assert torch.equal(c, b.t().contiguous())


def test_w4_strided_operands_and_output():
    torch.manual_seed(3)
    big_a = torch.randn(1024, 1024 + 64, device="cuda").bfloat16()
    big_b = torch.randn(512, 1024 + 128, device="cuda").bfloat16()
    a, b = big_a[:, :1024], big_b[:, :1024]
    out = torch.randn(1024, 512 + 256, device="cuda").bfloat16()
    view = out[:, :512]
    before = out.clone()
    G.gemm_w4(a, b, out=view)
    ref = before[:, :512].float() + a.float() @ b.float().t()
    assert rel(view, ref) < 4e-3
    assert torch.equal(out[:, 512:], before[:, 512:])   # nothing written outside the view


def test_w4_model_dispatch_matches_library():
    """linear_any / dgrad / dgrad_add_ with the kernel on vs hipBLASLt, same inputs (T large enough
    for every product to pass the tile-count rule, which is checked too)."""
    torch.manual_seed(4)
    T = 256 * 1024
    x = torch.randn(T, H, device="cuda").bfloat16()
    w = (torch.randn(3 * H, H, device="cuda") * 0.05).bfloat16()
    bias = torch.randn(3 * H, device="cuda").bfloat16()
    dy = torch.randn(T, 3 * H, device="cuda").bfloat16()
    res = torch.randn(T, H, device="cuda").bfloat16()
    prev = (G._W4[0], G._W4_ADD[0])
    assert (T // 256) * (H // 256) >= G.w4_min_tiles()
    try:
        outs = {}
        for on in (False, True):
            G.set_w4(on, add=on)
            G.clear_transposes()
            r = res.clone()
            outs[on] = (G.linear_any(x, w, bias), G.dgrad(dy, w), G.dgrad_add_(r, dy, w))
        for lib_out, w4_out in zip(outs[False], outs[True]):
            assert rel(w4_out, lib_out) < 4e-3
    finally:
        G.set_w4(*prev)


def test_w4_dispatch_tile_rule():
    """Small products (the b4 step's 2048 tokens) stay on the library, large ones take the kernel."""
    n = G.w4_min_tiles()
    assert G.w4_supported(2048, 768, 768) and not G._w4_pick(2048, 768, 768)
    m = 256 * ((n + 2) // 3)
    assert G._w4_pick(m, 768, 768) == G.w4_enabled()
