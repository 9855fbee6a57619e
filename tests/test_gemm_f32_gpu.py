"""Reference-precision fp32 GEMM (ops/csrc/gemm_f32.hip, exact f32 MFMA products, fp32
accumulation) vs an fp64 PyTorch oracle: NT forward/input-gradient form with bias, TN split-K
weight-gradient partials, the asymmetric-operand transpose check, and the model-level fp32 path
(DTD_GEMM_F32=1) against the library path."""
import pytest
import torch

from distributed_training_and_deepspeed_amd.ops import gemm as G

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


@pytest.fixture(params=["reg", "lds"])
def f32_on(request):
    """Every case runs on both hand-written forms (the register-direct and the LDS-staged kernel)."""
    prev = (G._F32[0], G._F32_WGRAD[0], G._F32_DG[0])
    G.set_f32(True)
    G.set_f32_kernel(request.param)
    yield
    G.set_f32_kernel("auto")
    G._F32[0], G._F32_WGRAD[0], G._F32_DG[0] = prev   # back to the process default (DTD_GEMM_F32)


# LDS form: the smaller grids launch 64-wide tiles (they fill the last round of 2 workgroups per CU
# better), 8192 x 1024 is exactly 512 128-wide tiles and takes the 128-wide form; register form:
# 768-wide products take 128 x 96 wave tiles, the others 128 x 128
@pytest.mark.parametrize("M,N,K", [(128, 128, 32), (256, 384, 64), (512, 768, 768), (1024, 3072, 768),
                                   (768, 768, 3072), (8192, 1024, 256)])
def test_gemm_f32_nt_matches_fp64(f32_on, M, N, K):
    torch.manual_seed(0)
    a = torch.randn(M, K, device="cuda")
    b = torch.randn(N, K, device="cuda")
    bias = torch.randn(N, device="cuda")
    assert G.f32_supported(M, N, K, a, b)
    c = G.gemm_f32_nt(a, b, bias)
    ref = a.double() @ b.double().t() + bias.double()
    assert rel(c, ref) < 2e-6, rel(c, ref)
    c0 = G.gemm_f32_nt(a, b)
    assert rel(c0, ref - bias.double()) < 2e-6


def test_gemm_f32_nt_strided_and_asymmetric(f32_on):
    """A = I over a strided (column-sliced) B: the result is B's slice itself; a swapped
    accumulator map would return its transpose."""
    n = 256
    eye = torch.eye(n, device="cuda")
    big = torch.randn(n, 2 * n, device="cuda")
    b = big[:, :n]                                   # ldb = 2n
    c = G.gemm_f32_nt(eye, b)                        # I . b^T = b^T
    assert torch.equal(c, b.t().contiguous())


# NN form (the input gradient dY W straight from the weight): 1024 x 3072 takes 128 x 96 wave tiles
@pytest.mark.parametrize("M,N,K", [(512, 768, 2304), (1024, 3072, 768), (256, 128, 128)])
def test_gemm_f32_nn_matches_fp64(f32_on, M, N, K):
    torch.manual_seed(2)
    a = torch.randn(M, K, device="cuda")
    b = torch.randn(K, N, device="cuda")
    ref = a.double() @ b.double()
    assert rel(G.gemm_f32_nn(a, b), ref) < 2e-6
    base = torch.randn(M, N, device="cuda")
    out = base.clone()
    G.gemm_f32_nn(a, b, out=out)
    assert rel(out, ref + base.double()) < 2e-6


def test_transpose_many_f32_exact(f32_on):
    """The batched fp32 W^T copies the input-gradient NT form reads (ops/gemm.py::prepare_transposes):
    exact, over several entries with partial 64 x 64 tiles."""
    torch.manual_seed(5)
    ws = [torch.randn(r, c, device="cuda") for r, c in ((2304, 768), (768, 3072), (100, 36), (4, 260))]
    G.clear_transposes()
    G.prepare_transposes(ws)
    for w in ws:
        wt = G._t32(w)
        assert wt is not None and torch.equal(wt, w.t()), w.shape
    G.clear_transposes()


def test_gemm_f32_nt_accumulate(f32_on):
    torch.manual_seed(4)
    a = torch.randn(1024, 768, device="cuda")
    b = torch.randn(768, 768, device="cuda")
    bias = torch.randn(768, device="cuda")
    base = torch.randn(1024, 768, device="cuda")
    out = base.clone()
    G.gemm_f32_nt(a, b, bias, out=out)
    assert rel(out, a.double() @ b.double().t() + bias.double() + base.double()) < 2e-6


@pytest.mark.parametrize("T,o,i,splits", [(512, 256, 128, 1), (4096, 768, 768, None), (8192, 768, 3072, None),
                                          (1024, 128, 384, 3)])
def test_gemm_f32_tn_splitk_matches_fp64(f32_on, T, o, i, splits):
    torch.manual_seed(1)
    dy = torch.randn(T, o, device="cuda")
    x = torch.randn(T, i, device="cuda")
    part = G.gemm_f32_tn(dy, x, splits)
    ref = dy.double().t() @ x.double()
    assert part.shape[1:] == (o, i)
    assert rel(part.double().sum(0), ref) < 2e-6, rel(part.double().sum(0), ref)


def test_gemm_f32_tn_identity_exact(f32_on):
    n = 256
    dy = torch.eye(n, device="cuda")
    x = torch.arange(n * n, device="cuda").float().view(n, n).remainder(29)
    part = G.gemm_f32_tn(dy, x, 1)
    assert torch.equal(part[0], x)


def test_fp32_model_path_matches_library(f32_on):
    """BERT-tiny in fp32: loss and every gradient through the hand-written fp32 GEMMs match the
    hipBLASLt path to fp32 rounding (the products are exact in both; only summation order differs)."""
    from distributed_training_and_deepspeed_amd.data import SyntheticLMDataset
    from distributed_training_and_deepspeed_amd.models import build_model
    out = []
    prev = (G._F32[0], G._F32_WGRAD[0], G._F32_DG[0])
    for on in (False, True):
        G.set_f32(on)                     # off: library everywhere; on: every fp32 product hand-written
        model = build_model("bert-tiny", impl="fused", dtype=torch.float32, device="cuda", seed=5)
        ds = SyntheticLMDataset(model.cfg, 4, seq_len=128, seed=3)
        loss = model(ds.input_ids.cuda(), labels=ds.labels.cuda()).loss
        loss.backward()
        torch.cuda.synchronize()
        out.append((loss.item(), {n: p.grad.double().clone() for n, p in model.named_parameters()
                                  if p.grad is not None}))
    G._F32[0], G._F32_WGRAD[0], G._F32_DG[0] = prev
    (l0, g0), (l1, g1) = out
    assert abs(l0 - l1) < 1e-5 * abs(l0)
    assert g0.keys() == g1.keys()
    for n in g0:
        assert rel(g1[n], g0[n]) < 1e-4, (n, rel(g1[n], g0[n]))
