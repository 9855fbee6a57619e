"""Hand-written MFMA GEMM (ops/csrc/gemm.hip) and its fused FFN epilogues vs fp32 PyTorch."""
import pytest
import torch

from distributed_training_and_deepspeed_amd.ops import functional as Fx
from distributed_training_and_deepspeed_amd.ops import gemm as G

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (256, 512, 192), (512, 768, 768), (1024, 3072, 768),
                                   (768, 768, 3072), (512, 768, 2304)])
def test_gemm_bt_matches_fp32(M, N, K):
    torch.manual_seed(0)
    a = torch.randn(M, K, device="cuda").bfloat16()
    b = torch.randn(N, K, device="cuda").bfloat16()
    bias = torch.randn(N, device="cuda").bfloat16()
    assert G.supported(M, N, K, a, b)
    c = G.gemm_bt(a, b, bias)
    ref = a.float() @ b.float().t() + bias.float()
    assert rel(c, ref) < 1e-2, rel(c, ref)


def test_gemm_bt_asymmetric_operands_detect_transpose():
    """A = I with an asymmetric B: a swapped accumulator map would return B^T (SKILL §3)."""
    n = 256
    a = torch.eye(n, device="cuda").bfloat16()
    b = torch.arange(n * n, device="cuda").float().view(n, n).remainder(97).bfloat16()
    c = G.gemm_bt(a, b)           # I . B^T = B^T
    assert torch.equal(c, b.t().contiguous())


def _gelu_ref(x, act):
    if act == "relu":
        return torch.relu(x)
    if act == "gelu":
        return 0.5 * x * (1 + torch.erf(x / 2 ** 0.5))
    return 0.5 * x * (1 + torch.tanh(0.7978845608028654 * (x + 0.044715 * x ** 3)))


def _gelu_grad_ref(x, act):
    if act == "relu":
        return (x > 0).float()
    if act == "gelu":
        return 0.5 * (1 + torch.erf(x / 2 ** 0.5)) + x * torch.exp(-0.5 * x * x) / (2 * torch.pi) ** 0.5
    k = 0.7978845608028654
    t = torch.tanh(k * (x + 0.044715 * x ** 3))
    return 0.5 * (1 + t) + 0.5 * x * (1 - t * t) * k * (1 + 3 * 0.044715 * x * x)


# (8448, 768) / (16384, 768) / (8448, 512): more tiles than workgroups, so every persistent
# workgroup runs several epilogues back to back (uneven tile counts per workgroup)
@pytest.mark.parametrize("M,K", [(512, 768), (8448, 768), (16384, 768), (8448, 512)])
@pytest.mark.parametrize("act", ["gelu", "gelu_tanh", "relu"])
def test_linear_gelu_epilogue(act, M, K):
    torch.manual_seed(1)
    N = 3072
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    b = torch.randn(N, device="cuda").bfloat16()
    u, a = G.linear_gelu(x, w, b, act)
    uref = x.float() @ w.float().t() + b.float()
    assert rel(u, uref) < 1e-2
    # the activation is GELU of the stored (bf16) pre-activation: the unfused kernel's value
    # (same formula; at most a bf16 rounding step apart where the compilers contract differently)
    unf = Fx.act_fwd(u, act)
    assert (a.float() - unf.float()).abs().max().item() <= 1e-2 * max(1.0, unf.float().abs().max().item())
    assert rel(a, unf) < 1e-3
    assert rel(a, _gelu_ref(u.float(), act)) < 1e-2


@pytest.mark.parametrize("act", ["gelu", "gelu_tanh", "relu"])
def test_gelu_bwd_gemm_epilogue_and_bias_grad(act):
    torch.manual_seed(2)
    M, H, F = 512, 768, 3072
    dy = torch.randn(M, H, device="cuda").bfloat16()
    w2 = (torch.randn(H, F, device="cuda") * 0.05).bfloat16()        # fc2 weight [out=H, in=F]
    u = torch.randn(M, F, device="cuda").bfloat16()
    db = torch.full((F,), 0.5, device="cuda", dtype=torch.float32)
    du = G.gelu_bwd_gemm(dy, w2.t().contiguous(), u, dbias=(db, True), act=act)
    # unfused path: da = dy @ W2 (bf16), du = act_bwd(da, u)
    da = dy @ w2
    db_ref = torch.zeros(F, device="cuda", dtype=torch.float32)
    du_ref = Fx.act_bwd(da, u, act, dbias=(db_ref, False))
    assert rel(du, du_ref) < 1e-2, rel(du, du_ref)
    assert rel(db - 0.5, db_ref) < 1e-2
    # vs fp32 math
    g = _gelu_grad_ref(u.float(), act)
    assert rel(du, (dy.float() @ w2.float()) * g) < 2e-2


def test_gemm_nt_add_in_place_and_transpose():
    torch.manual_seed(3)
    M, N, K = 512, 768, 2304
    dy = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(K, N, device="cuda") * 0.05).bfloat16()          # qkv weight [out=K, in=N]
    wt = G.transpose(w)
    assert torch.equal(wt, w.t().contiguous())
    c = torch.randn(M, N, device="cuda").bfloat16()
    ref = c.float() + dy.float() @ w.float()
    G.matmul_nt_add_(c, dy, wt)
    assert rel(c, ref) < 1e-2, rel(c, ref)
    # odd transpose shapes (tile edges)
    x = torch.randn(100, 37, device="cuda").bfloat16()
    assert torch.equal(G.transpose(x), x.t().contiguous())


def test_gemm_strided_operands_and_many_tiles():
    """Row-strided views (lda > K) and a grid that is not a multiple of the 8 XCDs."""
    torch.manual_seed(4)
    M, N, K = 256 * 5, 256 * 3, 128
    big = torch.randn(M, K + 64, device="cuda").bfloat16()
    a = big[:, :K]
    b = torch.randn(N, K, device="cuda").bfloat16()
    assert G.supported(M, N, K, a, b)
    c = G.gemm_bt(a, b)
    assert rel(c, a.float() @ b.float().t()) < 1e-2


@pytest.mark.parametrize("T,o,i,splits", [(64, 256, 256, 1), (4096, 768, 3072, None), (8192, 2304, 768, 5),
                                          (1024, 512, 256, 64)])
def test_wgrad_tn_matches_fp32(T, o, i, splits):
    """dW = dy^T x through the TN kernel's split-K partials (incl. empty splits) + the reduce."""
    from distributed_training_and_deepspeed_amd.ops.grad import splitk_reduce
    torch.manual_seed(5)
    dy = torch.randn(T, o, device="cuda").bfloat16()
    x = torch.randn(T, i, device="cuda").bfloat16()
    assert G.wgrad_supported(dy, x)
    part = G.wgrad_tn(dy, x, splits)
    ref = dy.float().t() @ x.float()
    assert rel(part.sum(0), ref) < 2e-3, rel(part.sum(0), ref)
    dst = torch.full((o, i), 1.0, device="cuda", dtype=torch.float32)
    splitk_reduce(part, dst, True)
    assert rel(dst - 1.0, ref) < 2e-3


@pytest.mark.parametrize("variant", [4, 5, 44])
@pytest.mark.parametrize("T,o,i,splits", [(32, 256, 256, 1), (16384, 2304, 768, None), (16384, 768, 768, None),
                                          (16384, 3072, 768, None), (16384, 768, 3072, None),
                                          (4128, 512, 256, 7), (96, 256, 512, 8)])
def test_wgrad_tn_ring_matches_fp32(T, o, i, splits, variant):
    """Ring-pipelined TN weight-gradient kernel (ops/csrc/wgrad.hip) on every BERT-base weight
    shape, uneven ranges (4128 tokens = 129 K-steps over 7 ranges) and ranges shorter than the
    ring / empty ranges (96 tokens over 8), against an fp32 dy^T x."""
    from distributed_training_and_deepspeed_amd.ops.grad import splitk_reduce
    torch.manual_seed(7)
    dy = torch.randn(T, o, device="cuda").bfloat16()
    x = torch.randn(T, i, device="cuda").bfloat16()
    assert G.wgrad_supported(dy, x)
    part = G.wgrad_tn(dy, x, splits, variant=variant)
    ref = dy.float().t() @ x.float()
    assert rel(part.sum(0), ref) < 2e-3, rel(part.sum(0), ref)
    dst = torch.full((o, i), 1.0, device="cuda", dtype=torch.float32)
    splitk_reduce(part, dst, True)
    assert rel(dst - 1.0, ref) < 2e-3


@pytest.mark.parametrize("variant", [4, 5, 44])
def test_wgrad_tn_asymmetric_and_strided(variant):
    """I^T x = x exactly (a swapped accumulator map would return a transposed / permuted tile), on
    column-sliced (strided) operands."""
    T, n = 512, 256
    big = torch.zeros(T, 3 * n, device="cuda").bfloat16()
    big[:, n:2 * n] = torch.eye(n, device="cuda").bfloat16().repeat(T // n, 1)
    dy = big[:, n:2 * n]
    xb = torch.arange(T * 2 * n, device="cuda").float().view(T, 2 * n).remainder(13).bfloat16()
    x = xb[:, n:]
    part = G.wgrad_tn(dy, x, 1, variant=variant)
    ref = (dy.float().t() @ x.float())
    assert torch.equal(part[0], ref)


def test_wgrad_tn_asymmetric_detects_transpose():
    T, n = 256, 256
    dy = torch.eye(n, device="cuda").bfloat16().repeat(T // n, 1)          # [T, n]
    x = torch.arange(T * n, device="cuda").float().view(T, n).remainder(13).bfloat16()
    part = G.wgrad_tn(dy, x, 1)
    assert torch.equal(part[0], x.float())       # I^T x = x (exact small integers)


def test_tn_wgrad_path_in_model_matches_default():
    """The TN weight-gradient kernel (default; taken for every layer weight at >= 8192 tokens)
    gives the same gradients as the hipBLASLt split-K path (DTD_GEMM_WGRAD=0)."""
    from distributed_training_and_deepspeed_amd.data import SyntheticLMDataset
    from distributed_training_and_deepspeed_amd.models import build_model
    grads = []
    prev = G._WGRAD[0]
    for on in (False, True):
        G._WGRAD[0] = on
        try:
            model = build_model("bert-base-cased", dtype=torch.bfloat16, device="cuda", seed=11)
            ds = SyntheticLMDataset(model.cfg, 16, seq_len=512, seed=2)          # 8192 tokens
            model(ds.input_ids.cuda(), labels=ds.labels.cuda()).loss.backward()
            torch.cuda.synchronize()
            grads.append({n: p.grad.float().clone() for n, p in model.named_parameters() if p.grad is not None})
        finally:
            G._WGRAD[0] = prev
    assert grads[0].keys() == grads[1].keys()
    for n in grads[0]:
        g0, g1 = grads[0][n], grads[1][n]
        err = ((g0 - g1).norm() / (g0.norm() + 1e-12)).item()
        assert err < 2e-2, (n, err)
    assert sum(n.endswith(".o_w") for n in grads[0]) == 12      # the weights the TN path takes


@pytest.mark.parametrize("M", [512, 8448])
@pytest.mark.parametrize("act", ["gelu", "gelu_tanh"])
def test_act_grad_epilogue_pair_matches_fp32(act, M):
    """linear_act_grad stores (act'(u), act(u)) with u = bf16(x W^T + b); mul_bwd_gemm multiplies
    the dgrad by the stored derivative.  Checked against fp32 math on the same bf16 u, and the
    derivative's single bf16 rounding is the only difference to the u-storing pair."""
    torch.manual_seed(6)
    F, H = 3072, 768
    x = torch.randn(M, H, device="cuda").bfloat16()
    w1 = (torch.randn(F, H, device="cuda") * 0.05).bfloat16()
    b1 = torch.randn(F, device="cuda").bfloat16()
    g, a = G.linear_act_grad(x, w1, b1, act)
    u, a_ref = G.linear_gelu(x, w1, b1, act)
    assert torch.equal(a, a_ref)                       # same activation values bit for bit
    d_ref = _gelu_grad_ref(u.float(), act)
    assert (g.float() - d_ref).abs().max().item() < 1e-2          # one bf16 rounding of values <= ~1.13
    assert rel(g, d_ref) < 4e-3
    dy = torch.randn(M, H, device="cuda").bfloat16()
    w2 = (torch.randn(H, F, device="cuda") * 0.05).bfloat16()
    w2t = w2.t().contiguous()
    db = torch.zeros(F, device="cuda", dtype=torch.float32)
    du = G.mul_bwd_gemm(dy, w2t, g, dbias=(db, False))
    db_u = torch.zeros(F, device="cuda", dtype=torch.float32)
    du_u = G.gelu_bwd_gemm(dy, w2t, u, dbias=(db_u, False), act=act)
    ref = (dy.float() @ w2.float()) * d_ref
    assert rel(du, ref) < 2e-2, rel(du, ref)
    assert rel(du, du_u) < 1e-2, rel(du, du_u)
    assert rel(db, ref.sum(0)) < 2e-2
    assert rel(db, db_u) < 1e-2


def test_store_grad_ffn_path_in_model_matches_u_path():
    """The model's FFN with the derivative stored in the forward (default) gives the same
    gradients as the pre-activation-storing pair (DTD_GEMM_FFN_STORE_GRAD=0)."""
    from distributed_training_and_deepspeed_amd.data import SyntheticLMDataset
    from distributed_training_and_deepspeed_amd.models import build_model
    grads, losses = [], []
    for on in (False, True):
        G._FFN_STORE_GRAD[0] = on
        try:
            model = build_model("bert-base-cased", dtype=torch.bfloat16, device="cuda", seed=12)
            ds = SyntheticLMDataset(model.cfg, 16, seq_len=512, seed=3)
            out = model(ds.input_ids.cuda(), labels=ds.labels.cuda())
            out.loss.backward()
            torch.cuda.synchronize()
            losses.append(out.loss.item())
            grads.append({n: p.grad.float().clone() for n, p in model.named_parameters() if p.grad is not None})
        finally:
            G._FFN_STORE_GRAD[0] = True
    assert losses[0] == losses[1]                      # identical forward values
    assert grads[0].keys() == grads[1].keys()
    for n in grads[0]:
        g0, g1 = grads[0][n], grads[1][n]
        err = ((g0 - g1).norm() / (g0.norm() + 1e-12)).item()
        assert err < 2e-2, (n, err)


@pytest.mark.parametrize("M,N,K", [(32768, 1024, 64), (16384, 3072, 768), (2048, 768, 3072), (512, 256, 128)])
def test_dynamic_tile_queue_bitwise_equals_static(M, N, K):
    """The persistent form's dynamic tile queue (default) only changes which workgroup computes a
    tile: outputs are bitwise equal to the static order, across repeated launches (the queue
    re-zeroes itself), with CUs held by a side-stream kernel, and on two streams at once (one
    queue per stream).  K = 64 covers the single-K-step (synchronous claim) path."""
    from distributed_training_and_deepspeed_amd.ops import _lib
    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    b = torch.randn(N, device="cuda").bfloat16()
    prev = G._SCHED[0]
    try:
        G.set_sched("static")
        g_ref, a_ref = G.linear_act_grad(x, w, b)
        c_ref = G.gemm_bt(x, w, b)
        G.set_sched("dynamic")
        for _ in range(3):
            g, a = G.linear_act_grad(x, w, b)
            assert torch.equal(g, g_ref) and torch.equal(a, a_ref)
            assert torch.equal(G.gemm_bt(x, w, b), c_ref)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            _lib.call("dtd_spin_occupy", 48, 200.0, side.cuda_stream)
        g, a = G.linear_act_grad(x, w, b)
        outs = []
        s2 = torch.cuda.Stream()
        s2.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s2):
            outs.append(G.linear_act_grad(x, w, b))
        outs.append(G.linear_act_grad(x, w, b))
        torch.cuda.synchronize()
        assert torch.equal(g, g_ref) and torch.equal(a, a_ref)
        for g2, a2 in outs:
            assert torch.equal(g2, g_ref) and torch.equal(a2, a_ref)
        for q in G._QUEUES.values():   # every queue is back at zero
            assert int(q.abs().sum()) == 0
    finally:
        G.set_sched(prev)
