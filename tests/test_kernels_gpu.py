"""Numerics of every gfx950 HIP kernel against the fp32 PyTorch reference of the same op.

The CPU branch of ``ops/functional.py`` is the reference (fp32 math on the same inputs,
bit-identical dropout masks), so each test runs the op once on the GPU (kernel) and once on
CPU copies of the inputs.
"""
import pytest
import torch

from distributed_training_and_deepspeed_amd.ops import _lib
from distributed_training_and_deepspeed_amd.ops import functional as Fx
from distributed_training_and_deepspeed_amd.ops.rng import RngState, keep_mask

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rng_pair(seed=7, step=3):
    g = RngState(seed, device=DEV)
    c = RngState(seed, device="cpu")
    g.state[1] = step
    c.state[1] = step
    return g, c


def close(a, b, tol):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    scale = b.abs().max().item() + 1e-6
    assert err <= tol * scale, f"max err {err} vs scale {scale} (tol {tol})"


def test_library_loads_and_is_native():
    lib = _lib.lib()
    assert lib is not None and hasattr(lib, "dtd_ln_fwd")


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_dropout_mask_matches_reference(dtype):
    g, c = rng_pair()
    x = torch.ones(1000003, dtype=dtype, device=DEV)
    y = Fx.dropout(x, 0.1, g, 77)
    keep = keep_mask(x.numel(), 0.1, 7, 3, 77)
    assert torch.equal((y.cpu() != 0), keep)
    frac = keep.float().mean().item()
    assert abs(frac - 0.9) < 0.002


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_dropout_add_fused_residual(dtype):
    """res + dropout(x) in one pass: same keep bits as dropout(), sum taken in fp32."""
    g, c = rng_pair()
    n = 1000003   # odd: the scalar tail path
    x = torch.randn(n, dtype=dtype, device=DEV)
    res = torch.randn(n, dtype=dtype, device=DEV)
    y = Fx.dropout_add(x, res, 0.1, g, 78)
    keep = keep_mask(n, 0.1, 7, 3, 78).to(DEV)
    ref = (res.float() + x.float() * keep.float() / 0.9).to(dtype)
    close(y, ref, 1e-2 if dtype == torch.bfloat16 else 1e-6)
    z = Fx.dropout_add(x, res, 0.0, g, 78)      # eval: plain residual add
    close(z, (res.float() + x.float()).to(dtype), 1e-2 if dtype == torch.bfloat16 else 1e-6)


@pytest.mark.parametrize("h", [128, 768, 1024, 1280, 384, 2304])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_layernorm_fwd_bwd(h, dtype):
    torch.manual_seed(0)
    rows = 301  # odd: the two-rows-per-wave variants see a padded half-wave
    g, c = rng_pair()
    y = torch.randn(rows, h, dtype=dtype)
    r = torch.randn(rows, h, dtype=dtype)
    gamma = (1 + 0.1 * torch.randn(h)).to(dtype)
    beta = (0.1 * torch.randn(h)).to(dtype)
    dout = torch.randn(rows, h, dtype=dtype)
    dext = torch.randn(rows, h, dtype=dtype)
    dout2 = torch.randn(rows, h, dtype=dtype) if h != 384 else None   # second upstream term
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    outs = {}
    for dev, rng in ((DEV, g), ("cpu", c)):
        z, o, m, rs = Fx.ln_fwd(y.to(dev), r.to(dev), gamma.to(dev), beta.to(dev), 1e-5, 0.1, rng, 5)
        dg = torch.zeros(h, dtype=torch.float32, device=dev)
        db = torch.zeros(h, dtype=torch.float32, device=dev)
        dbias = torch.zeros(h, dtype=torch.float32, device=dev)
        dz, dy = Fx.ln_bwd(dout.to(dev), dext.to(dev), z, m, rs, gamma.to(dev), 0.1, rng, 5, want_dz=True,
                           want_dy=True, dgamma=dg, dbeta=db, dbias=dbias,
                           dout2=None if dout2 is None else dout2.to(dev))
        outs[dev] = (z, o, m, rs, dz, dy, dg, db, dbias)
    for a, b in zip(outs[DEV], outs["cpu"]):
        close(a, b, tol)


@pytest.mark.parametrize("h", [768, 1024, 2304])
@pytest.mark.parametrize("prefetch", ["0", "1"])
def test_layernorm_bwd_from_output(h, prefetch, monkeypatch):
    """Memory-efficient LN backward (x-hat from the stored output, no z) on the GPU vs the fp32
    CPU backward from z; both row-loop forms of the wave kernel (h = 2304: block kernel)."""
    monkeypatch.setenv("DTD_LN_BWD_PREFETCH", prefetch)
    torch.manual_seed(2)
    rows, dtype = 4099, torch.bfloat16
    g, c = rng_pair()
    y = torch.randn(rows, h, dtype=dtype)
    r = torch.randn(rows, h, dtype=dtype)
    gamma = (1 + 0.1 * torch.randn(h)).to(dtype)
    beta = (0.1 * torch.randn(h)).to(dtype)
    dout = torch.randn(rows, h, dtype=dtype)
    dout2 = torch.randn(rows, h, dtype=dtype)
    outs = {}
    for dev, rng in ((DEV, g), ("cpu", c)):
        fo = dev != "cpu"
        z, o, m, rs = Fx.ln_fwd(y.to(dev), r.to(dev), gamma.to(dev), beta.to(dev), 1e-5, 0.1, rng, 5,
                                store_z=not fo)
        assert (z is None) == fo
        dg, db, dbias = (torch.zeros(h, dtype=torch.float32, device=dev) for _ in range(3))
        kw = dict(xout=o, beta=beta.to(dev)) if fo else {}
        dz, dy = Fx.ln_bwd(dout.to(dev), None, z, m, rs, gamma.to(dev), 0.1, rng, 5, want_dz=True, want_dy=True,
                           dgamma=dg, dbeta=db, dbias=dbias, dout2=dout2.to(dev), **kw)
        outs[dev] = (o, dz, dy, dg, db, dbias)
    for a, b in zip(outs[DEV], outs["cpu"]):
        close(a, b, 3e-2)


@pytest.mark.parametrize("act", ["gelu", "gelu_tanh", "relu"])
def test_activation_fwd_bwd(act):
    torch.manual_seed(1)
    u = torch.randn(257, 3072, dtype=torch.bfloat16)
    dy = torch.randn_like(u)
    res = {}
    for dev in (DEV, "cpu"):
        a = Fx.act_fwd(u.to(dev), act)
        db = torch.zeros(3072, dtype=torch.float32, device=dev)
        du = Fx.act_bwd(dy.to(dev), u.to(dev), act, dbias=db)
        db2 = torch.zeros(3072, dtype=torch.float32, device=dev)
        du2, a2 = Fx.act_bwd(dy.to(dev), u.to(dev), act, dbias=db2, want_act=True)  # fused recompute
        res[dev] = (a, du, db, a2, du2, db2)
    for a, b in zip(res[DEV], res["cpu"]):
        close(a, b, 2e-2)
    assert torch.equal(res[DEV][0], res[DEV][3]) and torch.equal(res[DEV][1], res[DEV][4])


@pytest.mark.parametrize("act", ["gelu", "gelu_tanh"])
def test_activation_fast_math_accuracy_fp32(act):
    """The kernels' one-exponential erf (A&S 7.1.26) and exp-based tanh vs float64 torch over
    the range that matters (|x| <= 10, incl. the saturated tails)."""
    x = torch.linspace(-10, 10, 200_003, dtype=torch.float64)
    dy = torch.ones_like(x)
    xr = x.clone().requires_grad_(True)
    yr = torch.nn.functional.gelu(xr, approximate="none" if act == "gelu" else "tanh")
    (gr,) = torch.autograd.grad(yr.sum(), xr)
    y = Fx.act_fwd(x.float().to(DEV), act).double().cpu()
    g = Fx.act_bwd(dy.float().to(DEV), x.float().to(DEV), act).double().cpu()
    assert (y - yr.detach()).abs().max().item() < 2e-6
    assert (g - gr).abs().max().item() < 2e-6


@pytest.mark.parametrize("V,dtype,offset", [(28996, torch.bfloat16, 0), (50257, torch.bfloat16, 0), (1000, torch.bfloat16, 0),
                                            (250880, torch.bfloat16, 0), (7, torch.bfloat16, 0), (50257, torch.bfloat16, 3),
                                            (50257, torch.float32, 1), (13, torch.float32, 0)])
def test_softmax_xent(V, dtype, offset):
    """Odd vocabularies / unaligned bases: every row mixes a scalar head, 16-byte body and tail."""
    torch.manual_seed(2)
    rows = 64
    z = (3 * torch.randn(rows * V + offset))[offset:].view(rows, V).to(dtype)
    lab = torch.randint(0, V, (rows,))
    lab[::3] = -100
    gout = torch.tensor(0.7)
    res = {}
    for dev in (DEV, "cpu"):
        zd = z.to(dev)
        if offset and dev == DEV:   # an unaligned device view
            zd = torch.empty(rows * V + offset, dtype=dtype, device=dev)[offset:].view(rows, V).copy_(zd)
        loss, lse, st = Fx.xent_fwd(zd, lab.to(dev))
        d = Fx.xent_bwd(zd, lab.to(dev), lse, st, gout.to(dev))
        res[dev] = (loss, lse, st, d)
    ref = torch.nn.functional.cross_entropy(z.float(), lab, ignore_index=-100)
    close(res[DEV][0], ref, 1e-4)
    valid = lab != -100  # the kernel writes lse = 0 for ignored rows
    close(res[DEV][1][valid.to(DEV)], res["cpu"][1][valid], 1e-4)
    close(res[DEV][2], res["cpu"][2], 1e-4)
    close(res[DEV][3], res["cpu"][3], 2e-2)


@pytest.mark.parametrize("V,rows,offset", [(28996, 600, 0), (28996, 37, 0), (1000, 300, 0), (50257, 70, 0),
                                           (28996, 40, 2)])
def test_softmax_xent_bwd_fused_bias_grad(V, rows, offset):
    """xent_bwd(dbias=...) writes dlogits and the column sums of dlogits (the decoder-bias gradient)
    in one pass on the kernel path (V % 4 == 0, 8-byte aligned); other vocabularies / bases take
    the two-pass fallback.  dlogits are bit-identical to the unfused kernel; the bias gradient
    equals an fp32 column sum of the same bf16 dlogits (accumulate and overwrite)."""
    torch.manual_seed(5)
    z = (3 * torch.randn(rows * V + offset, device=DEV))[offset:].view(rows, V).bfloat16()
    lab = torch.randint(0, V, (rows,), device=DEV)
    lab[::4] = -100
    gout = torch.tensor(0.9, device=DEV)
    loss, lse, st = Fx.xent_fwd(z, lab)
    d_ref = Fx.xent_bwd(z, lab, lse, st, gout)
    ref = d_ref.float().sum(0)
    for acc in (False, True):
        db = torch.full((V,), 0.25, device=DEV)
        d = Fx.xent_bwd(z, lab, lse, st, gout, dbias=(db, acc))
        assert torch.equal(d, d_ref)
        close(db - (0.25 if acc else 0.0), ref, 1e-4)


def test_embedding_fwd_bwd():
    torch.manual_seed(3)
    V, h, B, S = 1000, 768, 4, 64
    word = torch.randn(V, h, dtype=torch.bfloat16)
    pos = torch.randn(S + 2, h, dtype=torch.bfloat16)
    typ = torch.randn(2, h, dtype=torch.bfloat16)
    ids = torch.randint(0, 50, (B, S))  # many repeats -> exercises segment sums
    dz = torch.randn(B * S, h, dtype=torch.bfloat16)
    res = {}
    for dev in (DEV, "cpu"):
        out = Fx.embed_fwd(ids.to(dev), word.to(dev), pos.to(dev), typ.to(dev), S, 2)
        gw = torch.full((V, h), 0.5, dtype=torch.float32, device=dev)
        gp = torch.zeros(S + 2, h, dtype=torch.float32, device=dev)
        Fx.embed_word_bwd(ids.to(dev), dz.to(dev), gw, True, padding_idx=0)
        Fx.embed_pos_bwd(dz.to(dev), gp, B, S, 2, False)
        res[dev] = (out, gw, gp)
    for a, b in zip(res[DEV], res["cpu"]):
        close(a, b, 2e-2)


@pytest.mark.parametrize("acc,gdt", [(True, torch.float32), (False, torch.bfloat16)])
def test_embedding_bwd_long_segments(acc, gdt):
    """Skewed ids (one id repeated 1000x, a pad run): segments far longer than the 16-row chunks
    of the sorted segment sum, bf16 and fp32 tables, overwrite and accumulate."""
    torch.manual_seed(5)
    V, h, n = 3000, 768, 4096
    ids = torch.randint(0, V, (n,))
    ids[:1000] = 7
    ids[1000:1300] = 0
    ids = ids[torch.randperm(n)]
    dz = torch.randn(n, h, dtype=torch.bfloat16)
    res = {}
    for dev in (DEV, "cpu"):
        g = torch.full((V, h), 0.25, dtype=gdt, device=dev)
        Fx.embed_word_bwd(ids.to(dev), dz.to(dev), g, acc, padding_idx=0)
        res[dev] = g.float().cpu()
    close(res[DEV], res["cpu"], 2e-2)


@pytest.mark.parametrize("hf", [False, True])
def test_fused_adam_matches_reference(hf):
    from distributed_training_and_deepspeed_amd.optim.fused_adam import (MODE_ADAMW, MODE_BIAS_CORR, MODE_HF_EPS,
                                                                          adam_reference_)
    torch.manual_seed(4)
    n = 100003
    p = torch.randn(n)
    m = torch.randn(n).abs() * 0.1
    v = torch.randn(n).abs() * 0.01
    gr = torch.randn(n).to(torch.bfloat16)
    mode = MODE_ADAMW | MODE_BIAS_CORR | (MODE_HF_EPS if hf else 0)
    hp = torch.tensor([1e-3, 0.9, 0.999, 1e-6, 0.01, 3.0, 0.5, 0.0], device=DEV)
    pg, mg, vg = p.to(DEV), m.to(DEV), v.to(DEV)
    lowp = torch.empty(n, dtype=torch.bfloat16, device=DEV)
    _lib.call("dtd_adam_step", pg.data_ptr(), mg.data_ptr(), vg.data_ptr(), gr.to(DEV).data_ptr(), 1, lowp.data_ptr(),
              n, hp.data_ptr(), mode, _lib.stream())
    adam_reference_(p, m, v, gr, 1e-3, 0.9, 0.999, 1e-6, 0.01, 3, mode, grad_scale=0.5)
    close(pg, p, 1e-5)
    close(mg, m, 1e-5)
    close(vg, v, 1e-5)
    close(lowp, p, 1e-2)


def test_sqnorm_and_scale_cast():
    x = torch.randn(123457, device=DEV).to(torch.bfloat16)
    close(Fx.sq_norm(x), x.float().pow(2).sum(), 1e-4)
    y = torch.empty(x.numel(), dtype=torch.float32, device=DEV)
    Fx.scale_cast_(x, y, 0.25)
    close(y, x.float() * 0.25, 1e-6)


@pytest.mark.parametrize("pdt,ddt,acc", [(torch.float32, torch.bfloat16, False), (torch.float32, torch.bfloat16, True),
                                         (torch.bfloat16, torch.float32, True), (torch.float32, torch.float32, False)])
def test_splitk_reduce(pdt, ddt, acc):
    from distributed_training_and_deepspeed_amd.ops.grad import splitk_reduce
    torch.manual_seed(0)
    part = torch.randn(4, 96, 40).to(pdt)
    dst = torch.randn(96, 40).to(ddt)
    ref = (dst.float() if acc else 0) + part.float().sum(0)
    g = dst.to(DEV)
    splitk_reduce(part.to(DEV), g, acc)
    close(g, ref, 1e-2 if ddt == torch.bfloat16 else 1e-5)


def test_split_k_wgrad_matches_fp32():
    from distributed_training_and_deepspeed_amd.ops.grad import emit_wgrad, wgrad_splits
    torch.manual_seed(0)
    T, o, i = 16384, 768, 3072
    assert wgrad_splits(T, o, i) > 1
    w = torch.nn.Parameter(torch.zeros(o, i, dtype=torch.bfloat16, device=DEV))
    dy = torch.randn(T, o, device=DEV).to(torch.bfloat16)
    x = torch.randn(T, i, device=DEV).to(torch.bfloat16)
    emit_wgrad(w, dy, x)
    ref = dy.float().t() @ x.float()
    close(w.grad, ref, 1e-2)
    emit_wgrad(w, dy, x)               # second contribution accumulates
    close(w.grad, 2 * ref, 1e-2)


@pytest.mark.parametrize("n", [512, 100, 4096, 8200])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_row_softmax_fwd_bwd(n, dtype):
    torch.manual_seed(3)
    x = (3 * torch.randn(37, n)).to(dtype)
    dy = torch.randn(37, n).to(dtype)
    y = Fx.softmax_fwd(x.to(DEV))
    ref = torch.softmax(x.float(), -1)
    close(y, ref, 2e-2 if dtype == torch.bfloat16 else 1e-5)
    dx = Fx.softmax_bwd(y, dy.to(DEV))
    rdx = ref * (dy.float() - (ref * dy.float()).sum(-1, keepdim=True))
    close(dx, rdx, 3e-2 if dtype == torch.bfloat16 else 1e-4)


@pytest.mark.parametrize("h,rows,seq,offset,p", [(768, 131 * 3, 131, 0, 0.1), (768, 512 * 4, 512, 0, 0.0),
                                                 (1024, 67 * 3, 67, 2, 0.1)])
def test_embed_ln_dropout_fused_bit_identical(h, rows, seq, offset, p):
    """embed_ln_fwd (one kernel) == embed_fwd -> ln_fwd -> dropout: z (the LN input kept for the
    backward) and mean bit for bit, rstd to the last fp32 bits (the two kernels' rsqrt codegen may
    differ by an ulp), the dropped-out output to one bf16 rounding at most, with identical keep
    bits; rows not a multiple of the 8 rows per block."""
    from distributed_training_and_deepspeed_amd.ops.rng import RngState
    torch.manual_seed(7)
    V = 1000
    word = (torch.randn(V, h, device=DEV) * 0.5).bfloat16()
    pos = (torch.randn(seq + offset, h, device=DEV) * 0.1).bfloat16()
    typ = (torch.randn(2, h, device=DEV) * 0.1).bfloat16()
    g = (1 + 0.1 * torch.randn(h, device=DEV)).bfloat16()
    b = (0.1 * torch.randn(h, device=DEV)).bfloat16()
    ids = torch.randint(0, V, (rows // seq, seq), device=DEV)
    rng = RngState(1234, device=DEV)
    out, z, m, r = Fx.embed_ln_fwd(ids, word, pos, typ, seq, offset, g, b, 1e-12, p, rng, 5)
    z_ref = Fx.embed_fwd(ids, word, pos, typ, seq, offset)
    _, x_ref, m_ref, r_ref = Fx.ln_fwd(None, z_ref, g, b, 1e-12, 0.0, rng, 0)
    out_ref = Fx.dropout(x_ref, p, rng, 5)
    assert torch.equal(z, z_ref)
    assert torch.equal(m, m_ref)
    assert ((r - r_ref).abs() <= 4e-7 * r_ref.abs()).all()
    assert torch.equal(out == 0, out_ref == 0)                       # the same dropped elements
    assert ((out.float() - out_ref.float()).abs() <= 8e-3 * out_ref.float().abs() + 1e-6).all()
