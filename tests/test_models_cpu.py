"""CPU tests: model presets, fused-vs-reference backward parity, data pipeline, optimizer math."""
import math

import pytest
import torch

from distributed_training_and_deepspeed_amd.data import DistributedSampler, SyntheticLMDataset
from distributed_training_and_deepspeed_amd.models import build_model, count_parameters
from distributed_training_and_deepspeed_amd.models import config as C
from distributed_training_and_deepspeed_amd.ops.rng import keep_mask

EXPECTED = {  # SURVEY.md section 6 [derived] parameter counts
    "bert-base-cased": 108_340_804,
    "bert-large-cased": 333_610_308,
    "bigscience/bloom-560m": 559_214_592,
    "facebook/opt-125m": 125_239_296,
    "gpt2-medium": 354_823_168,
}


@pytest.mark.parametrize("name", sorted(EXPECTED))
def test_preset_parameter_counts(name):
    with torch.device("meta"):
        m = build_model(name, device="meta")
    assert count_parameters(m) == EXPECTED[name]


PARITY = [
    ("tiny", {}),
    ("causal-tiny", {}),
    ("causal-tiny", {"alibi": True, "embedding_ln": True, "family": "bloom"}),
    ("causal-tiny", {"family": "opt", "position_offset": 2, "activation": "relu", "pad_token_id": 1}),
]


@pytest.mark.parametrize("name,extra", PARITY)
def test_fused_backward_matches_autograd(name, extra):
    """The hand-written per-layer backward (with regenerated dropout masks and direct gradient
    emission) equals autograd through the reference ops, fp32 on CPU."""
    cfg = C.get_config(name).with_(**extra)
    C.PRESETS["_p"] = cfg
    ref = build_model("_p", impl="reference", seed=3)
    fus = build_model("_p", impl="fused", seed=3)
    fus.load_state_dict(ref.state_dict())
    ds = SyntheticLMDataset(cfg, 2, seq_len=24, seed=5)
    l1 = ref(ds.input_ids, labels=ds.labels).loss
    l1.backward()
    l2 = fus(ds.input_ids, labels=ds.labels).loss
    l2.backward()
    assert abs(l1.item() - l2.item()) < 1e-5
    for (n, p1), (_, p2) in zip(ref.named_parameters(), fus.named_parameters()):
        err = (p1.grad - p2.grad).abs().max().item()
        assert err <= 1e-4 * (p1.grad.abs().max().item() + 1e-8), (n, err)


@pytest.mark.parametrize("memeff", [True, False])
def test_post_ln_backward_with_and_without_stored_z(memeff, monkeypatch):
    """Post-LN (BERT) layers: the memory-efficient LayerNorm backward (x-hat from the LN output,
    no z kept by the forward; the default) and the stored-z backward both equal autograd."""
    from distributed_training_and_deepspeed_amd.models import transformer as TR
    monkeypatch.setattr(TR, "_LN_MEMEFF", [memeff])
    test_fused_backward_matches_autograd("tiny", {})


def test_ln_bwd_from_output_matches_stored_z_form():
    """ops.functional.ln_bwd: x-hat recomputed from the LN output (memory-efficient form) gives the
    stored-z gradients in fp32 on CPU; z=None without the output is refused."""
    from distributed_training_and_deepspeed_amd.ops import functional as Fx
    from distributed_training_and_deepspeed_amd.ops.rng import RngState
    torch.manual_seed(0)
    rows, h = 37, 64
    y, r, dout, dout2 = (torch.randn(rows, h) for _ in range(4))
    gamma, beta = 1 + 0.1 * torch.randn(h), 0.1 * torch.randn(h)
    rng = RngState(3)
    res = {}
    for fo in (False, True):
        z, o, m, rs = Fx.ln_fwd(y, r, gamma, beta, 1e-5, 0.1, rng, 7, store_z=not fo)
        dg, db, dbias = (torch.zeros(h) for _ in range(3))
        kw = dict(xout=o, beta=beta) if fo else {}
        dz, dy = Fx.ln_bwd(dout, None, z, m, rs, gamma, 0.1, rng, 7, want_dz=True, want_dy=True, dgamma=dg,
                           dbeta=db, dbias=dbias, dout2=dout2, **kw)
        res[fo] = (dz, dy, dg, db, dbias)
    for a, b in zip(res[False], res[True]):
        assert torch.allclose(a, b, atol=1e-4, rtol=1e-4)
    with pytest.raises(ValueError):
        Fx.ln_bwd(dout, None, None, m, rs, gamma, 0.1, rng, 7)


@pytest.mark.parametrize("ratio,bound", [(8.0, (3e-3, 2e-2)), (64.0, None)])
def test_ln_memeff_error_at_the_guard_limit(ratio, bound):
    """x-hat = (out - beta) / gamma from a bf16 output: the error grows with |beta| / |gamma|.  At
    the guard's limit (ratio 8, models/transformer.py _LN_BETA_RATIO) dx and dgamma stay within
    0.3 % / 2 % of the fp32 stored-z backward; at ratio 64 -- what the guard refuses -- dgamma is
    off by ~10 %."""
    from distributed_training_and_deepspeed_amd.models import transformer as TR
    from distributed_training_and_deepspeed_amd.ops import functional as Fx
    from distributed_training_and_deepspeed_amd.ops.rng import RngState
    torch.manual_seed(0)
    rows, h = 512, 256
    y, r, dout = (torch.randn(rows, h) for _ in range(3))
    beta = torch.empty(h).uniform_(-1, 1)
    gamma = torch.clamp(beta.abs() / ratio, min=1e-3) * torch.sign(torch.randn(h))
    rng = RngState(3)
    res = {}
    for fo in (False, True):
        z, o, m, rs = Fx.ln_fwd(y, r, gamma, beta, 1e-5, 0.0, rng, 7, store_z=not fo)
        dg, db = torch.zeros(h), torch.zeros(h)
        kw = dict(xout=o.bfloat16().float(), beta=beta) if fo else {}
        dz, _ = Fx.ln_bwd(dout, None, z, m, rs, gamma, 0.0, rng, 7, want_dz=True, want_dy=False, dgamma=dg,
                          dbeta=db, **kw)
        res[fo] = (dz, dg)
    err = [((a - b).norm() / b.norm()).item() for a, b in zip(res[True], res[False])]
    if bound is None:
        assert err[1] > 0.05
        assert ratio > TR._LN_BETA_RATIO
    else:
        assert ratio <= TR._LN_BETA_RATIO and err[0] < bound[0] and err[1] < bound[1], err


def test_loading_ill_conditioned_layernorm_selects_stored_z_backward():
    """A state dict whose post-LN gamma is (near) zero where beta is not switches that model to the
    stored-z LayerNorm backward at load time; a well-conditioned one (or an explicit choice) does
    not."""
    from distributed_training_and_deepspeed_amd.models import build_model
    from distributed_training_and_deepspeed_amd.models import transformer as TR
    m = build_model("tiny")
    assert m.rt.ln_memeff is None and TR.ln_memeff_safe(m.layers)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m.load_state_dict(sd)
    assert m.rt.ln_memeff is None
    key = [k for k in sd if k.endswith("ln2_g")][1]
    sd[key][5] = 0.0
    sd[key.replace("ln2_g", "ln2_b")][5] = 0.5
    m2 = build_model("tiny")
    with pytest.warns(RuntimeWarning, match="stored-z"):
        m2.load_state_dict(sd)
    assert m2.rt.ln_memeff is False and not TR.ln_memeff_safe(m2.layers)
    m3 = build_model("tiny")
    m3.rt.ln_memeff = True
    m3.load_state_dict(sd)
    assert m3.rt.ln_memeff is True


def test_mlm_masking_law():
    cfg = C.BERT_BASE
    ds = SyntheticLMDataset(cfg, 64, seq_len=512, seed=0)
    orig = SyntheticLMDataset.__new__(SyntheticLMDataset)
    lab = ds.labels
    masked = lab != -100
    frac = masked.float().mean().item()
    assert 0.13 < frac < 0.17  # p=0.15 over non-special tokens ([CLS]/[SEP] never masked)
    assert not masked[:, 0].any() and not masked[:, -1].any()
    inp = ds.input_ids[masked]
    tgt = lab[masked]
    mask_frac = (inp == cfg.mask_token_id).float().mean().item()
    same_frac = (inp == tgt).float().mean().item()
    assert 0.77 < mask_frac < 0.83
    assert 0.08 < same_frac < 0.12


def test_causal_labels_are_inputs():
    ds = SyntheticLMDataset(C.OPT_125M, 4, seq_len=64, seed=0)
    assert torch.equal(ds.input_ids, ds.labels)


def test_dropout_mask_rate_and_determinism():
    m1 = keep_mask(200_000, 0.1, 5, 2, 17)
    m2 = keep_mask(200_000, 0.1, 5, 2, 17)
    m3 = keep_mask(200_000, 0.1, 5, 3, 17)
    assert torch.equal(m1, m2)
    assert not torch.equal(m1, m3)
    assert abs(m1.float().mean().item() - 0.9) < 0.005
    # neighbouring elements are not correlated
    a, b = m1[0::2].float(), m1[1::2].float()
    assert abs(((a - a.mean()) * (b - b.mean())).mean().item()) < 2e-3


@pytest.mark.parametrize("n,world", [(10, 3), (16, 4), (7, 2), (100, 8)])
def test_sampler_matches_torch(n, world):
    ds = list(range(n))
    for r in range(world):
        ours = list(DistributedSampler(ds, num_replicas=world, rank=r, seed=0))
        ref = list(torch.utils.data.distributed.DistributedSampler(ds, num_replicas=world, rank=r, seed=0))
        assert ours == ref


def test_fused_adam_matches_torch_adamw():
    from distributed_training_and_deepspeed_amd.optim import torch_adamw
    torch.manual_seed(0)
    w = torch.nn.Linear(16, 8)
    w2 = torch.nn.Linear(16, 8)
    w2.load_state_dict(w.state_dict())
    ours = torch_adamw(w.parameters(), lr=1e-2)
    ref = torch.optim.AdamW(w2.parameters(), lr=1e-2)
    for _ in range(5):
        x = torch.randn(4, 16)
        for mod, opt in ((w, ours), (w2, ref)):
            opt.zero_grad()
            mod(x).pow(2).sum().backward()
            opt.step()
    for a, b in zip(w.parameters(), w2.parameters()):
        assert torch.allclose(a, b, atol=1e-6)


def test_fused_adam_hf_eps_semantics():
    """transformers.AdamW: p -= lr*sqrt(1-b2^t)/(1-b1^t) * m / (sqrt(v) + eps)."""
    from distributed_training_and_deepspeed_amd.optim import hf_adamw
    p = torch.nn.Parameter(torch.tensor([1.0, -2.0, 3.0]))
    opt = hf_adamw([p], lr=0.1)
    g = torch.tensor([0.5, -0.25, 1.0])
    p.grad = g.clone()
    opt.step()
    m = 0.1 * g
    v = 0.001 * g * g
    exp = torch.tensor([1.0, -2.0, 3.0]) - 0.1 * math.sqrt(1 - 0.999) / (1 - 0.9) * m / (v.sqrt() + 1e-6)
    assert torch.allclose(p.detach(), exp, atol=1e-6)


def test_comm_busbw_factors():
    from distributed_training_and_deepspeed_amd.comm.logger import _busbw_factor
    assert _busbw_factor("all_reduce", 8) == pytest.approx(2 * 7 / 8)
    assert _busbw_factor("reduce_scatter_tensor", 8) == pytest.approx(7 / 8)
    assert _busbw_factor("all_gather_into_tensor", 4) == pytest.approx(3 / 4)


def test_replicated_checkpoint_resume_is_exact(tmp_path):
    from distributed_training_and_deepspeed_amd.data import SyntheticLMDataset
    from distributed_training_and_deepspeed_amd.models import build_model
    from distributed_training_and_deepspeed_amd.optim import hf_adamw
    from distributed_training_and_deepspeed_amd.utils.checkpoint import load_checkpoint, save_checkpoint
    ds = SyntheticLMDataset(build_model("tiny").cfg, 8, seq_len=32, seed=4)

    def step(m, o, i):
        m(ds.input_ids[2 * i:2 * i + 2], labels=ds.labels[2 * i:2 * i + 2]).loss.backward()
        o.step()
        o.zero_grad()
        m.rt.rng.advance()

    a = build_model("tiny", seed=3)
    oa = hf_adamw(a.parameters(), lr=1e-3)
    for i in range(2):
        step(a, oa, i)
    save_checkpoint(str(tmp_path / "ck.pt"), a, oa, step=2, extra={"note": "x"})
    for i in range(2, 4):
        step(a, oa, i)
    # the resumed process is started like the original (same per-rank dropout seed); the file
    # restores the parameters, the optimizer and the dropout STEP but never overrides the seed
    b = build_model("tiny", seed=11)
    b.rt.rng.reseed(a.rt.rng.seed)
    ob = hf_adamw(b.parameters(), lr=1e-3)
    c = build_model("tiny", seed=11)                 # another rank: its own seed survives the load
    meta = load_checkpoint(str(tmp_path / "ck.pt"), c, hf_adamw(c.parameters(), lr=1e-3))
    assert int(c.rt.rng.state[0]) == 11 and int(c.rt.rng.state[1]) == 2
    meta = load_checkpoint(str(tmp_path / "ck.pt"), b, ob)
    assert meta == {"step": 2, "extra": {"note": "x"}}
    for i in range(2, 4):
        step(b, ob, i)
    for (n, p), q in zip(a.named_parameters(), b.parameters()):
        assert torch.equal(p, q), n


def test_static_capacity_mlm_head_matches_exact_gather():
    """The graph-capturable MLM head (static labelled-row capacity) gives the same loss and
    gradients as the exact-size gather, and flags an over-full batch."""
    from distributed_training_and_deepspeed_amd.data import SyntheticLMDataset
    from distributed_training_and_deepspeed_amd.models import build_model
    from distributed_training_and_deepspeed_amd.utils.graphs import mlm_capacity
    ds = SyntheticLMDataset(build_model("tiny").cfg, 4, seq_len=64, seed=2)
    res = []
    for cap in (None, mlm_capacity(4 * 64)):
        m = build_model("tiny", impl="fused", seed=3)
        m.rt.mlm_capacity = cap
        m.rt.mlm_overflow = torch.zeros((), dtype=torch.bool)
        loss = m(ds.input_ids, labels=ds.labels).loss
        loss.backward()
        res.append((loss.detach(), {n: p.grad.clone() for n, p in m.named_parameters()}))
        assert not bool(m.rt.mlm_overflow)
    assert torch.allclose(res[0][0], res[1][0], atol=1e-6)
    for n in res[0][1]:
        assert torch.allclose(res[0][1][n], res[1][1][n], atol=1e-6), n
    m = build_model("tiny", impl="fused", seed=3)
    m.rt.mlm_capacity = 4
    m.rt.mlm_overflow = torch.zeros((), dtype=torch.bool)
    m(ds.input_ids, labels=ds.labels)
    assert bool(m.rt.mlm_overflow)


def test_attention_keep_word_layout_roundtrip():
    """ops.attention.decode_masks inverts the generator's permuted [B*H][W][32 W] keep-word layout
    (lm_pos: the words of positions c and c + 4 adjacent, as the forward's 64-bit lane masks need),
    for a sequence length that is not a multiple of 32."""
    import torch
    from distributed_training_and_deepspeed_amd.ops import attention as A
    from distributed_training_and_deepspeed_amd.ops.rng import attn_keep_mask
    B, H, S = 1, 2, 100
    W = (S + 31) // 32
    keep = attn_keep_mask(B, H, S, 0.1, 5, 0, 3).view(B * H, S, S).to(torch.int64)   # [bh][q][key]
    pos = A._lm_pos(S)
    assert sorted(set(pos.tolist())) == sorted(pos.tolist()) and int(pos.max()) < 32 * W
    masks = torch.zeros((2, A.mask_words(B, H, S)), dtype=torch.int64)
    ma, mb = masks[0].view(B * H, W, 32 * W), masks[1].view(B * H, W, 32 * W)
    for w in range(W):
        bits = keep[:, :, 32 * w:32 * w + 32]            # keys of word w, per query
        shifts = torch.arange(bits.shape[2], dtype=torch.int64)
        ma[:, w, pos] = (bits << shifts).sum(-1)         # A: word (w, q), bit j = key 32w + j
        qb = keep[:, 32 * w:32 * w + 32, :].transpose(1, 2)   # queries of word w, per key
        shifts = torch.arange(qb.shape[2], dtype=torch.int64)
        mb[:, w, pos] = (qb << shifts).sum(-1)           # B: word (w, key), bit j = query 32w + j
    enc = (masks & 0xFFFFFFFF).to(torch.int64)
    enc = torch.where(enc >= 2**31, enc - 2**32, enc).to(torch.int32)
    a, b = A.decode_masks(enc, B, H, S)
    assert torch.equal(a, keep) and torch.equal(b, keep)


@pytest.mark.parametrize("name", ["tiny", "causal-tiny"])
def test_prewarm_model_kernels_leaves_the_global_rng_alone(name):
    """utils/prewarm.py: the throwaway 1-layer forward/backward that the entry scripts run before
    creating the RCCL group must not shift the global torch RNG (the real model's init draws)."""
    from distributed_training_and_deepspeed_amd.utils.prewarm import prewarm_model_kernels
    torch.manual_seed(11)
    state = torch.random.get_rng_state()
    prewarm_model_kernels(name, "cpu", dtype=torch.float32, seq_len=64)
    assert torch.equal(state, torch.random.get_rng_state())
