"""Transformer layer with two interchangeable implementations.

* ``fused`` (GPU, bf16/fp32): one autograd node per layer with a hand-written backward that
  calls the gfx950 HIP kernels (flash attention, residual+dropout+LayerNorm, activation with
  fused bias-gradient partials) and hipBLASLt GEMMs, writing weight gradients straight into
  the flat gradient buckets (``ops/grad.py``).  Activations saved per layer: the layer input,
  qkv, attention context + LSE, the two LayerNorm pre-normalisation sums with their row
  statistics, and the FFN pre-activation -- dropout masks are regenerated, attention scores
  are never materialised.
* ``reference``: the same math with plain differentiable PyTorch ops (CPU tests, the fp32
  parity oracle, and the "torch-eager" baseline).

Covers every layer flavour the reference trains: post-LN BERT (HF BertLayer, SURVEY.md D15;
reference model/bert_mp.py:22-24), pre-LN OPT/GPT-2/BLOOM blocks (D17) including causal
masking and BLOOM ALiBi, and the instrumented OPT-style block of reference
model/transformer.py:18-106 (see ``models/transformer_block.py`` for the hookable variant).
"""
from __future__ import annotations

import os
import warnings

import math

import torch
import torch.nn.functional as F
from torch import nn

from ..ops import attention as A
from ..ops import functional as Fx
from ..ops import gemm as G
from ..ops.grad import emit_wgrad, grad_done, grad_dst, note_use
from ..ops.rng import RngState, attn_keep_mask
from .config import TransformerConfig


def init_linear_(w: torch.Tensor, b: torch.Tensor | None, std: float = 0.02) -> None:
    with torch.no_grad():
        w.normal_(0.0, std)
        if b is not None:
            b.zero_()


class Runtime:
    """Per-model execution settings shared by all submodules."""

    def __init__(self, impl: str = "auto", rng: RngState | None = None, exact_dropout: bool = True):
        self.impl = impl              # "auto" | "fused" | "reference"
        self.rng = rng or RngState(seed=0)
        self.exact_dropout = exact_dropout  # reference path uses the counter RNG masks
        self._next_sid = 1
        # Sparse MLM head with a STATIC row capacity (graph capture: no data-dependent shapes,
        # no host sync).  None -> exact-size gather (nonzero).  See MLMHead.loss.
        self.mlm_capacity: int | None = None
        self.mlm_overflow: torch.Tensor | None = None   # device flag: a batch exceeded the capacity
        # Keep the FFN activation act(u) from the forward for the backward (fc2 weight-gradient
        # input) instead of recomputing it in the activation-backward pass.  Costs one T x ffn
        # tensor per layer (4.8 GB for BERT-base at 128 x 512 tokens, ~2 % of 288 GB) and saves
        # its rewrite: the backward pass then moves 3 instead of 4 T x ffn tensors through HBM.
        # Memory-bound runs (max-params ZeRO-3) turn it off.
        self.keep_ffn_act = True
        self.pending_wt: list | None = None   # weights to batch-transpose at the start of the backward
        # memory-efficient post-LN backward for this model: None follows DTD_LN_MEMEFF; loading a
        # state dict whose LayerNorms are ill-conditioned for it sets False (ln_memeff_safe)
        self.ln_memeff: bool | None = None

    def new_sid(self) -> int:
        """Dropout stream id for one call site; deterministic per model structure so two
        builds of the same model (fused vs reference) draw identical masks."""
        s = self._next_sid
        self._next_sid += 1
        return s

    def use_fused(self, x: torch.Tensor) -> bool:
        if self.impl == "fused":
            return True
        if self.impl == "reference":
            return False
        return x.is_cuda


def stage_dgrad_transposes(layers, x: torch.Tensor) -> None:
    """End of a forward: drop the previous backward's W^T copies, and for a training forward on the
    fused path let the first layer backward transpose every layer's NT input-gradient operands in
    one batched launch (ops/gemm.py::prepare_transposes)."""
    G.clear_transposes()
    if not layers:
        return
    rt = layers[0].rt
    rt.pending_wt = None
    if layers[0].training and torch.is_grad_enabled() and x.is_cuda and rt.use_fused(x):
        # which W^T the backward will read: every projection's in the NT input-gradient form, else
        # only fc2's (the fused FFN-backward GEMM, which needs the kept activation)
        if G.dgrad_nt_enabled():
            names = ("qkv_w", "o_w", "fc1_w", "fc2_w")
        else:
            names = ("fc2_w",) if rt.keep_ffn_act else ()
        rt.pending_wt = [getattr(layer, n) for layer in layers for n in names] or None


def prefetch_masks(layers, input_ids: torch.Tensor) -> None:
    """Issue every layer's attention-dropout mask generation (fused bf16 path only)."""
    B, S = input_ids.shape[0], input_ids.shape[1]
    for layer in layers:
        if layer.rt.use_fused(input_ids) and layer.qkv_w.dtype in (torch.bfloat16, torch.float32):
            layer.prefetch_attention_masks(B, S, input_ids.device)


def ref_dropout(x, p, training, rt: Runtime, sid):
    if not training or p <= 0:
        return x
    if rt.exact_dropout:
        return Fx._ref_dropout(x, p, rt.rng, sid)
    return F.dropout(x, p, True)


def ref_attn_dropout(prob, p, training, rt: Runtime, sid):
    """Attention-probability dropout [B, H, S, S] with the HIP mask generator's stream
    (ops/rng.attn_keep_mask), so fused and reference models draw identical masks."""
    if not training or p <= 0:
        return prob
    if rt.exact_dropout:
        B, H, S, _ = prob.shape
        seed, step = (int(v) for v in rt.rng.state.tolist())
        keep = attn_keep_mask(B, H, S, p, seed, step, sid, device=prob.device)
        return (prob.float() * keep / (1.0 - p)).to(prob.dtype)
    return F.dropout(prob, p, True)


class TransformerLayer(nn.Module):
    def __init__(self, cfg: TransformerConfig, rt: Runtime):
        super().__init__()
        h, f = cfg.hidden_size, cfg.ffn_size
        self.cfg, self.rt = cfg, rt
        self._prefetched = None  # (sid, B, S, PendingMasks) from prefetch_attention_masks
        self.qkv_w = nn.Parameter(torch.empty(3 * h, h))
        self.qkv_b = nn.Parameter(torch.zeros(3 * h))
        self.o_w = nn.Parameter(torch.empty(h, h))
        self.o_b = nn.Parameter(torch.zeros(h))
        self.ln1_g = nn.Parameter(torch.ones(h))
        self.ln1_b = nn.Parameter(torch.zeros(h))
        self.fc1_w = nn.Parameter(torch.empty(f, h))
        self.fc1_b = nn.Parameter(torch.zeros(f))
        self.fc2_w = nn.Parameter(torch.empty(h, f))
        self.fc2_b = nn.Parameter(torch.zeros(h))
        self.ln2_g = nn.Parameter(torch.ones(h))
        self.ln2_b = nn.Parameter(torch.zeros(h))
        for w, b in ((self.qkv_w, self.qkv_b), (self.o_w, self.o_b), (self.fc1_w, self.fc1_b), (self.fc2_w, self.fc2_b)):
            init_linear_(w, b)
        self.sid_attn = rt.new_sid()
        self.sid_1 = rt.new_sid()
        self.sid_2 = rt.new_sid()
        if not cfg.pre_ln:
            self.register_load_state_dict_post_hook(_check_loaded_ln)
        # ALiBi slopes stay fp32 (not a buffer, so model.to(bfloat16) does not round them).
        self._alibi = A.alibi_slopes(cfg.num_heads) if cfg.alibi else None

    @property
    def alibi(self):
        if self._alibi is None:
            return None
        dev = self.qkv_w.device
        if self._alibi.device != dev:
            self._alibi = self._alibi.to(dev)
        return self._alibi

    def params(self):
        return (self.qkv_w, self.qkv_b, self.o_w, self.o_b, self.ln1_g, self.ln1_b,
                self.fc1_w, self.fc1_b, self.fc2_w, self.fc2_b, self.ln2_g, self.ln2_b)

    def prefetch_attention_masks(self, B: int, S: int, device) -> None:
        """Start generating this layer's attention-dropout keep bits now, on the side stream.
        The masks depend only on (seed, step, call site), not on activations, so a model issues
        every layer's generation at the start of its forward and the VALU-only hash work runs
        under the whole forward's GEMMs instead of in front of each attention.  The masks are
        kept for the backward anyway, so this costs no extra peak memory."""
        c = self.cfg
        if not (self.training and c.attn_dropout > 0 and torch.is_grad_enabled()):
            return
        sid = self.rt.rng.sid(self.sid_attn)
        pend = A.attn_masks_async(B, S, c.num_heads, c.head_dim, c.attn_dropout, self.rt.rng, sid, device)
        if pend is not None:
            self._prefetched = (sid, B, S, pend)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """x: [B, S, h] -> [B, S, h]"""
        # the fused backward reads the parameters at backward time (no saved weight views): ZeRO-3
        # may release and later re-gather them in between (parallel/zero.py)
        self._dtd_weightless_bwd = self.rt.use_fused(x)
        if self._dtd_weightless_bwd:
            note_use(self.params())
            return _FusedLayerFn.apply(x, self, *self.params())
        return self._reference(x)

    # ------------------------------------------------------------------ reference path
    def _reference(self, x: torch.Tensor) -> torch.Tensor:
        c, rt = self.cfg, self.rt
        B, S, h = x.shape
        H, D = c.num_heads, c.head_dim
        tr = self.training
        p_h = c.hidden_dropout if tr else 0.0
        p_a = c.attn_dropout if tr else 0.0

        def attn(inp):
            qkv = F.linear(inp, self.qkv_w, self.qkv_b).view(B, S, 3, H, D)
            q, k, v = (qkv[:, :, i].transpose(1, 2) for i in range(3))
            s = torch.matmul(q, k.transpose(-1, -2)) * (1.0 / math.sqrt(D))
            if self.alibi is not None:
                s = s + self.alibi.view(1, H, 1, 1).to(s.dtype) * torch.arange(S, device=s.device, dtype=s.dtype)
            if c.causal:
                s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device=s.device).triu(1), float("-inf"))
            prob = torch.softmax(s.float(), -1).to(s.dtype)
            prob = ref_attn_dropout(prob, p_a, tr, rt, rt.rng.sid(self.sid_attn))
            ctx = torch.matmul(prob, v).transpose(1, 2).reshape(B, S, h)
            return F.linear(ctx, self.o_w, self.o_b)

        def mlp(inp):
            u = F.linear(inp, self.fc1_w, self.fc1_b)
            return F.linear(Fx._ref_act(u, c.activation) if c.activation != "gelu" else F.gelu(u), self.fc2_w, self.fc2_b)

        ln = lambda t, g, b: F.layer_norm(t, (h,), g, b, c.ln_eps)
        if c.pre_ln:
            x = x + ref_dropout(attn(ln(x, self.ln1_g, self.ln1_b)), p_h, tr, rt, rt.rng.sid(self.sid_1))
            x = x + ref_dropout(mlp(ln(x, self.ln2_g, self.ln2_b)), p_h, tr, rt, rt.rng.sid(self.sid_2))
            return x
        x = ln(x + ref_dropout(attn(x), p_h, tr, rt, rt.rng.sid(self.sid_1)), self.ln1_g, self.ln1_b)
        x = ln(x + ref_dropout(mlp(x), p_h, tr, rt, rt.rng.sid(self.sid_2)), self.ln2_g, self.ln2_b)
        return x


# qkv bias gradient from the attention-backward epilogues (DTD_ATTN_QKV_BIAS=0: separate pass)
_FUSED_QKV_BIAS = [os.environ.get("DTD_ATTN_QKV_BIAS", "1") == "1"]
# Memory-efficient post-LN LayerNorms (DTD_LN_MEMEFF=0: store z): the forward keeps no
# z = residual + dropout(y) -- the backward recomputes x-hat = (out - beta) / gamma from the LN
# output, which the layer keeps anyway (fc1's input / the next layer's input).  One [T, h] write
# per LayerNorm forward and one [T, h] activation per LayerNorm less.
_LN_MEMEFF = [os.environ.get("DTD_LN_MEMEFF", "1") == "1"]
# (out - beta) / gamma multiplies the bf16 rounding of out by about |beta| / |gamma|, and a gamma of
# exactly 0 would leave its column's dgamma at 0 for good.  The recompute is used only while every
# post-LN column has |gamma| >= max(_LN_GAMMA_FLOOR, |beta| / _LN_BETA_RATIO).  At the ratio limit the
# recomputed dgamma is within ~1.3 % (relative L2) of the fp32 stored-z one, dx within ~0.1 %
# (tests/test_models_cpu.py::test_ln_memeff_error_at_the_guard_limit).
_LN_BETA_RATIO, _LN_GAMMA_FLOOR = 8.0, 1e-3


def ln_memeff_safe(layers) -> bool:
    """True if every post-LN LayerNorm of `layers` is well-conditioned for the memory-efficient
    backward (x-hat recomputed from the output).  One host sync; run at load time, not per step."""
    with torch.no_grad():
        for layer in layers:
            if layer.cfg.pre_ln:
                continue
            for g, b in ((layer.ln1_g, layer.ln1_b), (layer.ln2_g, layer.ln2_b)):
                if g.numel() == 0 or g.numel() != b.numel():   # released ZeRO-3 shard: no data here
                    continue
                lim = torch.clamp(b.detach().float().abs() / _LN_BETA_RATIO, min=_LN_GAMMA_FLOOR)
                if bool((g.detach().float().abs() < lim).any()):
                    return False
    return True


def _check_loaded_ln(layer, incompatible_keys) -> None:
    """load_state_dict post-hook of a post-LN layer: loaded LayerNorm parameters outside the
    memory-efficient backward's safe range switch the model to the stored-z backward (an explicit
    rt.ln_memeff is left alone).  The reference's HF LayerNorm always stores its input."""
    rt = layer.rt
    if rt.ln_memeff is None and _LN_MEMEFF[0] and not ln_memeff_safe([layer]):
        rt.ln_memeff = False
        warnings.warn("post-LN LayerNorm with |gamma| < max(1e-3, |beta|/8) loaded: using the "
                      "stored-z LayerNorm backward for this model", RuntimeWarning)


_dgrad = G.dgrad


def _acc(p):
    return grad_dst(p)


def _ffn_gemm_ok(c, x: torch.Tensor, w: torch.Tensor, *more) -> bool:
    """The hand-written GEMM with the GELU epilogues (ops/csrc/gemm.hip) takes the FFN products
    when the activation is GELU (erf or tanh), the tensors are bf16 on the GPU and the shape tiles
    by 256 into at least a tile per CU (``G.ffn_tiles_ok``)."""
    return (c.activation in G.FUSED_ACTS and x.is_cuda and x.dtype == torch.bfloat16 and G.enabled()
            and G.supported(x.shape[0], w.shape[0], x.shape[1], x, w, *more)
            and G.ffn_tiles_ok(x.shape[0], w.shape[0]))


def _proj_ln(inp, w, bias, res, gamma, beta, eps, p, rng, sid, store_z):
    """Post-LN sublayer output: LN(res + dropout(inp @ w.T + bias)) -> (z, out, mean, rstd).  One
    kernel (projection GEMM with the LayerNorm in its epilogue, ops/csrc/gemm_ln.hip) when enabled
    (DTD_GEMM_LN=1) and the shape tiles; else the Linear, then the fused residual/dropout/LN pass."""
    if G.ln_fused_enabled() and G.linear_ln_supported(inp, w, res, bias, gamma, beta):
        return G.linear_ln(inp, w, bias, res, gamma, beta, eps, p, rng, sid, store_z=store_z)
    return Fx.ln_fwd(G.linear_any(inp, w, bias), res, gamma, beta, eps, p, rng, sid, store_z=store_z)


class _FusedLayerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, layer: TransformerLayer, *params):
        c, rt = layer.cfg, layer.rt
        (qkv_w, qkv_b, o_w, o_b, g1, b1, w1, bf1, w2, bf2, g2, b2) = params
        B, S, h = x.shape
        H, D = c.num_heads, c.head_dim
        T = B * S
        tr = layer.training
        p_h = c.hidden_dropout if tr else 0.0
        p_a = c.attn_dropout if tr else 0.0
        rng = rt.rng
        sa, s1, s2 = rng.sid(layer.sid_attn), rng.sid(layer.sid_1), rng.sid(layer.sid_2)
        x2d = x.reshape(T, h)
        eps = c.ln_eps
        # attention-dropout keep bits: generated on a side stream -- prefetched by the model at
        # the start of its forward, else issued here to overlap at least the QKV GEMM
        pre, layer._prefetched = layer._prefetched, None
        if pre is not None and pre[:3] == (sa, B, S) and p_a > 0:
            pend = pre[3]
        else:
            pend = A.attn_masks_async(B, S, H, D, p_a, rng, sa, x.device) \
                if x.is_cuda and x.dtype in (torch.bfloat16, torch.float32) else None
        if c.pre_ln:
            _, a_in, m1, r1 = Fx.ln_fwd(None, x2d, g1, b1, eps, 0.0, rng, 0)
        else:
            a_in = x2d
        qkv = G.linear_any(a_in, qkv_w, qkv_b)
        actx, lse, amask = A.attn_fwd(qkv, B, S, H, D, c.causal, layer.alibi, p_a, rng, sa, masks=pend)
        ln_fo = (_LN_MEMEFF[0] if rt.ln_memeff is None else rt.ln_memeff) and not c.pre_ln
        if c.pre_ln:
            o = G.linear_any(actx, o_w, o_b)
            z1, f_in, m2, r2 = Fx.ln_fwd(o, x2d, g2, b2, eps, p_h, rng, s1)
        else:
            z1, f_in, m1, r1 = _proj_ln(actx, o_w, o_b, x2d, g1, b1, eps, p_h, rng, s1, store_z=not ln_fo)
        ffn_g = False   # u holds act'(pre-activation) instead of the pre-activation
        if G.ffn_fwd_enabled() and _ffn_gemm_ok(c, f_in, w1):
            if rt.keep_ffn_act and c.activation in G.GRAD_ACTS and G.ffn_store_grad_enabled():
                # fc1 + bias + GELU + GELU' in one kernel: the backward multiplies by the stored
                # derivative (its exp / rcp shared with the forward GELU here)
                u, a = G.linear_act_grad(f_in, w1, bf1, c.activation)
                ffn_g = True
            else:
                u, a = G.linear_gelu(f_in, w1, bf1, c.activation)     # fc1 + bias + GELU in one kernel
        else:
            u = G.linear_any(f_in, w1, bf1)
            a = Fx.act_fwd(u, c.activation)
        if c.pre_ln:
            y = G.linear_any(a, w2, bf2)
            out = Fx.dropout_add(y, z1, p_h, rng, s2)
            z2 = m3 = r3 = None
        else:
            z2, out, m3, r3 = _proj_ln(a, w2, bf2, f_in, g2, b2, eps, p_h, rng, s2, store_z=not ln_fo)
        a_keep = a if rt.keep_ffn_act else None
        if c.pre_ln:
            ctx.save_for_backward(x2d, a_in, qkv, actx, lse, z1, f_in, u, m1, r1, m2, r2, a_keep)
        else:
            # memory-efficient form: the LN2 output stands in for z2 (z1's stand-in, f_in, is saved)
            ctx.save_for_backward(x2d, qkv, actx, lse, z1, f_in, u, m1, r1, out if ln_fo else z2, m3, r3, a_keep)
        ctx.ln_fo = ln_fo
        ctx.layer = layer
        ctx.amask = amask  # attention dropout keep bits (kernel path) for the backward
        ctx.rng = rng  # the RngState of this forward's device (pipeline stages differ)
        ctx.meta = (B, S, h, H, D, p_h, p_a, sa, s1, s2)
        ctx.ffn_g = ffn_g
        return out.view(B, S, h)

    @staticmethod
    def backward(ctx, dout):
        layer = ctx.layer
        c, rng = layer.cfg, ctx.rng
        B, S, h, H, D, p_h, p_a, sa, s1, s2 = ctx.meta
        T = B * S
        (qkv_w, qkv_b, o_w, o_b, g1, b1, w1, bf1, w2, bf2, g2, b2) = layer.params()
        pend, layer.rt.pending_wt = layer.rt.pending_wt, None
        if pend:   # first layer backward of the step: every layer's W^T in one launch
            G.prepare_transposes(pend)
        dout = dout.reshape(T, h).contiguous()
        if c.pre_ln:
            x2d, a_in, qkv, actx, lse, z1, f_in, u, m1, r1, m2, r2, a = ctx.saved_tensors
            # out = z1 + dropout(y)
            dy = Fx.dropout(dout, p_h, rng, s2)
            Fx.bias_grad(dy, *_pair(bf2))
            grad_done(bf2)
        else:
            x2d, qkv, actx, lse, z1, f_in, u, m1, r1, z2, m3, r3, a = ctx.saved_tensors
            # out = LN2(f_in + dropout(y)); dz2 = d(out)/d(z2), flows to f_in (residual) and y
            lo2 = dict(xout=z2, beta=b2) if ctx.ln_fo else {}
            dz2, dy = Fx.ln_bwd(dout, None, None if ctx.ln_fo else z2, m3, r3, g2, p_h, rng, s2, want_dz=True,
                                want_dy=True, dgamma=_acc(g2), dbeta=_acc(b2), dbias=_acc(bf2), **lo2)
            for p in (g2, b2, bf2):
                grad_done(p)
        # dgrad first; without a kept forward activation, a = act(u) (fc2's wgrad input) is
        # recomputed inside the activation-backward pass (no separate act_fwd read/write)
        w2t = None
        if (a is not None and G.ffn_bwd_enabled() and c.activation in G.FUSED_ACTS and dy.is_cuda
                and dy.dtype == torch.bfloat16 and G.supported(dy.shape[0], w2.shape[1], dy.shape[1], dy, u)
                and G.ffn_tiles_ok(dy.shape[0], w2.shape[1])):
            w2t = G.transposed(w2)                     # [ffn, hidden]: K-contiguous B operand
        if ctx.ffn_g:
            # u holds act'(u): dU = dA * u
            if w2t is not None:
                du = G.mul_bwd_gemm(dy, w2t, u, dbias=_acc(bf1))
                del w2t
            else:
                du = ((dy @ w2).float() * u.float()).to(dy.dtype)
                Fx.bias_grad(du, *_pair(bf1))
        elif w2t is not None:
            # fc2 dgrad, GELU' and fc1's bias gradient in one kernel (no da round trip)
            du = G.gelu_bwd_gemm(dy, w2t, u, dbias=_acc(bf1), act=c.activation)
            del w2t
        else:
            da = _dgrad(dy, w2)
            if a is None:
                du, a = Fx.act_bwd(da, u, c.activation, dbias=_acc(bf1), want_act=True)
            else:
                du = Fx.act_bwd(da, u, c.activation, dbias=_acc(bf1))
        grad_done(bf1)
        emit_wgrad(w2, dy, a, async_ok=True)
        del a
        emit_wgrad(w1, du, f_in, async_ok=True)
        if c.pre_ln:
            dfin = _dgrad(du, w1)
            # z1 = x + dropout(o); f_in = LN2(z1); dz1 also receives dout (residual of out)
            dz1, do = Fx.ln_bwd(dfin, dout, z1, m2, r2, g2, p_h, rng, s1, want_dz=True, want_dy=True,
                                dgamma=_acc(g2), dbeta=_acc(b2), dbias=_acc(o_b))
            for p in (g2, b2, o_b):
                grad_done(p)
        else:
            # f_in = LN1(z1) feeds both the FFN and (as residual) z2: d f_in = du.W1 + dz2, with
            # the residual term summed inside the LN kernel (no addmm C-copy, no add pass)
            dfin = _dgrad(du, w1)
            lo1 = dict(xout=f_in, beta=b1) if ctx.ln_fo else {}
            dz1, do = Fx.ln_bwd(dfin, None, z1, m1, r1, g1, p_h, rng, s1, want_dz=True, want_dy=True,
                                dgamma=_acc(g1), dbeta=_acc(b1), dbias=_acc(o_b), dout2=dz2, **lo1)
            for p in (g1, b1, o_b):
                grad_done(p)
        emit_wgrad(o_w, do, actx, async_ok=True)
        dctx = _dgrad(do, o_w)
        # the qkv bias gradient comes out of the attention-backward epilogues (column partials)
        if _FUSED_QKV_BIAS[0]:
            dqkv = A.attn_bwd(dctx, qkv, actx, lse, B, S, H, D, c.causal, layer.alibi, p_a, rng, sa, ctx.amask,
                              dbias=_pair(qkv_b))
        else:
            dqkv = A.attn_bwd(dctx, qkv, actx, lse, B, S, H, D, c.causal, layer.alibi, p_a, rng, sa, ctx.amask)
            Fx.bias_grad(dqkv, *_pair(qkv_b))
        grad_done(qkv_b)
        if c.pre_ln:
            emit_wgrad(qkv_w, dqkv, a_in, async_ok=True)
            dain = _dgrad(dqkv, qkv_w)
            dx, _ = Fx.ln_bwd(dain, dz1, x2d, m1, r1, g1, 0.0, rng, 0, want_dz=True, want_dy=False,
                              dgamma=_acc(g1), dbeta=_acc(b1))
            for p in (g1, b1):
                grad_done(p)
        else:
            emit_wgrad(qkv_w, dqkv, x2d, async_ok=True)
            # in place: dz1 is this backward's own buffer (no C copy); NT form through the transposed weight
            dx = G.dgrad_add_(dz1, dqkv, qkv_w)
        return (dx.view(B, S, h), None) + (None,) * 12


def _pair(p):
    dst, acc = grad_dst(p)
    return dst, acc
