"""Embedding, LayerNorm and LM-head modules (fused + reference implementations).

* ``Embeddings``: word (+ learned positions with OPT's offset) (+ BERT token types) (+ LN)
  (+ dropout).  HF BertEmbeddings / GPT-2 wte+wpe / OPT embed_tokens+positions / BLOOM
  word_embeddings(+layernorm) -- SURVEY.md D15-D17, K7.
* ``LayerNorm``: final LN of pre-LN models, fused kernel forward/backward.
* ``MLMHead``: BERT BertOnlyMLMHead (dense -> GELU -> LN -> decoder + bias; decoder weight
  tied to the word embeddings unless ``tied=False`` as in reference model/bert_mp.py:24) with
  the softmax cross-entropy fused in.  With ``sparse=True`` the head runs only on positions
  that carry an MLM label (~15% of tokens): the loss and every gradient are mathematically
  identical to the dense head (unlabelled rows contribute exactly zero), it just skips the
  logits that CrossEntropyLoss(ignore_index=-100) would discard.
* ``LMHead``: tied causal-LM head with the shifted-label cross entropy of HF *ForCausalLM,
  computed only on the S-1 positions that have a next-token label.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F
from torch import nn

from ..ops import functional as Fx
from ..ops import gemm as G
from ..ops.grad import emit_wgrad, grad_done, grad_dst, note_use

from .config import TransformerConfig
from .transformer import Runtime, init_linear_, ref_dropout


# ----------------------------------------------------------------------------- LayerNorm
class _LNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g, b, eps):
        h = x.shape[-1]
        x2 = x.reshape(-1, h)
        _, out, m, r = Fx.ln_fwd(None, x2, g, b, eps, 0.0, _DUMMY_RNG(x), 0)
        ctx.save_for_backward(x2, m, r)
        ctx.g, ctx.b = g, b
        return out.view_as(x)

    @staticmethod
    def backward(ctx, dout):
        x2, m, r = ctx.saved_tensors
        g, b = ctx.g, ctx.b
        h = x2.shape[-1]
        dx, _ = Fx.ln_bwd(dout.reshape(-1, h), None, x2, m, r, g, 0.0, _DUMMY_RNG(x2), 0, want_dz=True,
                          dgamma=grad_dst(g), dbeta=grad_dst(b))
        grad_done(g)
        grad_done(b)
        return dx.view_as(dout), None, None, None


_RNGS: dict = {}


def _DUMMY_RNG(x):
    from ..ops.rng import RngState
    k = str(x.device)
    if k not in _RNGS:
        _RNGS[k] = RngState(0, device=x.device)
    return _RNGS[k]


class LayerNorm(nn.Module):
    def __init__(self, h: int, eps: float, rt: Runtime):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(h))
        self.bias = nn.Parameter(torch.zeros(h))
        self.eps, self.rt = eps, rt

    def forward(self, x):
        self._dtd_weightless_bwd = self.rt.use_fused(x)   # see TransformerLayer.forward
        if self._dtd_weightless_bwd:
            note_use((self.weight, self.bias))
            return _LNFn.apply(x, self.weight, self.bias, self.eps)
        return F.layer_norm(x, (x.shape[-1],), self.weight, self.bias, self.eps)


# ----------------------------------------------------------------------------- Embeddings
# DTD_FUSED_EMBED_LN=0 keeps the three-pass embedding forward (A/B runs)
_FUSED_EMBED_LN = [os.environ.get("DTD_FUSED_EMBED_LN", "1") == "1"]


class _EmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, mod, *params):
        c, rt = mod.cfg, mod.rt
        B, S = ids.shape
        h = c.hidden_size
        word = mod.word
        pos = mod.pos
        typ = mod.tok_type
        p = c.hidden_dropout if mod.training else 0.0
        sid = rt.rng.sid(mod.sid)
        fused = None
        if mod.ln_g is not None and _FUSED_EMBED_LN[0]:
            # gather-sum + LN + dropout in one pass (bit-identical to the three passes below)
            fused = Fx.embed_ln_fwd(ids, word, pos, typ, S, c.position_offset, mod.ln_g, mod.ln_b, c.ln_eps,
                                    p, rt.rng, sid)
        if fused is not None:
            out, z, m, r = fused
        else:
            z = Fx.embed_fwd(ids, word, pos, typ, S, c.position_offset)
            if mod.ln_g is not None:
                _, x, m, r = Fx.ln_fwd(None, z, mod.ln_g, mod.ln_b, c.ln_eps, 0.0, rt.rng, 0)
            else:
                x, m, r = z, None, None
            out = Fx.dropout(x, p, rt.rng, sid)
        ctx.save_for_backward(ids, z, m, r)
        ctx.mod, ctx.p, ctx.sid, ctx.rng = mod, p, sid, rt.rng
        return out.view(B, S, h)

    @staticmethod
    def backward(ctx, dout):
        ids, z, m, r = ctx.saved_tensors
        mod = ctx.mod
        c, rng = mod.cfg, ctx.rng
        B, S = ids.shape
        h = c.hidden_size
        dx = Fx.dropout(dout.reshape(B * S, h).contiguous(), ctx.p, rng, ctx.sid)
        if mod.ln_g is not None:
            dz, _ = Fx.ln_bwd(dx, None, z, m, r, mod.ln_g, 0.0, rng, 0, want_dz=True,
                              dgamma=grad_dst(mod.ln_g), dbeta=grad_dst(mod.ln_b))
            grad_done(mod.ln_g)
            grad_done(mod.ln_b)
        else:
            dz = dx
        dst, acc = grad_dst(mod.word)
        Fx.embed_word_bwd(ids, dz, dst, acc, c.pad_token_id if c.family in ("bert", "opt") else -1)
        grad_done(mod.word)
        if mod.pos is not None:
            dst, acc = grad_dst(mod.pos)
            Fx.embed_pos_bwd(dz, dst, B, S, c.position_offset, acc)
            grad_done(mod.pos)
        if mod.tok_type is not None:
            dst, acc = grad_dst(mod.tok_type)
            if not acc:
                dst.zero_()
            Fx.bias_grad(dz, dst[0], True)
            grad_done(mod.tok_type)
        return (None, None) + (None,) * len(mod.params())


class Embeddings(nn.Module):
    token_input = True   # takes integer token ids (no input gradient): parallel/pipeline.py idle hooks

    def __init__(self, cfg: TransformerConfig, rt: Runtime):
        super().__init__()
        self.cfg, self.rt = cfg, rt
        h = cfg.hidden_size
        self.word = nn.Parameter(torch.empty(cfg.vocab_size, h))
        self.pos = nn.Parameter(torch.empty(cfg.max_positions + cfg.position_offset, h)) \
            if cfg.family in ("bert", "opt", "gpt2") else None
        self.tok_type = nn.Parameter(torch.empty(cfg.type_vocab_size, h)) if cfg.type_vocab_size else None
        if cfg.embedding_ln:
            self.ln_g = nn.Parameter(torch.ones(h))
            self.ln_b = nn.Parameter(torch.zeros(h))
        else:
            self.ln_g = self.ln_b = None
        with torch.no_grad():
            for p in (self.word, self.pos, self.tok_type):
                if p is not None:
                    p.normal_(0.0, 0.02)
            if cfg.family in ("bert", "opt"):
                self.word[cfg.pad_token_id].zero_()
        self.sid = rt.new_sid()

    def params(self):
        return tuple(p for p in (self.word, self.pos, self.tok_type, self.ln_g, self.ln_b) if p is not None)

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        self._dtd_weightless_bwd = self.rt.use_fused(self.word)   # see TransformerLayer.forward
        if self._dtd_weightless_bwd:
            note_use(self.params())
            return _EmbedFn.apply(ids, self, *self.params())
        c = self.cfg
        B, S = ids.shape
        x = F.embedding(ids, self.word, padding_idx=c.pad_token_id if c.family in ("bert", "opt") else None)
        if self.pos is not None:
            x = x + self.pos[c.position_offset:c.position_offset + S][None]
        if self.tok_type is not None:
            x = x + self.tok_type[0][None, None]
        if self.ln_g is not None:
            x = F.layer_norm(x, (c.hidden_size,), self.ln_g, self.ln_b, c.ln_eps)
        return ref_dropout(x, c.hidden_dropout, self.training, self.rt, self.rt.rng.sid(self.sid))


# ----------------------------------------------------------------------------- MLM head
# DTD_FUSED_XENT=1: the training forward computes loss, dlogits and the decoder-bias gradient in
# one pass (Fx.xent_fwd_train).  Off by default: -0.6 % end-to-end same box -- its per-row block
# reductions serialise the column-owning blocks (profiles/r2_ab_fused_xent_experiment.jsonl)
_FUSED_XENT = [os.environ.get("DTD_FUSED_XENT", "0") == "1"]


class _MLMHeadFn(torch.autograd.Function):
    """x [T,h] rows (already gathered for the sparse head) -> loss (mean over valid labels)."""

    @staticmethod
    def forward(ctx, x, labels, head, *params):
        c = head.cfg
        u = F.linear(x, head.dense_w, head.dense_b)
        a = Fx.act_fwd(u, c.activation)
        ctx.rng = head.rt.rng
        _, t, m, r = Fx.ln_fwd(None, a, head.ln_g, head.ln_b, c.ln_eps, 0.0, ctx.rng, 0)
        logits = F.linear(t, head.decoder_weight, head.decoder_bias)
        fused = Fx.xent_fwd_train(logits, labels) if any(ctx.needs_input_grad) and _FUSED_XENT[0] else None
        if fused is not None:
            # loss, dlogits and the decoder-bias gradient in one pass over the logits (for a loss
            # gradient of 1; the backward rescales otherwise): the logits are not kept
            loss, _, _, dlogits, dbias = fused
            ctx.save_for_backward(x, labels, u, a, t, m, r, dlogits, dbias)
        else:
            loss, lse, stats = Fx.xent_fwd(logits, labels)
            ctx.save_for_backward(x, labels, u, a, t, m, r, logits, lse, stats)
        ctx.fused = fused is not None
        ctx.head = head
        return loss

    @staticmethod
    def backward(ctx, gloss):
        head = ctx.head
        c = head.cfg
        if ctx.fused:
            x, labels, u, a, t, m, r, dlogits, dbias = ctx.saved_tensors
            Fx.xent_grad_scale_(dlogits, gloss)
            dst, acc = grad_dst(head.decoder_bias)
            g = dbias * gloss.reshape(1).float()
            if acc:
                dst.add_(g.to(dst.dtype))
            else:
                dst.copy_(g)
        else:
            x, labels, u, a, t, m, r, logits, lse, stats = ctx.saved_tensors
            # decoder-bias gradient (column sums of dlogits) from the same pass
            dlogits = Fx.xent_bwd(logits, labels, lse, stats, gloss, dbias=grad_dst(head.decoder_bias))
            del logits
        grad_done(head.decoder_bias)
        emit_wgrad(head.decoder_weight, dlogits, t)
        dt = G.dgrad(dlogits, head.decoder_weight)
        da, _ = Fx.ln_bwd(dt, None, a, m, r, head.ln_g, 0.0, ctx.rng, 0, want_dz=True,
                          dgamma=grad_dst(head.ln_g), dbeta=grad_dst(head.ln_b))
        grad_done(head.ln_g)
        grad_done(head.ln_b)
        du = Fx.act_bwd(da, u, c.activation, dbias=grad_dst(head.dense_b))
        grad_done(head.dense_b)
        emit_wgrad(head.dense_w, du, x)
        dx = G.dgrad(du, head.dense_w)
        return (dx, None, None) + (None,) * len(head.params())


class MLMHead(nn.Module):
    def __init__(self, cfg: TransformerConfig, rt: Runtime, word_embeddings: nn.Parameter | None,
                 sparse: bool = True):
        super().__init__()
        h = cfg.hidden_size
        self.cfg, self.rt, self.sparse = cfg, rt, sparse
        self.dense_w = nn.Parameter(torch.empty(h, h))
        self.dense_b = nn.Parameter(torch.zeros(h))
        init_linear_(self.dense_w, self.dense_b)
        self.ln_g = nn.Parameter(torch.ones(h))
        self.ln_b = nn.Parameter(torch.zeros(h))
        self.decoder_bias = nn.Parameter(torch.zeros(cfg.vocab_size))
        if word_embeddings is None:  # untied (BertModelWithMP builds its own head, bert_mp.py:24)
            self.decoder_w = nn.Parameter(torch.empty(cfg.vocab_size, h))
            init_linear_(self.decoder_w, None)
            self._tied = None
        else:
            self.decoder_w = None
            self._tied = [word_embeddings]  # list: not registered twice as a parameter

    @property
    def decoder_weight(self) -> nn.Parameter:
        return self.decoder_w if self.decoder_w is not None else self._tied[0]

    def params(self):
        return (self.dense_w, self.dense_b, self.ln_g, self.ln_b, self.decoder_weight, self.decoder_bias)

    def forward(self, x: torch.Tensor, labels: torch.Tensor | None = None) -> torch.Tensor:
        """Loss when labels are given, else logits (module call so ZeRO-3 unit hooks fire)."""
        # only the fused loss path keeps no weight views for the backward (TransformerLayer.forward)
        self._dtd_weightless_bwd = labels is not None and self.rt.use_fused(x)
        return self.loss(x, labels) if labels is not None else self.logits(x)

    def logits(self, x: torch.Tensor) -> torch.Tensor:
        """Full [.., V] prediction scores (differentiable through autograd)."""
        c = self.cfg
        u = F.linear(x, self.dense_w, self.dense_b)
        a = F.gelu(u) if c.activation == "gelu" else Fx._ref_act(u, c.activation)
        t = F.layer_norm(a, (c.hidden_size,), self.ln_g, self.ln_b, c.ln_eps)
        return F.linear(t, self.decoder_weight, self.decoder_bias)

    def _gather_labelled(self, x2: torch.Tensor, lab: torch.Tensor):
        """Rows with a label (~15% under MLM): the head GEMMs, CE and their backward run on
        these only.  With ``rt.mlm_capacity`` the gather has a static size (HIP-graph
        capturable): padding rows point at row 0 with label -100 (zero loss / gradient), and
        ``rt.mlm_overflow`` records on the device whether a batch had more labelled rows than
        the capacity (the caller checks it; identical loss and gradients otherwise)."""
        valid = lab != Fx.IGNORE_INDEX
        cap = self.rt.mlm_capacity
        if cap is None:
            idx = valid.nonzero().squeeze(1)
            return _gather_rows(x2, idx, None, idx.numel()), lab.index_select(0, idx)
        cap = min(cap, lab.numel())
        idx = torch.nonzero_static(valid, size=cap, fill_value=0).squeeze(1)
        count = valid.sum()
        keep = torch.arange(cap, device=lab.device) < count
        lab_sel = torch.where(keep, lab.index_select(0, idx), torch.full_like(idx, Fx.IGNORE_INDEX))
        if self.rt.mlm_overflow is not None:
            self.rt.mlm_overflow.logical_or_(count > cap)
        return _gather_rows(x2, idx, count, cap), lab_sel

    def loss(self, x: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        h = self.cfg.hidden_size
        x2 = x.reshape(-1, h)
        lab = labels.reshape(-1)
        if self.rt.use_fused(x):
            if self.sparse:
                x2, lab = self._gather_labelled(x2, lab)
            note_use(self.params())
            return _MLMHeadFn.apply(x2, lab, self, *self.params())
        logits = self.logits(x2)
        return F.cross_entropy(logits.float(), lab, ignore_index=Fx.IGNORE_INDEX)


class _GatherRows(torch.autograd.Function):
    """x[idx] whose backward writes the whole [rows, h] input gradient in one kernel pass
    (ops/csrc/embed.hip scatter_rows_kernel: labelled rows copied, the rest zero) instead of a zero
    fill plus index_add.  idx[0:n) ascending and unique, n = min(count, cap); entries past n are
    static-capacity padding whose gradient rows are zero (label -100)."""

    @staticmethod
    def forward(ctx, x, idx, count, cap):
        ctx.rows, ctx.cap, ctx.has_count = x.shape[0], int(cap), count is not None
        ctx.save_for_backward(idx, count if count is not None else idx)
        return x.index_select(0, idx)

    @staticmethod
    def backward(ctx, g):
        idx, count = ctx.saved_tensors
        g = g.contiguous()
        return Fx.scatter_rows(g, idx, count if ctx.has_count else None, ctx.cap, ctx.rows), None, None, None


_SCATTER_ROWS = [os.environ.get("DTD_MLM_SCATTER", "1") == "1"]


def _gather_rows(x: torch.Tensor, idx: torch.Tensor, count, cap: int) -> torch.Tensor:
    if _SCATTER_ROWS[0] and Fx.scatter_rows_supported(x) and torch.is_grad_enabled() and x.requires_grad:
        return _GatherRows.apply(x, idx, count, cap)
    return x.index_select(0, idx)


# ----------------------------------------------------------------------------- causal LM head
class _LMHeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, labels, head, w):
        logits = F.linear(x, w)
        loss, lse, stats = Fx.xent_fwd(logits, labels)
        ctx.save_for_backward(x, labels, logits, lse, stats)
        ctx.head = head
        return loss

    @staticmethod
    def backward(ctx, gloss):
        x, labels, logits, lse, stats = ctx.saved_tensors
        w = ctx.head.weight
        dlogits = Fx.xent_bwd(logits, labels, lse, stats, gloss)
        emit_wgrad(w, dlogits, x)
        return G.head_dgrad(dlogits, w), None, None, None


class LMHead(nn.Module):
    def __init__(self, cfg: TransformerConfig, rt: Runtime, word_embeddings: nn.Parameter):
        super().__init__()
        self.cfg, self.rt = cfg, rt
        self._tied = [word_embeddings]

    @property
    def weight(self):
        return self._tied[0]

    def forward(self, x: torch.Tensor, labels: torch.Tensor | None = None) -> torch.Tensor:
        self._dtd_weightless_bwd = labels is not None and self.rt.use_fused(x)   # TransformerLayer.forward
        return self.loss(x, labels) if labels is not None else self.logits(x)

    def logits(self, x):
        return F.linear(x, self.weight)

    def loss(self, x: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        """HF causal-LM loss: logits[:, :-1] vs labels[:, 1:], ignore_index -100."""
        B, S, h = x.shape
        if self.rt.use_fused(x):
            note_use((self.weight,))
            # all B*S positions (tile-aligned head GEMMs, no sliced copy): each sequence's last
            # position has no next token and takes label -100 -- zero loss and gradient, and the mean
            # runs over the same labelled rows.  bloom-560m b1: 512 instead of 511 rows makes the
            # logits / weight-gradient GEMMs 251 / 376 us vs 292 / 426 (profiles/r6_head_rows.json)
            ls = torch.cat([labels[:, 1:], labels.new_full((B, 1), Fx.IGNORE_INDEX)], 1).reshape(-1)
            return _LMHeadFn.apply(x.reshape(-1, h), ls, self, self.weight)
        xs = x[:, :-1].reshape(-1, h)
        ls = labels[:, 1:].reshape(-1)
        return F.cross_entropy(self.logits(xs).float(), ls, ignore_index=Fx.IGNORE_INDEX)
