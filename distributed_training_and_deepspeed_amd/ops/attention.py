"""Scaled-dot-product attention core: flash-style HIP kernels (gfx950 MFMA) + math reference.

Layout contract (shared by kernels, reference and models): the fused projection output
``qkv`` is ``[B*S, 3*H*D]`` viewed as ``[B, S, 3, H, D]`` (q, k, v blocks), the context
output ``ctx`` is ``[B*S, H*D]`` and the log-sum-exp ``lse`` is ``[B, H, S]`` fp32 (natural
log of sum(exp(score)), score = q.k * scale + bias).  Supported score modifiers: causal mask,
ALiBi (BLOOM: bias = slope_h * key_position, which equals BLOOM's relative form up to a
per-row constant that softmax cancels) and dropout on the probabilities with the counter RNG
(mask element index = ((b*H + h)*S + i)*S + j, regenerated in backward).

Reference semantics: HF BertSelfAttention eager path (matmul, softmax, dropout, matmul --
SURVEY.md K2, reference model/transformer.py:80-86); the reference never passes an
attention mask for BERT (data_parallel_training.py:53), so padding is attended to.
"""
from __future__ import annotations

import math
import os

import torch

from . import _lib
from .rng import RngState, attn_keep_mask


def alibi_slopes(num_heads: int) -> torch.Tensor:
    """BLOOM/ALiBi head slopes (geometric sequence, with the interleaved extension for
    non-power-of-two head counts)."""
    def pow2(n):
        start = 2 ** (-(2 ** -(math.log2(n) - 3)))
        return [start * (start ** i) for i in range(n)]
    if math.log2(num_heads).is_integer():
        s = pow2(num_heads)
    else:
        c = 2 ** math.floor(math.log2(num_heads))
        s = pow2(c) + pow2(2 * c)[0::2][: num_heads - c]
    return torch.tensor(s, dtype=torch.float32)


def _split(qkv, B, S, H, D):
    x = qkv.view(B, S, 3, H, D)
    return x[:, :, 0].transpose(1, 2), x[:, :, 1].transpose(1, 2), x[:, :, 2].transpose(1, 2)


def _cdt(t: torch.Tensor) -> torch.dtype:
    """Compute dtype of the math reference: fp64 for fp64 inputs (kernel tests), else fp32."""
    return torch.float64 if t.dtype == torch.float64 else torch.float32


def _scores(q, k, scale, causal, slopes):
    c = _cdt(q)
    s = torch.matmul(q.to(c), k.to(c).transpose(-1, -2)) * scale
    S = q.shape[2]
    if slopes is not None:
        s = s + slopes.to(s.device).view(1, -1, 1, 1) * torch.arange(S, device=s.device, dtype=s.dtype).view(1, 1, 1, S)
    if causal:
        m = torch.ones(S, S, dtype=torch.bool, device=s.device).triu(1)
        s = s.masked_fill(m, float("-inf"))
    return s


def _drop_mask(B, H, S, p, rng, sid, device):
    seed, step = (int(v) for v in rng.state.tolist())
    return attn_keep_mask(B, H, S, p, seed, step, sid, device=device)


def attn_fwd_ref(qkv, B, S, H, D, causal=False, slopes=None, p=0.0, rng: RngState | None = None, sid=0,
                 scale=None):
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    q, k, v = _split(qkv, B, S, H, D)
    s = _scores(q, k, scale, causal, slopes)
    lse = torch.logsumexp(s, -1)
    prob = torch.exp(s - lse[..., None])
    if p > 0:
        prob = prob * _drop_mask(B, H, S, p, rng, sid, qkv.device) / (1.0 - p)
    ctx = torch.matmul(prob, v.to(prob.dtype))  # [B,H,S,D]
    return ctx.transpose(1, 2).reshape(B * S, H * D).to(qkv.dtype), lse


def attn_bwd_ref(dctx, qkv, ctx, lse, B, S, H, D, causal=False, slopes=None, p=0.0, rng=None, sid=0, scale=None):
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    q, k, v = _split(qkv, B, S, H, D)
    s = _scores(q, k, scale, causal, slopes)
    prob = torch.exp(s - lse[..., None].to(s.dtype))
    c = s.dtype
    do = dctx.view(B, S, H, D).transpose(1, 2).to(c)
    o = ctx.view(B, S, H, D).transpose(1, 2).to(c)
    if p > 0:
        keep = _drop_mask(B, H, S, p, rng, sid, qkv.device).to(c) / (1.0 - p)
        pd = prob * keep
    else:
        keep, pd = None, prob
    dv = torch.matmul(pd.transpose(-1, -2), do)
    dpd = torch.matmul(do, v.to(c).transpose(-1, -2))
    dp = dpd * keep if keep is not None else dpd
    delta = (do * o).sum(-1, keepdim=True)
    ds = prob * (dp - delta)
    dq = torch.matmul(ds, k.to(c)) * scale
    dk = torch.matmul(ds.transpose(-1, -2), q.to(c)) * scale
    dqkv = torch.stack([dq, dk, dv], dim=2)  # [B,H,3,S,D]
    return dqkv.permute(0, 3, 2, 1, 4).reshape(B * S, 3 * H * D).to(qkv.dtype)


_WARNED = []


def _warn_once():
    if not _WARNED:
        import warnings
        warnings.warn("HIP flash-attention kernel not built: using the math reference on GPU")
        _WARNED.append(1)


_BWD_FORMS = ("split", "fused", "fused4")


def set_bwd_form(form: str) -> str:
    """'fused': one-kernel backward (one workgroup per (batch, head), dQ summed in LDS) where it
    applies -- head_dim 64, no causal mask / ALiBi, S % 128 == 0, S <= 512; 8 waves (two per SIMD)
    at S = 512, else 4.  'fused4': the 4-wave form at every S.  'split': the dQ + dK/dV
    kernel pair.  Returns the previous form.  Without an experimental build every form runs the
    split kernels."""
    old = _lib.lib().dtd_attn_set_bwd_form(_BWD_FORMS.index(form))
    return _BWD_FORMS[old]


def fused_bwd_built() -> bool:
    """The one-kernel backward forms are compiled only into experimental builds
    (DTD_BUILD_EXPERIMENTAL=1): they measured no faster than the split kernels."""
    return _lib.has("dtd_attn_fused_bwd_built") and bool(_lib.lib().dtd_attn_fused_bwd_built())


def fused_bwd_applies(S: int, D: int, causal: bool, slopes) -> bool:
    return D == 64 and not causal and slopes is None and S % 128 == 0 and S <= 512 and fused_bwd_built()


def kernel_supported(qkv: torch.Tensor, D: int) -> bool:
    return qkv.is_cuda and qkv.dtype == torch.bfloat16 and D in (64, 128) and _lib.has("dtd_attn_fwd")


def f32_kernel_supported(qkv: torch.Tensor, D: int) -> bool:
    """The reference-precision kernels (ops/csrc/attention_f32.hip: exact f32 MFMA products)."""
    return (qkv.is_cuda and qkv.dtype == torch.float32 and D in (64, 128) and _lib.has("dtd_attn_fwd_f32")
            and _lib.has("dtd_attn_masks"))


def _masks_now(B, S, H, p, rng, sid, device) -> torch.Tensor:
    """Dropout keep bits generated on the current stream (the fp32 path)."""
    masks = alloc_masks(B, H, S, device)
    _lib.call("dtd_attn_masks", masks.data_ptr(), B, S, H, float(p), rng.state.data_ptr(), sid, _lib.stream())
    return masks


_SIDE = {}


def _side_stream(device) -> torch.cuda.Stream:
    s = _SIDE.get(device)
    if s is None:
        s = _SIDE[device] = torch.cuda.Stream(device)
    return s


def mask_words(B: int, H: int, S: int) -> int:
    """Words per keep-bit layout of one attention call: [B*H][W][32 W], W = ceil(S / 32)."""
    W = (S + 31) // 32
    return B * H * W * 32 * W


def alloc_masks(B: int, H: int, S: int, device) -> torch.Tensor:
    """[2, mask_words] int32 keep-bit buffer (both layouts back to back), exactly sized: every keep
    word the attention kernels read lies inside it (their scalar-load addresses are clamped into
    the (batch, head) plane and the row, ops/csrc/attention.hip keep_off; the vector prefetches go
    through bounded buffer resources)."""
    n = mask_words(B, H, S)
    return torch.empty((2, n), dtype=torch.int32, device=device)


def _lm_pos(n: int) -> torch.Tensor:
    """Word position of each of n positions inside its [32 W] row (ops/csrc/attention.hip lm_pos:
    within a 32-group, c = 8a + 4b + j sits at 8a + 2j + b)."""
    x = torch.arange(n)
    c = x & 31
    return (x & ~31) | (c & 24) | ((c & 3) << 1) | ((c >> 2) & 1)


def decode_masks(masks: torch.Tensor, B: int, H: int, S: int) -> tuple[torch.Tensor, torch.Tensor]:
    """The two generated keep-bit layouts as [B*H, S, S] 0/1 int64 tensors (query, key): A (key
    bits per query word) and B (query bits per key word) -- both must equal attn_keep_mask."""
    W = (S + 31) // 32
    m = masks.cpu().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    pos = _lm_pos(S)
    bits = torch.arange(32, dtype=torch.int64)
    out = []
    for li in range(2):
        words = m[li].view(B * H, W, 32 * W)[:, :, pos]          # [bh][w][position]
        d = ((words.unsqueeze(-1) >> bits) & 1).permute(0, 2, 1, 3).reshape(B * H, S, W * 32)[..., :S]
        out.append(d if li == 0 else d.transpose(1, 2))            # B: [bh][key][q] -> [bh][q][key]
    return out[0], out[1]


class PendingMasks:
    """Dropout keep-bit masks being generated on a side stream (see ``attn_masks_async``)."""

    def __init__(self, masks: torch.Tensor, event: torch.cuda.Event):
        self.masks, self.event = masks, event


_MASK_REPEAT = max(1, int(os.environ.get("DTD_ATTN_MASK_REPEAT", "1")))


def attn_masks_async(B, S, H, D, p, rng: RngState, sid, device) -> PendingMasks | None:
    """Start generating the attention-dropout keep bits on a side stream.  The kernel is pure
    VALU (counter-RNG hashing) and independent of the activations, so issued before the QKV
    projection it runs concurrently with that MFMA-bound GEMM; ``attn_fwd(masks=...)`` joins
    it.  Returns None when the kernel path is not used (CPU / reference)."""
    if p <= 0 or not torch.cuda.is_available() or torch.device(device).type != "cuda" or D not in (64, 128) \
            or not _lib.has("dtd_attn_masks"):
        return None
    cur = torch.cuda.current_stream(device)
    masks = alloc_masks(B, H, S, device)
    side = _side_stream(torch.device(device))
    side.wait_stream(cur)                      # the rng step / previous users of the buffer
    with torch.cuda.stream(side):
        for _ in range(_MASK_REPEAT):   # (diagnostic: DTD_ATTN_MASK_REPEAT > 1 prices the generator)
            _lib.call("dtd_attn_masks", masks.data_ptr(), B, S, H, float(p), rng.state.data_ptr(), sid,
                      side.cuda_stream)
        ev = torch.cuda.Event()
        ev.record(side)
    return PendingMasks(masks, ev)


def attn_fwd(qkv, B, S, H, D, causal=False, slopes=None, p=0.0, rng: RngState | None = None, sid=0,
             masks: PendingMasks | None = None):
    """Returns (ctx [B*S, H*D], lse [B, H, S] fp32, masks).  ``masks`` holds the dropout keep
    bits for the backward ([2, B*H*S*ceil(S/32)] int32 on the kernel path, None otherwise);
    pass the ``attn_masks_async`` result to reuse masks generated ahead on a side stream."""
    if f32_kernel_supported(qkv, D):
        return _attn_fwd_f32(qkv, B, S, H, D, causal, slopes, p, rng, sid, masks)
    if not kernel_supported(qkv, D):
        if qkv.is_cuda and qkv.dtype == torch.bfloat16 and _lib.has("dtd_attn_fwd") is False:
            _warn_once()
        ctx, lse = attn_fwd_ref(qkv, B, S, H, D, causal, slopes, p, rng, sid)
        return ctx, lse, None
    qkv = qkv.contiguous()
    ctx = torch.empty((B * S, H * D), dtype=qkv.dtype, device=qkv.device)
    lse = torch.empty((B, H, S), dtype=torch.float32, device=qkv.device)
    rng_ptr = rng.state.data_ptr() if rng is not None else None
    if p > 0 and masks is not None:
        torch.cuda.current_stream(qkv.device).wait_event(masks.event)
        masks, rng_ptr = masks.masks, None     # generated already
    elif p > 0:
        masks = alloc_masks(B, H, S, qkv.device)
    else:
        masks = None
    sl = slopes.to(device=qkv.device, dtype=torch.float32).contiguous() if slopes is not None else None
    # q/k/v are strided views into qkv: row stride 3*H*D, head stride D.
    ld = 3 * H * D
    base = qkv.data_ptr()
    es = qkv.element_size()
    _lib.call("dtd_attn_fwd", base, base + H * D * es, base + 2 * H * D * es, ctx.data_ptr(), lse.data_ptr(),
              _lib.ptr(sl), _lib.ptr(masks), B, S, H, D, ld, H * D, int(causal), 1.0 / math.sqrt(D), float(p),
              rng_ptr, sid, _lib.stream())
    return ctx, lse, masks


def attn_bwd(dctx, qkv, ctx, lse, B, S, H, D, causal=False, slopes=None, p=0.0, rng=None, sid=0, masks=None,
             dbias=None):
    """Returns dqkv [B*S, 3*H*D] in the qkv layout.  ``dbias`` = (dst, acc): also writes the
    column sums of dqkv (the qkv projection's bias gradient) -- on the kernel path as per-wave
    partials from the dQ / dK,dV epilogues (no extra pass over dqkv)."""
    from . import functional as Fx
    if f32_kernel_supported(qkv, D) and (p <= 0 or masks is not None):
        dqkv = _attn_bwd_f32(dctx, qkv, ctx, lse, B, S, H, D, causal, slopes, p, masks)
        if dbias is not None:
            Fx.bias_grad(dqkv, *dbias)
        return dqkv
    if not kernel_supported(qkv, D):
        dqkv = attn_bwd_ref(dctx, qkv, ctx, lse, B, S, H, D, causal, slopes, p, rng, sid)
        if dbias is not None:
            Fx.bias_grad(dqkv, *dbias)
        return dqkv
    dctx = dctx.contiguous()
    dqkv = torch.empty_like(qkv)
    delta = torch.empty((B, H, S), dtype=torch.float32, device=qkv.device)
    sl = slopes.to(device=qkv.device, dtype=torch.float32).contiguous() if slopes is not None else None
    ld = 3 * H * D
    es = qkv.element_size()
    qb, gb = qkv.data_ptr(), dqkv.data_ptr()
    part = None
    if dbias is not None and D == 64:
        # one row per (batch, 32-row block of a 128-row workgroup tile); every entry is written
        part = torch.empty((B * 4 * ((S + 127) // 128), ld), dtype=torch.float32, device=qkv.device)
    _lib.call("dtd_attn_bwd", qb, qb + H * D * es, qb + 2 * H * D * es, ctx.data_ptr(), dctx.data_ptr(),
              lse.data_ptr(), delta.data_ptr(), _lib.ptr(masks), gb, gb + H * D * es, gb + 2 * H * D * es,
              _lib.ptr(sl), B, S, H, D, ld, H * D, int(causal), 1.0 / math.sqrt(D), float(p), _lib.ptr(part),
              _lib.stream())
    if dbias is not None:
        if part is not None:
            dst, acc = dbias
            Fx._finalize(part, part.shape[0], ld, (dst, acc), acc)
        else:
            Fx.bias_grad(dqkv, *dbias)
    return dqkv


def _attn_fwd_f32(qkv, B, S, H, D, causal, slopes, p, rng, sid, masks):
    qkv = qkv.contiguous()
    ctx = torch.empty((B * S, H * D), dtype=qkv.dtype, device=qkv.device)
    lse = torch.empty((B, H, S), dtype=torch.float32, device=qkv.device)
    if p > 0:
        if masks is not None:
            torch.cuda.current_stream(qkv.device).wait_event(masks.event)
            masks = masks.masks
        else:
            masks = _masks_now(B, S, H, p, rng, sid, qkv.device)
    else:
        masks = None
    sl = slopes.to(device=qkv.device, dtype=torch.float32).contiguous() if slopes is not None else None
    ld, es, base = 3 * H * D, qkv.element_size(), qkv.data_ptr()
    _lib.call("dtd_attn_fwd_f32", base, base + H * D * es, base + 2 * H * D * es, ctx.data_ptr(), lse.data_ptr(),
              _lib.ptr(sl), _lib.ptr(masks), B, S, H, D, ld, H * D, int(causal), 1.0 / math.sqrt(D), float(p),
              _lib.stream())
    return ctx, lse, masks


def _attn_bwd_f32(dctx, qkv, ctx, lse, B, S, H, D, causal, slopes, p, masks):
    dctx = dctx.contiguous()
    dqkv = torch.empty_like(qkv)
    delta = torch.empty((B, H, S), dtype=torch.float32, device=qkv.device)
    sl = slopes.to(device=qkv.device, dtype=torch.float32).contiguous() if slopes is not None else None
    ld, es = 3 * H * D, qkv.element_size()
    qb, gb = qkv.data_ptr(), dqkv.data_ptr()
    _lib.call("dtd_attn_bwd_f32", qb, qb + H * D * es, qb + 2 * H * D * es, ctx.data_ptr(), dctx.data_ptr(),
              lse.data_ptr(), delta.data_ptr(), _lib.ptr(masks if p > 0 else None), gb, gb + H * D * es,
              gb + 2 * H * D * es, _lib.ptr(sl), B, S, H, D, ld, H * D, int(causal), 1.0 / math.sqrt(D), float(p),
              _lib.stream())
    return dqkv
