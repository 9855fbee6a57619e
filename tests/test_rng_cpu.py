"""Statistics of the attention-dropout keep stream (ops/rng.py attn_keep_mask, the bit-exact CPU
form of ops/csrc/attention.hip attn_mask_kernel: hash-seeded per-query state, one additive
lagged-Fibonacci round with rotation per 32-key word, bit-plane comparator).  The GPU kernel is
checked bit for bit against this function in tests/test_attention_gpu.py."""
import pytest
import torch

from distributed_training_and_deepspeed_amd.ops.rng import attn_keep_mask, keep_threshold


def _corr(a, b):
    a, b = a - a.mean(), b - b.mean()
    return ((a * b).mean() / (a.std() * b.std())).item()


@pytest.mark.parametrize("p", [0.05, 0.1, 0.5, 0.9])
def test_keep_rate_matches_threshold(p):
    k = attn_keep_mask(2, 2, 256, p, 9, 1, 2).float()
    want = 1.0 - keep_threshold(p) / 65536.0
    # 262 k Bernoulli draws: 5 sigma
    assert abs(k.mean().item() - want) < 5 * (want * (1 - want) / k.numel()) ** 0.5


def test_keep_stream_has_no_neighbour_correlation():
    k = attn_keep_mask(2, 4, 512, 0.1, 5, 3, 7).float()          # 2.1 M decisions
    lim = 5 / k[..., 1:].numel() ** 0.5
    assert abs(_corr(k[..., :-1], k[..., 1:])) < lim              # adjacent keys (one word / plane)
    assert abs(_corr(k[..., :-32], k[..., 32:])) < lim            # same bit of consecutive words
    assert abs(_corr(k[:, :, :-1], k[:, :, 1:])) < lim            # adjacent queries (streams)
    assert abs(_corr(k[:, 0], k[:, 1])) < 2 * lim                 # heads
    rates = k.view(2, 4, 512, 16, 32).mean((0, 1, 2))             # [word][bit]
    assert (rates - 0.9).abs().max().item() < 0.02               # no weak word or bit column


def test_keep_stream_edges():
    assert attn_keep_mask(1, 2, 100, 0.0, 1, 1, 1).all()
    assert not attn_keep_mask(1, 2, 100, 1.0, 1, 1, 1).any()
    a = attn_keep_mask(1, 2, 64, 0.1, 1, 1, 1)
    assert not torch.equal(a, attn_keep_mask(1, 2, 64, 0.1, 1, 2, 1))     # step advances the stream
    assert not torch.equal(a, attn_keep_mask(1, 2, 64, 0.1, 1, 1, 2))     # call sites differ
    assert torch.equal(a, attn_keep_mask(1, 2, 64, 0.1, 1, 1, 1))
