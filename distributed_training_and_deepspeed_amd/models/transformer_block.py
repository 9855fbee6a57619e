"""Instrumented transformer block for memory estimation (reference model/transformer.py).

Every operation is its own ``nn.Module`` (Linear, ``MatMul``, Softmax, Dropout, ReLU, LayerNorm)
so forward hooks observe each activation the block materialises -- the input to the reference's
activation-memory measurement (estimate_transformer_memory.py:95-109).
OPT-style pre-LN block: LN -> q/k/v (q * head_dim^-0.5) -> bmm(QK^T) -> softmax -> dropout ->
bmm(PV) -> out_proj -> dropout -> +residual -> LN -> fc1 -> ReLU -> fc2 -> dropout -> +residual,
no attention mask (model/transformer.py:56-106).

The reference loads OPT-125m layer 0 from the hub to eyeball equivalence with HF's OPT layer;
without network access ``block_from_layer`` instead copies the weights of this framework's
fused ``TransformerLayer`` (pre-LN, ReLU, non-causal) into the instrumented block, and the test
suite asserts both produce the same output (an independent-implementation equivalence check).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
from torch import nn

from ..ops.functional import Softmax


class MatMul(nn.Module):
    """nn.Module wrapper for torch.bmm (so its output is visible to forward hooks)."""

    def forward(self, x, y):
        return torch.bmm(x, y)


@dataclass
class BlockConfig:
    hidden_size: int = 768
    num_attention_heads: int = 12
    ffn_dim: int = 3072
    max_position_embeddings: int = 2048
    dropout: float = 0.1
    enable_bias: bool = True
    layer_norm_eps: float = 1e-5


class TransformerBlock(nn.Module):
    def __init__(self, config: BlockConfig):
        super().__init__()
        self.config = config
        self.hidden_size = config.hidden_size
        self.num_attention_heads = config.num_attention_heads
        self.head_dim = config.hidden_size // config.num_attention_heads
        self.ffn_dim = config.ffn_dim
        self.scaling = self.head_dim ** -0.5
        h, b = self.hidden_size, config.enable_bias
        self.pre_attention_layer_norm = nn.LayerNorm(h, eps=config.layer_norm_eps)
        self.k_proj = nn.Linear(h, h, bias=b)
        self.v_proj = nn.Linear(h, h, bias=b)
        self.q_proj = nn.Linear(h, h, bias=b)
        self.out_proj = nn.Linear(h, h, bias=b)
        self.compute_attention_weights = MatMul()
        self.attention_weights_softmax = Softmax(dim=-1)   # HIP row-softmax kernel on the GPU
        self.attention_weights_dropout = nn.Dropout(config.dropout)
        self.compute_attentions = MatMul()
        self.attention_output_dropout = nn.Dropout(config.dropout)
        self.final_layer_norm = nn.LayerNorm(h, eps=config.layer_norm_eps)
        self.ffn_1 = nn.Linear(h, self.ffn_dim, bias=b)
        self.ffn_2 = nn.Linear(self.ffn_dim, h, bias=b)
        self.activation = nn.ReLU()
        self.final_dropout = nn.Dropout(config.dropout)

    def forward(self, hidden_states: torch.Tensor) -> torch.Tensor:
        residual = hidden_states
        B, T, _ = hidden_states.shape
        H, D = self.num_attention_heads, self.head_dim
        hidden_states = self.pre_attention_layer_norm(hidden_states)

        def heads(t):
            return t.view(B, T, H, D).transpose(1, 2).contiguous().view(B * H, T, D)
        query = heads(self.q_proj(hidden_states) * self.scaling)
        key = heads(self.k_proj(hidden_states))
        value = heads(self.v_proj(hidden_states))
        attn = self.compute_attention_weights(query, key.transpose(1, 2))
        attn = self.attention_weights_softmax(attn)
        attn = self.attention_weights_dropout(attn)
        out = self.compute_attentions(attn, value).view(B, H, T, D).transpose(1, 2).reshape(B, T, self.hidden_size)
        out = self.attention_output_dropout(self.out_proj(out))
        hidden_states = out + residual
        shape = hidden_states.shape
        hidden_states = hidden_states.reshape(-1, hidden_states.size(-1))
        residual = hidden_states
        hidden_states = self.final_layer_norm(hidden_states)
        hidden_states = self.ffn_2(self.activation(self.ffn_1(hidden_states)))
        hidden_states = self.final_dropout(hidden_states)
        return (residual + hidden_states).view(shape)


def block_from_layer(layer) -> TransformerBlock:
    """Copy a fused ``TransformerLayer`` (pre-LN, ReLU) into an instrumented block."""
    c = layer.cfg
    cfg = BlockConfig(hidden_size=c.hidden_size, num_attention_heads=c.num_heads, ffn_dim=c.ffn_size,
                      max_position_embeddings=c.max_positions, dropout=c.hidden_dropout, layer_norm_eps=c.ln_eps)
    blk = TransformerBlock(cfg).to(layer.qkv_w.dtype)
    h = c.hidden_size
    with torch.no_grad():
        q, k, v = layer.qkv_w.split(h, 0)
        qb, kb, vb = layer.qkv_b.split(h, 0)
        for lin, w, b in ((blk.q_proj, q, qb), (blk.k_proj, k, kb), (blk.v_proj, v, vb), (blk.out_proj, layer.o_w, layer.o_b),
                          (blk.ffn_1, layer.fc1_w, layer.fc1_b), (blk.ffn_2, layer.fc2_w, layer.fc2_b)):
            lin.weight.copy_(w)
            lin.bias.copy_(b)
        blk.pre_attention_layer_norm.weight.copy_(layer.ln1_g)
        blk.pre_attention_layer_norm.bias.copy_(layer.ln1_b)
        blk.final_layer_norm.weight.copy_(layer.ln2_g)
        blk.final_layer_norm.bias.copy_(layer.ln2_b)
    return blk
