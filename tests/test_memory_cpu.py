"""Memory estimators (reference estimate_*_memory.py) and the instrumented block."""
import torch

from distributed_training_and_deepspeed_amd.memory import (ActivationCounter, max_hidden_for_capacity,
                                                           project_training_memory, project_transformer_memory,
                                                           register_hooks_recursive)
from distributed_training_and_deepspeed_amd.models import config as C
from distributed_training_and_deepspeed_amd.models.transformer import Runtime, TransformerLayer
from distributed_training_and_deepspeed_amd.models.transformer_block import block_from_layer
from distributed_training_and_deepspeed_amd.utils import format_size


def test_estimate_nn_memory_demo():
    import estimate_nn_memory
    model_b, act_b = estimate_nn_memory.main()
    assert model_b == 12_597_248
    assert act_b == 4 * (1024 + 1024 + 1024 + 512) * 4 + 4 * 512 * 4


def test_reference_projection_17gb():
    n = 12 * 9216 ** 2 + 13 * 9216
    b = project_transformer_memory(1, 9216, 72, 4, 512, 8, num_params=n)
    assert format_size(b) == "17.0 GB"


def test_capacity_inversion_288gb():
    assert max_hidden_for_capacity() == 38144  # h ~ 38,144 under 288 GB


def test_zero_partitioning_shrinks_per_rank_state():
    full = project_training_memory(24, 1024, 16, 1, 512, precision="bf16", zero_stage=0, world_size=8)
    z1 = project_training_memory(24, 1024, 16, 1, 512, precision="bf16", zero_stage=1, world_size=8)
    z3 = project_training_memory(24, 1024, 16, 1, 512, precision="bf16", zero_stage=3, world_size=8)
    assert z1.optimizer == full.optimizer / 8 and z3.weights == full.weights / 8
    assert full.total > z1.total > z3.total


def test_activation_counter_dropout_is_one_byte():
    m = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Dropout(0.1))
    c = ActivationCounter()
    register_hooks_recursive(m, c)
    m(torch.randn(2, 8))
    assert c.activation_bytes == 2 * 16 * 4 + 2 * 16 * 1


def test_instrumented_block_equals_fused_layer():
    cfg = C.W4_BLOCK.with_(hidden_size=64, num_heads=4, ffn_size=256, hidden_dropout=0.0, attn_dropout=0.0)
    torch.manual_seed(0)
    layer = TransformerLayer(cfg, Runtime(impl="fused"))
    blk = block_from_layer(layer)
    blk.eval()
    x = torch.randn(2, 16, 64)
    assert torch.allclose(layer(x), blk(x), atol=1e-5)


def test_max_params_projection_grows_with_zero_stage():
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench"))
    import max_params
    rows = {(r["world"], r["stage"]): r for r in max_params.projection_table(0.92)}
    assert rows[(1, 0)]["params_B"] > 10                       # 16 B/param: >10 B params in 288 GB
    p8 = [rows[(8, s)]["params_B"] for s in range(4)]
    assert p8 == sorted(p8) and p8[3] > 5 * p8[0]               # partitioning multiplies capacity
    assert all(r["projected_GB_per_gpu"] <= 0.92 * 288 * 1.0737 for r in rows.values())
