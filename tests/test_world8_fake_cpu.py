"""World-8 bookkeeping without 8 processes: torch's ``fake`` process group (collectives are
no-ops) drives the real DDP bucketing and ZeRO partitioning code at the 8-GPU node size
(SURVEY.md section 4, item 4)."""
import pytest
import torch
import torch.distributed as dist

from distributed_training_and_deepspeed_amd.models import build_model, count_parameters


@pytest.fixture
def fake_world8():
    from torch.testing._internal.distributed.fake_pg import FakeStore
    dist.init_process_group("fake", store=FakeStore(), rank=3, world_size=8)
    yield
    dist.destroy_process_group()


def test_ddp_buckets_bert_base_world8(fake_world8):
    from distributed_training_and_deepspeed_amd.parallel import DistributedDataParallel
    model = build_model("bert-base", dtype=torch.float32, seed=0)
    ddp = DistributedDataParallel(model, bucket_cap_mb=25)       # reference default, fp32 grads
    sizes = ddp.bucket_sizes_bytes()
    total = sum(sizes)
    assert total >= count_parameters(model) * 4
    # ~17-18 buckets of <= 25 MiB plus the 89 MB word-embedding bucket
    assert 15 <= len(sizes) <= 20, len(sizes)
    assert max(sizes) >= 28996 * 768 * 4 and sorted(sizes)[-2] <= 25 * 2 ** 20
    # bf16 gradients halve the traffic (and the bucket count)
    ddp16 = DistributedDataParallel(model, bucket_cap_mb=25, grad_dtype=torch.bfloat16, broadcast_parameters=False)
    assert sum(ddp16.bucket_sizes_bytes()) * 2 == total


@pytest.mark.parametrize("stage", [1, 2, 3])
def test_zero_partitions_world8(fake_world8, stage):
    from distributed_training_and_deepspeed_amd.parallel.zero import initialize
    model = build_model("bert-base", dtype=torch.float32, seed=0)
    n = count_parameters(model)
    eng, opt, _, _ = initialize(model=model, model_parameters=model.parameters(),
                                config={"zero_optimization": {"stage": stage, "reduce_bucket_size": 5e6}})
    part = eng.partition_numel()
    assert n / 8 <= part <= n / 8 * 1.01 + 64 * 8 * len(eng.segments)   # 1/8 of the state (+ alignment)
    assert opt.exp_avg.numel() == part and eng.master.numel() == part
    st = eng.state_bytes_per_rank()
    assert st["adam_moments"] == 8 * part
    if stage == 3:   # only the shards of the stage-3 units stay resident
        resident = sum(p.numel() for p in model.parameters())
        assert resident < n / 2
