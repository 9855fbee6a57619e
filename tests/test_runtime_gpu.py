"""Native batch producer feeding the GPU: pinned slots reused across batches, H2D on a side stream."""
import pytest
import torch

from distributed_training_and_deepspeed_amd.data import DeviceBatchLoader, DistributedSampler, NativeSyntheticLM
from distributed_training_and_deepspeed_amd.data import SyntheticLMDataset
from distributed_training_and_deepspeed_amd.models import config as C

pytestmark = pytest.mark.gpu


def test_device_loader_native_rows_on_gpu():
    cfg = C.get_config("base")
    ds = NativeSyntheticLM(cfg, 64, seq_len=512, seed=9)
    loader = DeviceBatchLoader(ds, 8, sampler=DistributedSampler(ds, 1, 0, shuffle=False), device="cuda")
    full, lab = ds.batch(0, 64)
    got = [b for b in loader]
    torch.cuda.synchronize()
    assert len(got) == 8
    for i, b in enumerate(got):    # slots are reused: every handed-out batch must stay intact
        assert b["input_ids"].is_cuda
        assert torch.equal(b["input_ids"].cpu(), full[8 * i:8 * i + 8])
        assert torch.equal(b["labels"].cpu(), lab[8 * i:8 * i + 8])


def test_device_loader_gathers_materialised_dataset_on_gpu():
    cfg = C.get_config("tiny")
    ds = SyntheticLMDataset(cfg, 48, seq_len=64, seed=2)
    sampler = DistributedSampler(ds, 2, 1, shuffle=True)
    order = list(iter(sampler))
    batches = list(DeviceBatchLoader(ds, 6, sampler=sampler, device="cuda"))
    torch.cuda.synchronize()
    ref = ds.input_ids[torch.tensor(order)]
    assert torch.equal(torch.cat([b["input_ids"] for b in batches]).cpu(), ref)
