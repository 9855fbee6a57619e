"""Whole-step hipGraph capture (utils/graphs.py): replaying the captured step trains exactly like
running the same step eagerly (same kernels, same static MLM capacity, device-side RNG step)."""
import pytest
import torch

from distributed_training_and_deepspeed_amd.data import SyntheticLMDataset
from distributed_training_and_deepspeed_amd.models import build_model
from distributed_training_and_deepspeed_amd.optim import hf_adamw
from distributed_training_and_deepspeed_amd.parallel import DistributedDataParallel
from distributed_training_and_deepspeed_amd.utils.graphs import CapturedStep, mlm_capacity

pytestmark = pytest.mark.gpu


def _setup():
    model = build_model("tiny", dtype=torch.bfloat16, device="cuda", seed=3)
    model.rt.mlm_capacity = mlm_capacity(4 * 128)
    model.rt.mlm_overflow = torch.zeros((), dtype=torch.bool, device="cuda")
    ddp = DistributedDataParallel(model)
    opt = hf_adamw(ddp.parameters(), lr=1e-3)

    def step(input_ids, labels):
        out = ddp(input_ids, labels=labels)
        out.loss.backward()
        opt.step()
        model.rt.rng.advance()
        return out.loss.detach()
    return model, step


def test_captured_step_matches_eager():
    ds = SyntheticLMDataset(build_model("tiny").cfg, 4 * 8, seq_len=128, seed=5)
    ids = ds.input_ids.view(8, 4, 128).cuda()
    lab = ds.labels.view(8, 4, 128).cuda()
    ma, sa = _setup()
    mb, sb = _setup()
    # B: 3 warm-up steps run eagerly inside CapturedStep, then replays; A: the same 3 + replays eagerly
    cap = CapturedStep(sb, {"input_ids": ids[0], "labels": lab[0]}, warmup=3, runtime=mb.rt)
    la = [sa(ids[0], lab[0]) for _ in range(3)]
    la += [sa(ids[i], lab[i]) for i in range(1, 6)]
    lb = [cap(input_ids=ids[i], labels=lab[i]).clone() for i in range(1, 6)]
    torch.cuda.synchronize()
    cap.check()
    assert torch.equal(torch.stack(la[3:]), torch.stack(lb))
    for (n, p), q in zip(ma.named_parameters(), mb.parameters()):
        assert torch.equal(p, q), n
