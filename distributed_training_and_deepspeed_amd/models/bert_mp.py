"""BERT with layer-wise model parallelism and GPipe pipelining (reference model/bert_mp.py).

``BertModelWithMP(config, device_count, verbose)`` builds embeddings + N encoder layers + an
*untied* MLM head (130.6 M parameters for bert-base, reference model/bert_mp.py:22-24) and
places the flat module list [emb, L0..L{N-1}, head] on devices with the ``np.array_split``
law (model/bert_mp.py:39-47).  ``forward(input_ids)`` returns prediction logits on the head
device, moving activations between device groups on copy streams.  ``to_pipeline(chunks)``
returns a GPipe pipeline over the same groups (checkpointing every micro-batch except the
last, torch Pipe's default).  Idle time per device is tracked with HIP events
(``device_idle_time[d] = (sum_ms, count)``, as the reference's dict) and printed by
``model_parallel_training.py``.

Device clamping / warnings follow model/bert_mp.py:28-37 (including the reference's message
text, minus its missing f-prefix, quirk 5).  ``devices=[...]`` places stages explicitly, e.g.
two "stages" on one GPU to exercise the schedule on a single-GPU machine.
"""
from __future__ import annotations

import torch
from torch import nn

from ..ops.rng import RngState
from ..parallel.pipeline import GPipe, IdleTimeTracker, attach_idle_hooks, partition
from ..parallel.p2p import send_to
from ..utils import get_device, get_device_count
from .config import BERT_BASE, TransformerConfig
from .layers import Embeddings, MLMHead
from .transformer import Runtime, TransformerLayer


class _HeadLogits(nn.Module):
    def __init__(self, head: MLMHead):
        super().__init__()
        self.head = head

    def forward(self, x):
        return self.head.logits(x)


class BertModelWithMP(nn.Module):
    """Minimal BERT with support for model and pipeline parallelism."""

    def __init__(self, config: TransformerConfig = BERT_BASE, device_count: int | None = None, verbose: bool = False,
                 devices=None, dtype: torch.dtype = torch.float32, impl: str = "auto", timing: str = "device",
                 seed: int = 0):
        super().__init__()
        self.config = config
        self.verbose = verbose
        torch.manual_seed(seed)
        device_type = get_device()
        if devices is None:
            device_count = device_count or get_device_count()
            print("Using device: {}".format(device_type))
            if device_count <= 1:
                print(f"Only one {device_type} device is available. Training will be done without Model Parallelism.")
            elif device_count > get_device_count():
                print(f"Cannot use {device_count} {device_type} devices. Only {get_device_count()} devices are available. "
                      f"Training will be done using {get_device_count()} devices.")
                device_count = get_device_count()
            device_count = max(1, device_count)
            devices = [torch.device(device_type, i) if device_type != "cpu" else torch.device("cpu")
                       for i in range(device_count)]
        self.group_devices = [torch.device(d) for d in devices]
        self.rt = Runtime(impl=impl, rng=RngState(seed))
        self.embeddings = Embeddings(config, self.rt)
        self.encoders = nn.ModuleList([TransformerLayer(config, self.rt) for _ in range(config.num_layers)])
        self.head = MLMHead(config, self.rt, None)  # untied, like BertOnlyMLMHead built standalone
        self._head_logits = _HeadLogits(self.head)

        modules = [self.embeddings, *self.encoders, self._head_logits]
        self.groups = partition(modules, len(self.group_devices))
        self.devices = []
        for group, dev in zip(self.groups, self.group_devices):
            for m in group:
                m.to(device=dev, dtype=dtype)
                self.devices.append(dev)
        self.tracker = IdleTimeTracker(self.group_devices, timing=timing, verbose=verbose)
        attach_idle_hooks(self.groups, self.tracker)
        self.rng_states = {}
        for dev in set(self.group_devices):
            self.rng_states[str(dev)] = RngState(seed, device=dev)

    # ---- reference attribute names
    @property
    def device_idle_time(self):
        self.tracker.collect()
        return self.tracker.device_idle_time

    @property
    def embedding_device(self):
        return self.devices[0]

    @property
    def encoder_devices(self):
        return self.devices[1:-1]

    @property
    def head_device(self):
        return self.devices[-1]

    def _use_rng_for(self, dev):
        self.rt.rng = self.rng_states[str(dev)]

    def advance_rng(self):
        for r in self.rng_states.values():
            r.advance()

    def _set_micro(self, m: int):
        for r in self.rng_states.values():
            r.micro = m

    def _stage_modules(self):
        stages = []
        for group, dev in zip(self.groups, self.group_devices):
            stages.append(_Stage(group, dev, self))
        return stages

    def to_pipeline(self, chunks: int, checkpoint: str = "except_last") -> GPipe:
        """GPipe over the device groups (reference model/bert_mp.py:73-89, without RPC)."""
        return GPipe(self._stage_modules(), self.group_devices, chunks=chunks, checkpoint=checkpoint,
                     set_micro=self._set_micro, owner=self)

    def forward(self, input_ids: torch.Tensor) -> torch.Tensor:
        x = input_ids
        for stage in self._stage_modules():
            x = stage(send_to(x, stage.device) if x.is_floating_point() else x.to(stage.device))
        return x

    def step_boundary(self):
        self.tracker.step_boundary()


class _Stage(nn.Module):
    """One device group: runs its modules with that device's dropout RNG state."""

    def __init__(self, modules, device, owner: BertModelWithMP):
        super().__init__()
        self.mods = modules          # plain list: parameters stay registered on the owner only
        self.device = torch.device(device)
        self._owner = [owner]

    def forward(self, x):
        owner = self._owner[0]
        owner._use_rng_for(self.device)
        if not x.is_floating_point():
            x = x.to(self.device)
        for m in self.mods:
            x = m(x)
        return x
