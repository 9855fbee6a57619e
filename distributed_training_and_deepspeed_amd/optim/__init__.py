"""Optimizers.  ``FusedAdam`` is the single-kernel flat-buffer Adam/AdamW; the factories
reproduce the optimizer configuration each reference script uses."""
from .fused_adam import FusedAdam, adam_reference_  # noqa: F401


def hf_adamw(params, lr: float = 5e-5, **kw) -> FusedAdam:
    """transformers.AdamW defaults (data_parallel_training.py:34): eps 1e-6, wd 0, bias correction
    with the eps added before the bias-correction rescale."""
    return FusedAdam(params, lr=lr, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.0, adam_w_mode=True,
                     hf_eps=True, **kw)


def torch_adamw(params, lr: float = 5e-5, **kw) -> FusedAdam:
    """torch.optim.AdamW defaults (model_parallel_training.py:50): eps 1e-8, wd 0.01."""
    return FusedAdam(params, lr=lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01, adam_w_mode=True, **kw)


def deepspeed_adam(params, lr: float = 1.5e-4, **kw) -> FusedAdam:
    """DeepSpeed "Adam" -> FusedAdam(adam_w_mode=True) defaults (zero_dp_training.py:28-33)."""
    return FusedAdam(params, lr=lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, adam_w_mode=True, **kw)


class PerDeviceOptimizer:
    """One fused optimizer per device for models spread over several GPUs (model/pipeline
    parallelism): each device's parameters live in their own flat buffers."""

    def __init__(self, params, factory, **kw):
        groups = {}
        for p in params:
            if p.requires_grad:
                groups.setdefault(str(p.device), []).append(p)
        self.optimizers = [factory(ps, **kw) for ps in groups.values()]

    @property
    def param_groups(self):
        return [g for o in self.optimizers for g in o.param_groups]

    def step(self, closure=None):
        for o in self.optimizers:
            o.step()

    def zero_grad(self, set_to_none: bool = True):
        for o in self.optimizers:
            o.zero_grad(set_to_none)
