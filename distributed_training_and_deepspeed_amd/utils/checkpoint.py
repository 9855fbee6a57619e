"""Training checkpoints for the replicated paths (DDP, model/pipeline parallel).

SURVEY.md 5.4: the reference saves nothing (weights come from ``from_pretrained``); this
framework adds save/resume.  ZeRO engines have their own sharded layout
(``parallel/zero.py::ZeroEngine.save_checkpoint``).  Here every rank holds the same state, so
rank 0 writes one file with the module state, the optimizer state (fp32 master + moments for
``FusedAdam``), the step and the step of the device-resident dropout RNG, and every rank loads
it.  The dropout SEED is per rank (trainers reseed by rank so replicas draw independent masks)
and is not in the file: a resumed rank keeps the seed it was started with and continues the
saved step, exactly as if the run had not been interrupted.
Loading uses ``torch.load(weights_only=True)`` only.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def _cpu(obj):
    if torch.is_tensor(obj):
        return obj.detach().to("cpu", copy=True)
    if isinstance(obj, dict):
        return {k: _cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_cpu(v) for v in obj)
    return obj


def _rank() -> int:
    return dist.get_rank() if dist.is_initialized() else 0


def save_checkpoint(path: str, model: torch.nn.Module, optimizer=None, step: int = 0, extra: dict | None = None) -> str:
    """Rank 0 writes ``path`` (a file); all ranks return after the write completed."""
    if optimizer is not None and hasattr(optimizer, "synchronize"):
        optimizer.synchronize()   # a staged update (overlap_with_forward) may still be writing weights
    if _rank() == 0:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        rt = getattr(model, "rt", None)
        state = {"module": _cpu(model.state_dict()), "step": int(step), "extra": extra or {},
                 "optimizer": _cpu(optimizer.state_dict()) if optimizer is not None and hasattr(optimizer, "state_dict")
                 else None,
                 # only the step of the dropout stream: every rank keeps its own seed (DDP
                 # trainers reseed per rank so replicas draw independent masks)
                 "dropout_step": int(rt.rng.state[1].item()) if rt is not None else None}
        tmp = path + ".tmp"
        torch.save(state, tmp)
        os.replace(tmp, path)                  # never leave a half-written checkpoint behind
    if dist.is_initialized():
        dist.barrier()
    return path


@torch.no_grad()
def load_checkpoint(path: str, model: torch.nn.Module, optimizer=None) -> dict:
    """Restore module (+ optimizer, dropout RNG); returns {'step', 'extra'}."""
    state = torch.load(path, map_location="cpu", weights_only=True)
    if optimizer is not None and hasattr(optimizer, "synchronize"):
        optimizer.synchronize()
    model.load_state_dict(state["module"])
    if optimizer is not None and state.get("optimizer") is not None:
        optimizer.load_state_dict(state["optimizer"])
    rt = getattr(model, "rt", None)
    step = state.get("dropout_step")
    if step is None and state.get("dropout_rng") is not None:
        # checkpoints written before the key change kept the whole [seed, step] state
        step = int(torch.as_tensor(state["dropout_rng"]).reshape(-1)[1])
    if rt is not None and step is not None:
        rt.rng.state[1:2].fill_(int(step))   # this rank's seed stays as it is
    return {"step": state["step"], "extra": state["extra"]}
