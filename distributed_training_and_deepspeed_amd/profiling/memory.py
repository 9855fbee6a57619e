"""Device-memory reporting (DeepSpeed ``memory_status`` equivalent, zero_dp_training.py:8,92-94).

Prints one ``MEMSTATS`` line with current / delta / peak allocated and reserved (cached)
HBM in GB.  On MI355X this reads the HIP caching allocator through torch.cuda.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

_PREV = {"alloc": 0, "cache": 0}


def memory_status(msg: str = "", print_rank: int = 0, reset_max: bool = False) -> dict | None:
    if dist.is_initialized() and print_rank >= 0 and dist.get_rank() != print_rank:
        return None
    if not torch.cuda.is_available():
        return None
    torch.cuda.synchronize()
    gb = 1024 ** 3
    alloc, cache = torch.cuda.memory_allocated(), torch.cuda.memory_reserved()
    max_alloc, max_cache = torch.cuda.max_memory_allocated(), torch.cuda.max_memory_reserved()
    d_alloc, d_cache = alloc - _PREV["alloc"], cache - _PREV["cache"]
    _PREV.update(alloc=alloc, cache=cache)
    dev = torch.cuda.current_device()
    print(f"MEMSTATS {msg} device={dev} current alloc={alloc / gb:0.4f}GB (delta={d_alloc / gb:0.4f}GB "
          f"max={max_alloc / gb:0.4f}GB) current cache={cache / gb:0.4f}GB (delta={d_cache / gb:0.4f}GB "
          f"max={max_cache / gb:0.4f}GB)")
    if reset_max:
        torch.cuda.reset_peak_memory_stats()
    return {"alloc": alloc, "max_alloc": max_alloc, "cache": cache, "max_cache": max_cache}
