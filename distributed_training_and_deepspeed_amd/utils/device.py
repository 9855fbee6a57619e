"""Device discovery and small formatting helpers.

Parity with the reference helpers in ``util.py:6-35`` (``get_device``,
``get_device_count``, ``format_size``).  On this framework the accelerator is an
AMD Instinct MI355X driven through PyTorch-ROCm, which exposes HIP devices under
the ``cuda`` device type; MPS is kept in the priority order for API parity.
"""
from __future__ import annotations

import math
import os

import torch


def get_device() -> str:
    """Return the preferred device type: ``cuda`` (HIP on ROCm) > ``mps`` > ``cpu``.

    Same priority order as the reference ``util.py:8-13``.
    """
    if torch.cuda.is_available():
        return "cuda"
    mps = getattr(torch.backends, "mps", None)
    if mps is not None and mps.is_available():
        return "mps"
    return "cpu"


def get_device_count() -> int:
    """Number of visible accelerators, or 1 when only the CPU is available (``util.py:16-21``)."""
    if torch.cuda.is_available():
        return torch.cuda.device_count()
    return 1


def format_size(size_bytes: float) -> str:
    """1024-based human readable size with two decimals (``util.py:24-35``)."""
    if size_bytes == 0:
        return "0B"
    names = ("B", "KB", "MB", "GB", "TB", "PB", "EB", "ZB", "YB")
    i = int(math.floor(math.log(abs(size_bytes), 1024)))
    i = max(0, min(i, len(names) - 1))
    p = math.pow(1024, i)
    return "%s %s" % (round(size_bytes / p, 2), names[i])


def local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", "0"))


def is_rocm() -> bool:
    return torch.version.hip is not None


def gpu_arch() -> str | None:
    """gfx target of device 0 (``gfx950`` on MI355X), or None without a GPU."""
    if not torch.cuda.is_available():
        return None
    props = torch.cuda.get_device_properties(0)
    name = getattr(props, "gcnArchName", "") or ""
    return name.split(":")[0] or None
