"""Measured GEMM solution selection for hipBLASLt on MI355X (PyTorch TunableOp).

hipBLASLt's heuristic picks one solution per GEMM shape; for the BERT weight-gradient and
projection shapes a measured choice is faster (bench b32: +4% tokens/s).  ``tuning/`` holds a
TunableOp results table produced on an MI355X by

    PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 \
    PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results%d.csv python bench.py --steps 4

The table also carries the small-M shapes of the reference's own defaults (bloom-560m ZeRO at
batch 1, BERT-base DDP at batch 4), tuned the same way through ``zero_dp_training.py`` and
``data_parallel_training.py`` with ``--graph off`` (``scripts/sessions/gpu_r6_tune_refconfigs.sh``).

``use_tuned_gemms()`` loads it with tuning disabled: shapes in the table use the measured
solution, every other shape falls back to the default heuristic (no tuning pauses at run time).
The table's validator rows pin the torch / HIP / hipBLASLt versions it was measured with;
TunableOp ignores it if they do not match.
"""
from __future__ import annotations

import os
from pathlib import Path

import torch

DEFAULT_TABLE = Path(__file__).resolve().parent.parent / "tuning" / "tunableop_mi355x.csv"


def use_tuned_gemms(path: str | os.PathLike | None = None) -> bool:
    if not torch.cuda.is_available() or torch.version.hip is None:
        return False
    path = Path(path or os.environ.get("DTD_TUNED_TABLE") or DEFAULT_TABLE)
    if not path.exists():
        return False
    try:
        import torch.cuda.tunable as tunable
        tunable.enable(True)
        tunable.tuning_enable(False)
        tunable.record_untuned_enable(False)
        return bool(tunable.read_file(str(path)))
    except Exception:  # pragma: no cover - tunable API drift
        return False


def maybe_use_tuned_gemms() -> bool:
    """The entry scripts' call: the measured table unless the run configures TunableOp itself
    (``PYTORCH_TUNABLEOP_ENABLED`` set, e.g. a tuning run) or ``DTD_TUNED_GEMMS=0``."""
    if "PYTORCH_TUNABLEOP_ENABLED" in os.environ or os.environ.get("DTD_TUNED_GEMMS", "1") == "0":
        return False
    return use_tuned_gemms()
