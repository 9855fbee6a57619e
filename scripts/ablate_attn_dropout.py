#!/usr/bin/env python
"""Ablation (not a valid benchmark configuration): bench.py with attention-probability dropout
disabled, to price the dropout machinery (mask generation + keep-bit application)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from distributed_training_and_deepspeed_amd import models  # noqa: E402
from distributed_training_and_deepspeed_amd.models import config as C  # noqa: E402

_orig = C.get_config


def _no_attn_drop(name):
    return _orig(name).with_(attn_dropout=0.0)


models.get_config = _no_attn_drop      # build_model() looks the preset up through this name
bench.main()
