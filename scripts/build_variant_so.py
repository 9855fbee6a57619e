#!/usr/bin/env python
"""Build an alternative kernel library for same-box A/B runs (scripts/ab.py base_so, loaded through
DTD_KERNELS_SO): every ops/csrc + comm/csrc source compiled with extra hipcc flags into its own
object directory, linked as ops/_dtd_kernels_<name>.so.

    python scripts/build_variant_so.py dmabuiltin -DDTD_DMA_BUILTIN
"""
import os
import sys
from pathlib import Path

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_and_deepspeed_amd.ops import build as B  # noqa: E402


def main():
    name, flags = sys.argv[1], sys.argv[2:]
    B.OBJ_DIR = B.HERE / f"build_{name}"
    B.LIB_PATH = B.HERE / f"_dtd_kernels_{name}.so"
    os.environ["DTD_HIPCC_FLAGS"] = " ".join(flags)
    print(B._build_locked(force=True, jobs=None, verbose=True))


if __name__ == "__main__":
    main()
