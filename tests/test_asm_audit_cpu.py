"""ISA audit of the inline-asm MFMAs of the fused attention backward (ops/csrc/attention.hip):
no instruction touches an MFMA's result registers before its passes are done (hipcc does not
pad hazards of asm statements; scripts/diag/audit_fused_bwd_asm.py).  The audit itself is checked
on a synthetic listing with one early read.  Compiles attention.hip for gfx950 (CPU-only)."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts", "diag"))
from audit_fused_bwd_asm import audit, build_asm  # noqa: E402


def test_audit_flags_an_early_accumulator_read():
    listing = """_ZN12_GLOBAL__N_121attn_bwd_fused_kernelILi4ELb0EEEvNS_7BwdArgsE:
\tv_mfma_f32_32x32x16_bf16 a[0:15], v[2:5], v[6:9], a[0:15]
\ts_nop 3
\tv_accvgpr_read_b32 v10, a15
\tv_mfma_f32_32x32x16_bf16 a[16:31], v[2:5], v[6:9], a[16:31]
\ts_nop 11
\tv_accvgpr_read_b32 v11, a31
.Lfunc_end0:
"""
    probs = audit(listing)
    assert len(probs) == 1 and "a15" in probs[0]


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") and shutil.which("hipcc") is None,
                    reason="hipcc not available")
def test_fused_backward_asm_mfma_results_are_waited_out():
    text = build_asm(os.path.join(ROOT, "distributed_training_and_deepspeed_amd", "ops", "csrc", "attention.hip"))
    assert "attn_bwd_fused_kernel" in text
    assert audit(text) == []
