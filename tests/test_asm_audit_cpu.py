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
    text = build_asm(os.path.join(ROOT, "distributed_training_and_deepspeed_amd", "ops", "csrc", "attention.hip"),
                     ["-DDTD_ATTN_FUSED_BWD=1"])
    assert "attn_bwd_fused_kernel" in text
    assert audit(text) == []


def test_path_audit_follows_branches():
    """The control-flow-aware audit (scripts/diag/audit_mfma_hazards.py) follows a taken branch to
    an early read that the straight-line walk would not reach."""
    from audit_mfma_hazards import audit as audit_paths
    listing = """_Z3fooi:
\tv_mfma_f32_32x32x16_bf16 a[0:15], v[0:3], v[4:7], a[0:15]
\ts_cmp_eq_u32 s0, 1
\ts_cbranch_scc1 .LBB0_2
\ts_nop 15
\tv_accvgpr_read_b32 v8, a3
.LBB0_2:
\ts_nop 3
\tv_accvgpr_read_b32 v9, a5
\ts_endpgm
.Lfunc_end0:
"""
    probs = audit_paths(listing, "foo")
    assert len(probs) == 1 and "a5" in probs[0]


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") and shutil.which("hipcc") is None,
                    reason="hipcc not available")
def test_gemm_ln_asm_mfma_results_are_waited_out():
    """The fused projection + LayerNorm kernel issues its 384-accumulator MFMAs as asm (tiles pinned
    to AGPRs / VGPRs): every path from each MFMA -- loop back-edge, loop exit into the epilogue --
    waits its results out."""
    from audit_mfma_hazards import audit as audit_paths
    text = build_asm(os.path.join(ROOT, "distributed_training_and_deepspeed_amd", "ops", "csrc", "gemm_ln.hip"),
                     ["-DDTD_GEMM_LN_BUILD=1"])
    assert "gemm_ln_kernel" in text
    assert audit_paths(text, "gemm_ln_kernel") == []
