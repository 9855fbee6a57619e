"""ISA audit of ops/csrc/gemm_w4.hip (scripts/diag/audit_w4_asm.py): M0 untouched outside the
LDS-DMA statements, no early access to an asm fragment read's registers, two wait states behind
every epilogue store, MFMA results waited out.  The audit itself is checked on synthetic listings
with one violation each.  Compiles gemm_w4.hip for gfx950 (CPU-only)."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts", "diag"))
from audit_w4_asm import SRC, audit  # noqa: E402

HEAD = "_ZN12_GLOBAL__N_114gemm_w4_kernelILi0EEEvNS_6W4ArgsE:\n"
TAIL = ".Lfunc_end0:\n"


def _asm(*lines):
    return "".join(f"\t;;#ASMSTART\n\t{ln}\n\t;;#ASMEND\n" for ln in lines)


def test_audit_flags_store_data_rewritten_next():
    body = _asm("buffer_store_dwordx4 v[4:7], v1, s[8:11], s2 offen") + "\tv_accvgpr_read_b32 v4, a0\n"
    probs = audit(HEAD + body + TAIL)
    assert len(probs) == 1 and "buffer_store_dwordx4" in probs[0]
    ok = _asm("buffer_store_dwordx4 v[4:7], v1, s[8:11], s2 offen", "s_nop 1") + "\tv_accvgpr_read_b32 v4, a0\n"
    assert audit(HEAD + ok + TAIL) == []


def test_audit_flags_m0_use_outside_dma():
    body = _asm("s_mov_b32 m0, s4", "s_nop 0", "buffer_load_dwordx4 v1, s[8:11], s2 offen lds") + \
        "\ts_mov_b32 s5, m0\n"
    probs = audit(HEAD + body + TAIL)
    assert len(probs) == 1 and "M0" in probs[0]


def test_audit_flags_early_copy_of_a_fragment_read():
    body = _asm("ds_read_b128 v[8:11], v2 offset:0") + "\tv_mov_b32_e32 v20, v9\n" + _asm("s_waitcnt lgkmcnt(0)")
    probs = audit(HEAD + body + TAIL)
    assert len(probs) == 1 and "before its lgkmcnt wait" in probs[0]
    ok = _asm("ds_read_b128 v[8:11], v2 offset:0",
              "v_mfma_f32_16x16x32_bf16 a[0:3], v[12:15], v[16:19], a[0:3]", "s_waitcnt lgkmcnt(0)") + \
        "\tv_mov_b32_e32 v20, v9\n"
    assert audit(HEAD + ok + TAIL) == []


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") and shutil.which("hipcc") is None,
                    reason="hipcc not available")
def test_gemm_w4_kernels_pass_the_audit():
    from audit_fused_bwd_asm import build_asm
    text = build_asm(SRC, ())
    assert text.count("gemm_w4_kernel") >= 2
    assert audit(text) == []
