#!/usr/bin/env python
"""ISA audit of gemm_w4.hip (the one-wave-per-SIMD projection GEMM), which issues its MFMAs, LDS
fragment reads, LDS-DMA pieces and epilogue stores as inline asm.  hipcc neither waits out those
statements' hazards nor knows their results land late, so the kernel's correctness rests on
properties of the emitted code that this script checks:

1. m0: the DMA statements write M0 without restoring it, so nothing else in the kernel may read or
   write M0 (every M0 access is an ``s_mov_b32 m0`` immediately followed by ``s_nop`` and an
   ``... lds`` buffer load).
2. LDS fragment reads: between a ``ds_read_b128`` issued by asm and the next ``s_waitcnt
   lgkmcnt``, no instruction other than an MFMA or another fragment read touches its destination
   registers (a compiler copy there would read the registers before the data arrives); likewise
   no instruction touches an asm global load's registers before the next ``s_waitcnt vmcnt``.
3. Epilogue stores: no instruction writes a ``buffer_store_dwordx4``'s data registers within two
   wait states of it (on gfx950 the store then wrote corrupted data: scripts/diag/w4_debug.py).
4. MFMA results: scripts/diag/audit_mfma_hazards.py over the same kernels.

Usage: audit_w4_asm.py [FILE.s]   (default: compile ops/csrc/gemm_w4.hip; exit status 1 on a finding)
"""
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from audit_fused_bwd_asm import build_asm  # noqa: E402
from audit_mfma_hazards import audit as audit_mfma  # noqa: E402
from audit_mfma_hazards import parse, regs  # noqa: E402

SRC = os.path.join(os.path.dirname(os.path.dirname(HERE)), "distributed_training_and_deepspeed_amd", "ops", "csrc",
                   "gemm_w4.hip")


def _vregs(text):
    return regs(text, "v")


def _asm_flags(body):
    """Per instruction of ``parse(body)``: True when it comes from an inline-asm statement."""
    flags, inside = [], False
    for ln in body.split("\n"):
        t = ln.strip()
        if t.startswith(";;#ASMSTART"):
            inside = True
            continue
        if t.startswith(";;#ASMEND"):
            inside = False
            continue
        s = t.split(";")[0].strip()
        if not s or s.startswith(".") or s.endswith(":"):
            continue
        flags.append(inside)
    return flags


def audit_kernel(name, body):
    ins, _ = parse(body)
    from_asm = _asm_flags(body)
    assert len(from_asm) == len(ins), (len(from_asm), len(ins))
    probs = []
    for n, (op, args) in enumerate(ins):
        # 1. m0
        if re.search(r"\bm0\b", args):
            ok = (op == "s_mov_b32" and args.split(",")[0].strip() == "m0" and n + 2 < len(ins)
                  and ins[n + 1][0] == "s_nop" and ins[n + 2][0].startswith("buffer_load") and "lds" in ins[n + 2][1])
            if not ok:
                probs.append(f"{name}: [{n}] {op} {args}: M0 access outside a DMA statement")
        # 2. fragment reads
        if op == "ds_read_b128" and from_asm[n]:
            dst = _vregs(args.split(",")[0])
            for q in range(n + 1, len(ins)):
                o, a = ins[q]
                if o == "s_waitcnt" and "lgkmcnt" in a:
                    break
                if o.startswith("v_mfma") or o == "ds_read_b128" and not (_vregs(a.split(",")[0]) & dst):
                    if o.startswith("v_mfma") and _vregs(a.split(",")[0]) & dst:
                        probs.append(f"{name}: [{n}] ds_read {args} -> [{q}] {o} {a} writes it")
                    continue
                if o.startswith("s_") and not o.startswith("s_waitcnt"):
                    continue
                if _vregs(a) & dst:
                    probs.append(f"{name}: [{n}] ds_read {args} -> [{q}] {o} {a} before its lgkmcnt wait")
                    break
        # 2b. asm global loads (the EPI_ADD residual rows): untouched until a vmcnt wait
        if op == "buffer_load_dwordx4" and from_asm[n] and "lds" not in args:
            dst = _vregs(args.split(",")[0])
            for q in range(n + 1, len(ins)):
                o, a = ins[q]
                if o == "s_waitcnt" and "vmcnt" in a:
                    break
                if o.startswith("s_"):
                    continue
                if o.startswith("buffer_load") and (from_asm[q] or not (_vregs(a.split(",")[0]) & dst)):
                    continue   # another load: a later instance of the same asm prefetch (other code path)
                if _vregs(a) & dst:
                    probs.append(f"{name}: [{n}] {op} {args} -> [{q}] {o} {a} before a vmcnt wait")
                    break
        # 3. store data
        if op == "buffer_store_dwordx4":
            data = _vregs(args.split(",")[0])
            waited, q = 0, n + 1
            while q < len(ins) and waited < 2:
                o, a = ins[q]
                if o == "s_nop":
                    waited += int(a, 0) + 1
                else:
                    dst = _vregs(a.split(",")[0]) if o.startswith("v_") else set()
                    if dst & data:
                        probs.append(f"{name}: [{n}] {op} {args} -> [{q}] {o} {a} after {waited} wait states")
                        break
                    waited += 1
                q += 1
    return probs


def audit(text):
    probs = []
    for m in re.finditer(r"^(_Z\S*gemm_w4_kernel\S*):", text, re.M):
        body = text[m.end():text.index(".Lfunc_end", m.end())]
        probs += audit_kernel(m.group(1), body)
    return probs + audit_mfma(text, "gemm_w4_kernel")


def main():
    text = open(sys.argv[1]).read() if len(sys.argv) > 1 else build_asm(SRC, ())
    probs = audit(text)
    for p in probs:
        print(p)
    n = len(re.findall(r"^_Z\S*gemm_w4_kernel\S*:", text, re.M))
    print(f"{n} kernels, {len(probs)} findings")
    sys.exit(1 if probs or n == 0 else 0)


if __name__ == "__main__":
    main()
