#!/usr/bin/env python
"""ISA audit of hand-issued (inline-asm) MFMAs: hipcc takes an asm statement as complete when it
ends, but an MFMA's result registers are written over its passes -- any other instruction that
touches them too early reads (or clobbers) a stale value, silently (cdna_hip_programming.md §5.7).

For every MFMA in the given kernels, the first later instruction that reads or writes its
destination registers -- other than an MFMA taking them whole as its accumulator -- must come at
least WAIT wait states later (s_nop N counts N + 1): 12 for the 8-pass 32x32x16, 8 for the 4-pass
16x16x32 (the distances hipcc itself keeps for its own MFMAs on these kernels).

Usage: audit_fused_bwd_asm.py [file.s]   (default: compile ops/csrc/attention.hip for gfx950)
Exit status 1 and a listing when an early access is found."""
import os
import re
import subprocess
import sys
import tempfile

WAIT = {"v_mfma_f32_32x32x16_bf16": 12, "v_mfma_f32_16x16x32_bf16": 8}
KERNELS = r"attn_bwd_fused_kernel"


def regs(text, kind):
    out = set()
    for a, b, c in re.findall(kind + r"\[(\d+):(\d+)\]|\b" + kind + r"(\d+)\b", text):
        if a:
            out |= set(range(int(a), int(b) + 1))
        elif c:
            out.add(int(c))
    return out


def audit(asm_text: str, pattern: str = KERNELS) -> list[str]:
    problems = []
    for m in re.finditer(r"^(_Z\S*" + pattern + r"\S*):", asm_text, re.M):
        name = m.group(1)
        body = asm_text[m.end():asm_text.index(".Lfunc_end", m.end())]
        lines = [ln.strip() for ln in body.split("\n")]
        lines = [ln for ln in lines if ln and not ln.startswith((";", "."))]
        for n, ln in enumerate(lines):
            op = ln.split()[0]
            if op not in WAIT:
                continue
            dst = ln.split(None, 1)[1].split(",")[0].strip()
            kind = "a" if dst.startswith("a") else "v"
            dregs = regs(dst, kind)
            waited = 0
            for q in range(n + 1, min(n + 80, len(lines))):
                t = lines[q]
                tok = t.split()
                if tok[0] == "s_nop":
                    waited += int(tok[1], 0) + 1
                    continue
                if tok[0].endswith(":") or tok[0].startswith("s_cbranch") or tok[0] == "s_branch":
                    break                      # control flow: not followed
                args = t.split(None, 1)[1] if len(tok) > 1 else ""
                if tok[0].startswith("v_mfma"):
                    parts = [x.strip() for x in args.split(",")]
                    if len(parts) > 3 and regs(parts[3], kind) == dregs and regs(parts[0], kind) == dregs:
                        break                  # accumulate chain: takes the result whole as C
                    if (regs(parts[0], kind) | regs(",".join(parts[1:3]), kind)) & dregs and waited < WAIT[op]:
                        problems.append(f"{name}: {ln} -> {t} after {waited} wait states")
                        break
                    waited += 1
                    continue
                if regs(args, kind) & dregs:
                    if waited < WAIT[op]:
                        problems.append(f"{name}: {ln} -> {t} after {waited} wait states")
                    break
                waited += 1
                if waited >= WAIT[op]:
                    break
    return problems


def build_asm(src: str, defines=("-DDTD_ATTN_FUSED_BWD=1", "-DDTD_GEMM_LN_BUILD=1")) -> str:
    """Device ISA of `src` (the experimental kernels compiled in: they are what is audited)."""
    out = tempfile.NamedTemporaryFile(suffix=".s", delete=False).name
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S",
                    *defines, src, "-o", out], check=True, capture_output=True)
    with open(out) as f:
        text = f.read()
    os.unlink(out)
    return text


def main():
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    if len(sys.argv) > 1:
        text = open(sys.argv[1]).read()
    else:
        text = build_asm(os.path.join(root, "distributed_training_and_deepspeed_amd", "ops", "csrc", "attention.hip"))
    probs = audit(text)
    for p in probs:
        print(p)
    print(f"{len(probs)} early accesses")
    sys.exit(1 if probs else 0)


if __name__ == "__main__":
    main()
