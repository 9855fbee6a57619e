#!/usr/bin/env python
"""ISA audit of hand-issued (inline-asm) MFMAs along every control-flow path.

hipcc takes an asm statement as complete when it ends, but an MFMA writes its result registers
over its passes: any other instruction that reads or writes them too early sees a stale value,
silently (cdna_hip_programming.md §5.7).  For every MFMA of the matched kernels this walks the
successor paths -- fall-through, conditional and unconditional branch targets -- and requires at
least WAIT wait states (s_nop N counts N + 1, any other instruction 1) before the first
instruction that touches the destination, unless that instruction is an MFMA taking the whole
destination as its accumulator (a chain: the hardware interlocks it).

Usage: audit_mfma_hazards.py FILE.s KERNEL_REGEX   (exit status 1 and a listing on a finding)
Used by tests/test_asm_audit_cpu.py on ops/csrc/gemm_ln.hip."""
import re
import sys

WAIT = {"v_mfma_f32_32x32x16_bf16": 12, "v_mfma_f32_16x16x32_bf16": 8}


def regs(text, kind):
    out = set()
    for a, b, c in re.findall(kind + r"\[(\d+):(\d+)\]|\b" + kind + r"(\d+)\b", text):
        if a:
            out |= set(range(int(a), int(b) + 1))
        elif c:
            out.add(int(c))
    return out


def parse(body):
    """(instructions, label -> index): instructions as (op, args) with labels resolved."""
    ins, labels = [], {}
    for ln in body.split("\n"):
        s = ln.split(";")[0].strip()
        if not s or s.startswith("."):
            m = re.match(r"^(\.LBB[\w_]+):", s)
            if m:
                labels[m.group(1)] = len(ins)
            continue
        if s.endswith(":"):
            labels[s[:-1]] = len(ins)
            continue
        tok = s.split(None, 1)
        ins.append((tok[0], tok[1] if len(tok) > 1 else ""))
    return ins, labels


def audit_kernel(name, body):
    ins, labels = parse(body)
    problems = []
    for n, (op, args) in enumerate(ins):
        if op not in WAIT:
            continue
        dst = args.split(",")[0].strip()
        kind = "a" if dst.startswith("a") else "v"
        dregs = regs(dst, kind)
        # depth-first over paths: (index, wait states so far)
        stack, seen = [(n + 1, 0)], set()
        while stack:
            q, waited = stack.pop()
            while q < len(ins) and waited < WAIT[op]:
                if (q, waited) in seen:
                    break
                seen.add((q, waited))
                o, a = ins[q]
                if o == "s_nop":
                    waited += int(a, 0) + 1
                    q += 1
                    continue
                if o.startswith("v_mfma"):
                    parts = [x.strip() for x in a.split(",")]
                    if len(parts) > 3 and regs(parts[0], kind) == dregs and regs(parts[3], kind) == dregs:
                        break                         # accumulate chain
                    if (regs(parts[0], kind) | regs(",".join(parts[1:], ), kind)) & dregs:
                        problems.append(f"{name}: [{n}] {op} {args} -> [{q}] {o} {a} after {waited} wait states")
                        break
                elif regs(a, kind) & dregs:
                    problems.append(f"{name}: [{n}] {op} {args} -> [{q}] {o} {a} after {waited} wait states")
                    break
                waited += 1
                if o == "s_endpgm":
                    break
                if o.startswith("s_cbranch"):
                    t = a.split()[0]
                    if t in labels:
                        stack.append((labels[t], waited))
                elif o == "s_branch":
                    t = a.split()[0]
                    q = labels.get(t, len(ins))
                    continue
                q += 1
    return problems


def audit(asm_text, pattern):
    problems = []
    for m in re.finditer(r"^(_Z\S*" + pattern + r"\S*):", asm_text, re.M):
        body = asm_text[m.end():asm_text.index(".Lfunc_end", m.end())]
        problems += audit_kernel(m.group(1), body)
    return problems


def main():
    text = open(sys.argv[1]).read()
    probs = audit(text, sys.argv[2])
    for p in probs:
        print(p)
    print(f"{len(probs)} early accesses")
    sys.exit(1 if probs else 0)


if __name__ == "__main__":
    main()
