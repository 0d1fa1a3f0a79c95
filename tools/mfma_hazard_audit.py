#!/usr/bin/env python3
"""Audit inline-asm MFMAs in a gfx950 .s file for unpadded hazards.

hipcc does not model an MFMA written as inline asm (cdna_hip_programming.md
§5.7): it inserts no wait states around it.  This scans every kernel of a
-save-temps assembly file, linearly (fall-through order), and reports:

  * RAW  VALU/VMEM/DS write of a register -> MFMA reading it as A/B/C within
         2 instructions
  * RAW  MFMA dest (D) -> any non-MFMA instruction reading it within
         NPASS+4 instructions (8-pass 32x32x16: 12 wait states)
  * WAW  non-MFMA write of an MFMA dest within the same window
  * WAR  non-MFMA write of an MFMA C (accumulator) operand within the window
  * WAR  non-MFMA write of an MFMA A/B operand within WINDOW_AB states

Branches break the linear order, so this is a heuristic: it is conservative
inside straight-line code (every wait state is counted as one instruction;
s_nop N counts N+1).

    python tools/mfma_hazard_audit.py file.s [kernel-substring]
"""
from __future__ import annotations

import re
import sys

REG = re.compile(r"\b([va])\[(\d+):(\d+)\]|\b([va])(\d+)\b")
WINDOW_D = 12
WINDOW_AB = 8  # A/B operand reads of an 8-pass MFMA assumed spread over its first passes


def regs(tok: str) -> set:
    out = set()
    for m in REG.finditer(tok):
        if m.group(1):
            k, a, b = m.group(1), int(m.group(2)), int(m.group(3))
            out |= {f"{k}{i}" for i in range(a, b + 1)}
        else:
            out.add(f"{m.group(4)}{m.group(5)}")
    return out


def parse(line: str):
    line = line.split(";")[0].strip()
    if not line or line.startswith(".") or line.endswith(":"):
        return None
    parts = line.split(None, 1)
    op = parts[0]
    ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
    return op, ops


def states(op: str, ops) -> int:
    if op == "s_nop":
        return int(ops[0], 0) + 1
    return 1


def audit(lines, name):
    insts, lineno = [], []
    for n, ln in enumerate(lines):
        p = parse(ln)
        if p:
            insts.append(p)
            lineno.append(n + 1)
    issues = []
    for i, (op, ops) in enumerate(insts):
        if not op.startswith("v_mfma") or not ops:
            continue
        d = regs(ops[0])
        srcs = set().union(*(regs(o) for o in ops[1:4])) if len(ops) > 1 else set()
        c = regs(ops[3]) if len(ops) > 3 else set()
        # RAW into the MFMA: producers in the previous 2 wait states
        ws = 0
        for j in range(i - 1, max(-1, i - 8), -1):
            pop, pops = insts[j]
            if ws >= 2:
                break
            if not pop.startswith(("v_", "ds_", "global_load", "buffer_load")) or pop.startswith("v_mfma"):
                ws += states(pop, pops)
                continue
            w = regs(pops[0]) if pops else set()
            if pop.startswith(("ds_write", "global_store", "buffer_store")):
                w = set()
            if w & srcs:
                issues.append((i, f"RAW {pop} -> {op} ({sorted(w & srcs)[:3]}) {ws} states"))
            ws += states(pop, pops)
        # after the MFMA: readers / writers of D, writers of C
        ws = 0
        for j in range(i + 1, len(insts)):
            pop, pops = insts[j]
            if ws >= WINDOW_D:
                break
            if pop.startswith("v_mfma"):
                pd = regs(pops[0])
                psrc = set().union(*(regs(o) for o in pops[1:4]))
                # a dependent MFMA taking D whole as C is the accumulate chain (0 states)
                if (psrc & d) and not (regs(pops[3]) >= d if len(pops) > 3 else False):
                    issues.append((i, f"MFMA D -> MFMA A/B {pop} {ws} states"))
                ws += 1
                continue
            if pop.startswith(("s_", "buffer_", "global_", "scratch_")) and not pop.startswith("s_nop"):
                ws += 1
                continue
            w = regs(pops[0]) if pops and not pop.startswith(("ds_write", "global_store")) else set()
            rd = set().union(*(regs(o) for o in pops[1:])) if len(pops) > 1 else set()
            if pop.startswith(("ds_write",)):
                rd = set().union(*(regs(o) for o in pops))
            if rd & d:
                issues.append((i, f"RAW {op} D -> {pop} ({sorted(rd & d)[:3]}) {ws} states"))
            if w & d:
                issues.append((i, f"WAW {op} D -> {pop} {ws} states"))
            if w & c and not (w & d):
                issues.append((i, f"WAR {op} C <- {pop} {ws} states"))
            ab = set().union(*(regs(o) for o in ops[1:3])) if len(ops) > 2 else set()
            if w & ab and ws < WINDOW_AB:
                issues.append((i, f"WAR {op} A/B <- {pop} ({sorted(w & ab)[:2]}) {ws} states"))
            ws += states(pop, pops)
    for i, msg in issues:
        print(f"{name}: line {lineno[i]} (kernel-relative): {msg}")
    return len(issues)


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    text = open(path).read().splitlines()
    kernels, cur, name = [], [], None
    for ln in text:
        m = re.match(r"^(_Z\S+):", ln)
        if m:
            if name and cur:
                kernels.append((name, cur))
            name, cur = m.group(1), []
            continue
        if name:
            cur.append(ln)
            if "s_endpgm" in ln:
                kernels.append((name, cur))
                name, cur = None, []
    total = 0
    for nm, body in kernels:
        if sub in nm:
            total += audit(body, nm[:60])
    print(f"total issues: {total}")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())
