"""Static view of the generated v13 program: per hot section (between two
labels) the MFMA count, the fillers per gap and a cycle estimate from the
issue costs of MI355X_MICROARCH.md ('vector-instruction ISSUE cost': VALU 4,
transcendental 8, s_nop 4 per instruction + 1 per extra wait state, an MFMA
16 cycles of which 8 hold the issue port)."""
from __future__ import annotations

import sys

from .isa import finalize
from .kernel import Gen

COST = {"valu": 4, "trans": 8, "accw": 4, "ds": 2, "dma": 12, "vmload": 4, "vmstore": 4, "salu": 2,
        "branch": 2, "wait": 2, "barrier": 4, "smem": 2}


def cost(ins):
    k = ins.kind()
    if k == "nop":
        return 4 + int(ins.ops[0])
    return COST.get(k, 0)


def sections(prog):
    cur, name = [], "start"
    for ins in prog:
        if ins.op == "label":
            yield name, cur
            cur, name = [], ins.ops[0]
        else:
            cur.append(ins)
    yield name, cur


def estimate(seq):
    t, gap, nm = 0.0, 0.0, 0
    gaps = []
    for ins in seq:
        if ins.kind() == "mfma":
            if nm:
                gaps.append(gap)
                t += max(16, 8 + gap)
            nm += 1
            gap = 0.0
        else:
            gap += cost(ins)
    if nm:
        gaps.append(gap)
        t += max(16, 8 + gap)
    else:
        t = gap
    return nm, t, gaps


def main(argv):
    kw = {}
    for a in argv:
        k, v = a.split("=")
        kw[k] = int(v)
    prog, st = finalize(Gen(tag="r", **kw).build())
    print(st)
    for name, seq in sections(prog):
        nm, t, gaps = estimate(seq)
        nops = sum(int(i.ops[0]) + 1 for i in seq if i.op == "s_nop")
        waits = sum(1 for i in seq if i.op == "s_waitcnt")
        over = sum(max(0, g - 8) for g in gaps)
        print(f"{name:28s} mfma {nm:3d} instrs {len(seq):5d} est {t:7.0f} cyc  overflow {over:5.0f}  "
              f"nop-ws {nops:3d} waits {waits:2d}")


if __name__ == "__main__":
    main(sys.argv[1:])


def dump(label_name, kw=None):
    prog, _ = finalize(Gen(tag="r", **(kw or {})).build())
    on = False
    k = -1
    line = []
    for ins in prog:
        if ins.op == "label":
            if on:
                break
            on = ins.ops[0] == label_name
            continue
        if not on:
            continue
        if ins.kind() == "mfma":
            if line:
                print(f"{k:3d} [{sum(cost(i) for i in line):3d}] " + " | ".join(i.text()[:38] for i in line))
            k += 1
            line = []
        else:
            line.append(ins)
    print(f"{k:3d} [{sum(cost(i) for i in line):3d}] " + " | ".join(i.text()[:38] for i in line))
