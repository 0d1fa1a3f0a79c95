#!/usr/bin/env python3
"""Per-basic-block instruction mix of one kernel in a hipcc -S listing.

    python tools/asm_stats.py file.s NAME_SUBSTRING [--dump BLOCK]

Prints, for every basic block of the first function whose symbol contains
NAME_SUBSTRING: instruction count, MFMA / VALU / transcendental / LDS /
VMEM / scratch / waitcnt / barrier counts, so a kernel's main loop can be
checked for spills and its VALU-per-MFMA ratio read off without a GPU.
"""
from __future__ import annotations

import re
import sys


def categorize(op: str) -> str:
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("scratch_", "buffer_store_dword off", "buffer_load_dword off")):
        return "scratch"
    if op.startswith(("v_exp", "v_log", "v_rcp", "v_rsq", "v_sqrt", "v_sin", "v_cos")):
        return "trans"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, name = sys.argv[1], sys.argv[2]
    dump = sys.argv[sys.argv.index("--dump") + 1] if "--dump" in sys.argv else None
    text = open(path).read().split("\n")
    start = None
    for i, line in enumerate(text):
        if re.match(r"^\S+:", line) and name in line.split(":")[0] and not line.startswith("."):
            start = i
            break
    if start is None:
        sys.exit(f"no function matching {name}")
    blocks, cur, label = [], [], text[start].split(":")[0][:60]
    for line in text[start + 1:]:
        if line.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\S+):", line) or re.match(r"^; (%bb\.\d+):", line)
        if m:
            blocks.append((label, cur))
            label, cur = m.group(1), []
            continue
        s = line.strip()
        if not s or s.startswith((";", ".")):
            continue
        cur.append(s)
    blocks.append((label, cur))
    cats = ["mfma", "valu", "trans", "lds", "vmem", "scratch", "wait", "barrier", "salu"]
    print(f"{'block':28s} {'n':>5s} " + " ".join(f"{c:>7s}" for c in cats))
    for label, ins in blocks:
        cnt = {c: 0 for c in cats}
        for s in ins:
            c = categorize(s.split()[0] + (" off" if " off" in s and "scratch" not in s else ""))
            if c in cnt:
                cnt[c] += 1
        print(f"{label:28s} {len(ins):5d} " + " ".join(f"{cnt[c]:7d}" for c in cats))
        if dump and label == dump:
            print("\n".join("    " + s for s in ins))


if __name__ == "__main__":
    main()
