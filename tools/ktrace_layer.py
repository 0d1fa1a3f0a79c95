#!/usr/bin/env python3
"""Per-kernel mean duration over the last N dispatches of a rocprofv3
kernel_trace.csv: python tools/ktrace_layer.py <kernel_trace.csv> [N]."""
import collections
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 400
d = collections.defaultdict(list)
for r in rows[-n:]:
    name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
    key = (name.split("(")[0].replace("void ", "")[:70], r["Grid_Size_X"])
    d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
span = (int(rows[-1]["End_Timestamp"]) - int(rows[-n]["Start_Timestamp"])) / 1e3
for (k, g), v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k:70s} grid={g:>8} n={len(v):4d} mean_us={sum(v) / len(v):7.2f}")
for r in rows[-14:]:
    print("  seq", r["Kernel_Name"][:60], r["Grid_Size_X"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(f"span of the last {n} dispatches: {span:.1f} us")
