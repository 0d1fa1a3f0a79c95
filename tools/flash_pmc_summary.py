#!/usr/bin/env python3
"""Summarise tools/pmc_flash.sh passes: per flash variant (dispatch order =
argv order, PLI_PMC_REPS + 1 launches each, the first one dropped), the mean
counter value per dispatch, the kernel duration, the effective clock
(GRBM_GUI_ACTIVE / 8 XCDs / duration) and the MFMA-busy fraction
(SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x cycles)).

    python tools/flash_pmc_summary.py gpurun_out/fpmc 21 40 44
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root, variants = sys.argv[1], sys.argv[2:]
reps = int(os.environ.get("PLI_PMC_REPS", "3")) + 1
out = {v: defaultdict(list) for v in variants}
for path in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
    rows = defaultdict(lambda: defaultdict(float))
    meta = {}
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            if "attn_fwd" not in r["Kernel_Name"]:
                continue
            d = int(r["Dispatch_Id"])
            rows[d][r["Counter_Name"]] += float(r["Counter_Value"])
            meta[d] = r
    order = sorted(rows)
    for i, d in enumerate(order):
        vi = i // reps
        if vi >= len(variants) or i % reps == 0:
            continue
        for k, val in rows[d].items():
            out[variants[vi]][k].append(val)
for path in sorted(glob.glob(os.path.join(root, "p1", "**", "*kernel_trace.csv"), recursive=True)):
    with open(path, newline="") as f:
        tr = [r for r in csv.DictReader(f) if "attn_fwd" in r["Kernel_Name"]]
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    for i, r in enumerate(tr):
        vi = i // reps
        if vi < len(variants) and i % reps:
            out[variants[vi]]["dur_ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            out[variants[vi]]["kernel"] = r["Kernel_Name"][:90]
res = {}
for v, d in out.items():
    m = {k: (sum(x) / len(x) if isinstance(x, list) and x else x) for k, x in d.items()}
    if m.get("GRBM_GUI_ACTIVE") and m.get("dur_ns"):
        ghz = m["GRBM_GUI_ACTIVE"] / 8 / m["dur_ns"]
        m["clock_GHz_per_xcd"] = ghz
        if m.get("SQ_VALU_MFMA_BUSY_CYCLES"):
            m["mfma_busy_frac"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * m["dur_ns"] * ghz)
        m["TFLOP/s"] = 2 ** 41 / (m["dur_ns"] * 1e-9) / 1e12
    res["v" + v] = m
print(json.dumps(res, indent=1))
