#!/usr/bin/env python3
"""Cross-check bench.py's event-timed flash kernel_ms against the rocprofv3
kernel trace of the same run.

    python tools/trace_check.py <run_kernel_trace.csv> <bench json> [warmup] [steps]

bench.py launches `warmup` then `steps` non-causal flash steps first (the
timed region), then the causal extras with the same kernel instantiation, so
the stats file's single average mixes both; this takes the timed dispatches
by launch order.
"""
import csv
import json
import sys

trace, bench = sys.argv[1], sys.argv[2]
warmup = int(sys.argv[3]) if len(sys.argv) > 3 else 2
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 10
kname = sys.argv[5] if len(sys.argv) > 5 else "attn_fwd_v12"
rows = sorted((r for r in csv.DictReader(open(trace)) if kname in r["Kernel_Name"]),
              key=lambda r: int(r["Start_Timestamp"]))
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
timed = dur[warmup:warmup + steps]
b = json.load(open(bench))
k_ms = b["roofline"]["kernel_ms"]
mean_us = sum(timed) / len(timed)
print(json.dumps({"kernel": rows[0]["Kernel_Name"][:90], "dispatches": len(dur),
                  "timed_dispatch_us": [round(x, 1) for x in timed],
                  "rocprof_mean_us_timed": mean_us, "bench_event_kernel_us": k_ms * 1e3,
                  "rel_diff": (k_ms * 1e3 - mean_us) / mean_us}, indent=1))
