#!/usr/bin/env python3
"""Per-launch HBM bytes of the hot-path kernels from rocprofv3 PMC passes.

    python tools/pmc_summary.py <dir with pmc_FETCH_SIZE*/ pmc_WRITE_SIZE* csv> [out.json]

FETCH_SIZE and WRITE_SIZE are collected in separate passes (they do not fit
one TCC pass).  Both are in KiB per dispatch.  gfx950 tallies 128-B fabric
read requests at 64 B, so FETCH_SIZE is doubled (MI355X_MICROARCH.md, HBM);
WRITE_SIZE is exact for 16-B-per-lane streaming stores.  Infinity-Cache
hits are counted as fetches, so a kernel whose inputs fit the 256 MiB cache
can read back more than HBM actually served.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

KERNELS = ("gemm_w5", "attn_fwd_v13hc_d64", "attn_fwd_v13h_d64", "attn_fwd_v13c_d64", "attn_fwd_v13_d64",
           "attn_fwd_v13hc", "attn_fwd_v13h", "attn_fwd_v13c", "attn_fwd_v13", "attn_fwd_v12", "attn_fwd_v10", "attn_fwd_v7", "gemm_f32_mfma", "gemm_naive_f32", "hbm_read_probe", "attn_fwd_v2", "attn_decode_chunk", "attn_decode_combine", "gemv_vec", "gemm_mfma",
           "gemm_smallm_nt", "scale_copy_vec", "Cijk_")


def label(k: str, name: str) -> str:
    """Causal instantiations (template flag ``true``) share the name prefix
    with the non-causal kernel; keep them apart."""
    if k == "gemm_w5":  # gemm_w5<T, TRANS_B, BIAS, ...>: NT and NN apart by the first flag
        m = re.search(r"gemm_w5<[^,<>]+, (true|false)", name)
        return k + (" nt" if m and m.group(1) == "true" else " nn")
    if k.startswith("attn_fwd_v13"):
        return k
    if k == "Cijk_":  # hipBLASLt (torch F.linear / mm), for comparison
        return "hipblaslt " + name.split("_MT")[1].split("_")[0] if "_MT" in name else "hipblaslt"
    return k + " causal" if k.startswith("attn_fwd") and ", true>" in name else k


def kernel_label(name: str):
    for k in KERNELS:
        if k in name:
            return label(k, name)
    return None


def per_kernel(path_glob: str, counter: str) -> dict:
    """{(kernel, grid_size): [values]}"""
    vals = defaultdict(list)
    for path in glob.glob(path_glob, recursive=True):
        with open(path, newline="") as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                lab = kernel_label(row["Kernel_Name"])
                if lab:
                    vals[(lab, int(row["Grid_Size"]))].append(float(row["Counter_Value"]))
    return vals


def per_kernel_with_time(d: str, counter: str) -> dict:
    """{(kernel, grid): [(value, duration_ns)]} from a pass directory holding
    counter_collection.csv and kernel_trace.csv (joined on Correlation_Id;
    without a trace, the counter row's own dispatch timestamps)"""
    out = defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        dur = {}
        for tp in glob.glob(os.path.join(os.path.dirname(path), "*kernel_trace.csv")):
            with open(tp, newline="") as f:
                for row in csv.DictReader(f):
                    try:
                        dur[row["Correlation_Id"]] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
                    except (KeyError, ValueError):
                        pass
        with open(path, newline="") as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                lab = kernel_label(row["Kernel_Name"])
                if lab:
                    t = dur.get(row.get("Correlation_Id"))
                    if t is None and row.get("End_Timestamp") and row.get("Start_Timestamp"):
                        # rocprofv3 7.x also stamps the dispatch in the counter rows
                        t = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
                    out[(lab, int(row["Grid_Size"]))].append((float(row["Counter_Value"]), t))
    return out


SQ = ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CU_CYCLES", "SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_INSTS_LDS",
      "SQ_LDS_BANK_CONFLICT", "SQ_WAVES", "GRBM_GUI_ACTIVE")
N_SIMD = 1024  # 256 CUs x 4


def main():
    d = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(d, "traffic.json")
    fetch = per_kernel(os.path.join(d, "pmc_FETCH_SIZE*", "**", "*counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(d, "pmc_WRITE_SIZE*", "**", "*counter_collection.csv"), "WRITE_SIZE")
    res = {}
    mean = lambda v: sum(v) / len(v) if v else 0.0  # noqa: E731
    labels = sorted({kk for (kk, _) in set(fetch) | set(write)})
    for k in labels:
        grids = sorted({g for (kk, g) in set(fetch) | set(write) if kk == k})
        if not grids:
            continue
        by_grid = {}
        for g in grids:
            rd = mean(fetch.get((k, g), [])) * 1024 * 2
            wr = mean(write.get((k, g), [])) * 1024
            by_grid[str(g)] = {"read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                               "hbm_bytes_per_launch": rd + wr,
                               "dispatches": len(fetch.get((k, g), []))}
        # headline entry: the grid dispatched most often (the benchmarked shape)
        main_g = max(grids, key=lambda g: len(fetch.get((k, g), [])))
        res[k] = dict(by_grid[str(main_g)], grid_size=main_g, by_grid=by_grid,
                      note="FETCH_SIZE KiB x1024 x2 (gfx950 half-count), WRITE_SIZE KiB x1024; "
                           "mean over dispatches of that grid")
    # the SQ pass: instruction counts, MFMA busy, LDS conflicts, clock
    sq = {c: per_kernel_with_time(os.path.join(d, "pmc_SQ*"), c) for c in SQ}
    for (k, g) in sorted(set(sq["GRBM_GUI_ACTIVE"]) | set(sq["SQ_VALU_MFMA_BUSY_CYCLES"])):
        if k in res and res[k].get("grid_size") not in (None, g):
            continue
        ent = res.setdefault(k, {"grid_size": g})
        for c in SQ:
            vals = [v for v, _ in sq[c].get((k, g), [])]
            if vals:
                ent[c] = mean(vals)
        grbm = sq["GRBM_GUI_ACTIVE"].get((k, g), [])
        if ent.get("GRBM_GUI_ACTIVE") and ent.get("SQ_VALU_MFMA_BUSY_CYCLES") is not None:
            ent["mfma_busy"] = ent["SQ_VALU_MFMA_BUSY_CYCLES"] / (N_SIMD * ent["GRBM_GUI_ACTIVE"] / 8)
            # per-SIMD MFMA busy cycles per launch: with a live kernel time the
            # bench turns this into the unprofiled clock (busy is a cycle ratio)
            ent["mfma_busy_cycles_per_simd"] = ent["SQ_VALU_MFMA_BUSY_CYCLES"] / N_SIMD
        durs = [t for _, t in grbm if t]
        if durs and ent.get("GRBM_GUI_ACTIVE") and mean(durs) >= 1e5:  # (short launches: dispatch dominates)
            ent["duration_ns_pmc"] = mean(durs)
            ent["clock_GHz"] = ent["GRBM_GUI_ACTIVE"] / 8 / mean(durs)
        ent["sq_note"] = ("SQ pass (one rocprofv3 --pmc run): means over dispatches; mfma_busy = "
                          "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8); clock = "
                          "GRBM_GUI_ACTIVE / 8 / kernel-trace duration (counters slow the clock: compare fractions)")
    with open(out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
