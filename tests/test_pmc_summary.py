"""The PMC summary pipeline behind bench.py's roofline fields (CPU, no
GPU): tools/pmc_summary.py on synthetic rocprofv3 counter CSVs -- kernel
labels (gemm_w5 NN vs NT by its first template flag, v13 vs v13c), HBM bytes
(FETCH_SIZE KiB x 1024 x 2 on gfx950 + WRITE_SIZE KiB x 1024), MFMA busy
(SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)) and the
pass clock -- and bench.pmc_fields' unprofiled clock from a live kernel time."""
from __future__ import annotations

import csv
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

COLS = ["Correlation_Id", "Dispatch_Id", "Grid_Size", "Kernel_Name", "Counter_Name", "Counter_Value",
        "Start_Timestamp", "End_Timestamp"]
KERNELS = {  # name -> (grid, duration ns)
    "void pli::(anonymous namespace)::gemm_w5<pli::bf16_t, false, false, true, false, false>(...)": (65536, 100_000),
    "void pli::(anonymous namespace)::gemm_w5<pli::bf16_t, true, false, true, false, false>(...)": (65536, 98_000),
    "pli::(anonymous namespace)::attn_fwd_v13(pli::(anonymous namespace)::V13Args)": (65536, 1_600_000),
    "pli::(anonymous namespace)::attn_fwd_v13c(pli::(anonymous namespace)::V13Args)": (65536, 900_000),
}


def write_pass(d, tag, counters):
    os.makedirs(os.path.join(d, f"pmc_{tag}"), exist_ok=True)
    with open(os.path.join(d, f"pmc_{tag}", "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, COLS)
        w.writeheader()
        cid = 0
        for name, (grid, dur) in KERNELS.items():
            for rep in range(2):
                cid += 1
                for cname, val in counters(name, dur).items():
                    w.writerow({"Correlation_Id": cid, "Dispatch_Id": cid, "Grid_Size": grid, "Kernel_Name": name,
                                "Counter_Name": cname, "Counter_Value": val, "Start_Timestamp": 1000,
                                "End_Timestamp": 1000 + dur})


@pytest.fixture(scope="module")
def summary(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("pmc"))
    write_pass(d, "FETCH_SIZE", lambda n, t: {"FETCH_SIZE": 1000.0 + len(n)})
    write_pass(d, "WRITE_SIZE", lambda n, t: {"WRITE_SIZE": 500.0})
    # 2 GHz: GRBM_GUI_ACTIVE (summed over 8 XCDs) = 8 x 2 x ns; MFMA busy 0.75
    write_pass(d, "SQ", lambda n, t: {"GRBM_GUI_ACTIVE": 16.0 * t, "SQ_VALU_MFMA_BUSY_CYCLES": 0.75 * 1024 * 2.0 * t,
                                      "SQ_WAVES": 1024, "SQ_INSTS_MFMA": 8.0})
    out = os.path.join(d, "traffic.json")
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), d, out], check=True,
                   capture_output=True)
    return json.load(open(out))


def test_labels(summary):
    assert {"gemm_w5 nn", "gemm_w5 nt", "attn_fwd_v13", "attn_fwd_v13c"} <= set(summary)


def test_bytes(summary):
    name = next(n for n in KERNELS if "attn_fwd_v13(" in n)
    e = summary["attn_fwd_v13"]
    assert e["read_bytes_per_launch"] == (1000.0 + len(name)) * 1024 * 2
    assert e["hbm_bytes_per_launch"] == e["read_bytes_per_launch"] + 500.0 * 1024


@pytest.mark.parametrize("k", ["gemm_w5 nn", "attn_fwd_v13", "attn_fwd_v13c"])
def test_busy_and_clock(summary, k):
    e = summary[k]
    assert e["mfma_busy"] == pytest.approx(0.75)
    assert e["clock_GHz"] == pytest.approx(2.0)


def test_bench_implied_clock(summary, monkeypatch):
    """busy cycles per SIMD / busy / kernel time: a live kernel 10 % slower
    than the profiled one at the same cycles reads a 10 % lower clock"""
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.setattr(bench, "load_pmc", lambda kernel: summary[kernel])
    f = bench.pmc_fields("attn_fwd_v13", kernel_ms=1.6 * 1.1)
    assert f["mfma_busy"] == pytest.approx(0.75)
    assert f["implied_clock_GHz"] == pytest.approx(2.0 / 1.1)
