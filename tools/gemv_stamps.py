#!/usr/bin/env python3
"""Anatomy of the 4096 x 4096 bf16 decode GEMV (GPU box, diagnostic build:
tools/build_diag.sh -> tools/libpli_diag.so, tools/diag/gemv_diag.hip).

    python tools/gemv_stamps.py

1. Device time per launch (HIP graph of 24 launches over 24 HBM-resident W
   copies, like bench.py) of the product kernel and of persistent grids,
   with bitwise parity against pli_gemv.
2. One stamped launch per kernel: s_memrealtime (100 MHz) per wave at entry,
   loads returned, exit -> dispatch ramp, first-byte latency, tail."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "physics-llm-inference_amd"), ROOT]
import pli_hip  # noqa: E402

lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libpli_diag.so"))
lib.pli_diag_gemv.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                              ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
M = K = 4096
COPIES = 24
ws = [torch.randn(M, K, device="cuda", dtype=torch.bfloat16) for _ in range(COPIES)]
x = torch.randn(K, device="cuda", dtype=torch.bfloat16)
y = torch.empty(M, device="cuda", dtype=torch.bfloat16)
st = torch.cuda.current_stream()
WPB = {0: 2, 1: 4, 2: 8, 3: 2, 4: 4, 5: 2}


def launch(kind, grid, w, stamps=None):
    rc = lib.pli_diag_gemv(kind, w.data_ptr(), x.data_ptr(), y.data_ptr(), M, K, K, grid,
                           None if stamps is None else stamps.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert rc == 0, rc


def graph_us(fn):
    for w in ws:
        fn(w)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for w in ws:
            fn(w)
    for _ in range(3):
        g.replay()
    best = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            g.replay()
        e.record()
        e.synchronize()
        best.append(s.elapsed_time(e) * 1e3 / (20 * COPIES))
    return float(np.median(best))


configs = [(0, 0)] + [(1, g) for g in (256, 512, 1024)] + [(2, g) for g in (128, 256, 512)] + \
          [(3, g) for g in (512, 1024, 2048)] + [(4, g) for g in (128, 256, 512, 1024)] + \
          [(5, g) for g in (256, 512, 1024, 2048)]
if os.environ.get("GEMV_KINDS"):
    ks = {int(k) for k in os.environ["GEMV_KINDS"].split(",")}
    configs = [c for c in configs if c[0] in ks]
ref = pli_hip.gemv(ws[0], x)
out = {"product_pli_gemv_us": graph_us(lambda w: pli_hip.gemv(w, x, out=y))}
for kind, grid in configs:
    key = f"k{kind}_g{grid}"
    launch(kind, grid, ws[0])
    torch.cuda.synchronize()
    same = bool(torch.equal(y, ref))
    us = graph_us(lambda w: launch(kind, grid, w))
    nw = M if kind == 0 else grid * WPB[kind]
    stamps = torch.zeros(nw * 4, dtype=torch.int64, device="cuda")
    for i in range(6):
        launch(kind, grid, ws[(i * 5) % COPIES], stamps)
    torch.cuda.synchronize()
    t = stamps.view(nw, 4).cpu().numpy().astype(np.int64)
    t0, t1, t2, xcc = t[:, 0], t[:, 1], t[:, 2], t[:, 3]
    base = t0.min()
    r = lambda a: (a - base) * 0.01  # 100 MHz ticks -> us
    start, loaded, end = r(t0), r(t1), r(t2)
    out[key] = {"us": round(us, 3), "GB/s": round(M * K * 2 / us / 1e3, 1), "bitwise_eq_pli_gemv": same,
                "waves": nw,
                "start_us_p50_p90_max": [round(float(np.percentile(start, p)), 2) for p in (50, 90, 100)],
                "first_loaded_us_p10_p50_max": [round(float(np.percentile(loaded - start, p)), 2)
                                                for p in (10, 50, 100)],
                "end_us_p50_p90_max": [round(float(np.percentile(end, p)), 2) for p in (50, 90, 100)],
                "start_by_xcc_us": {int(c): round(float(start[xcc == c].min()), 2) for c in np.unique(xcc)}}
    print(json.dumps({key: out[key]}), flush=True)
print(json.dumps({"product_pli_gemv_us": out["product_pli_gemv_us"]}), flush=True)
