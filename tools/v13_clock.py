#!/usr/bin/env python3
"""In-kernel clock and cycles per wave-tile of attn_fwd_v13 under sustained
load (MI355X_MICROARCH.md 'DVFS give-back' item 6), GPU box: >= 2 s of
back-to-back product launches (variant 80) on random bench-config data, then
one stamped launch of the diagnostic build (tools/libpli_diag.so,
attn_fwd_v13_stamp: s_memtime / s_memrealtime at each wave's entry and exit
only) -> clock = sum(dtime) / sum(drealtime) x 100 MHz; cycles per wave-tile
= mean wave cycles / (64 x 64 wave-tiles per wave at B8 H32 S4096 over 256
workgroups = 1024 tiles).  v12 (variant 71) is timed beside it."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "physics-llm-inference_amd"), ROOT]
import pli_hip  # noqa: E402

lib = ctypes.CDLL(os.environ.get("DIAG_LIB") or os.path.join(ROOT, "tools", "libpli_diag.so"))
lib.pli_diag_v13_clock.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int] * 3 + [ctypes.c_void_p]
B, H, N, D = 8, 32, int(os.environ.get("N", "4096")), 128
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn(B, H, N, D, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
o = torch.empty_like(q)
flops = 4 * B * H * N * N * D
for rep in range(3):
    out = {}
    for var in (71, 80):
        t_end = time.perf_counter() + 2.0
        while time.perf_counter() < t_end:
            for _ in range(20):
                pli_hip.flash_attn_fwd(q, k, v, out=o, variant=var)
            torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            pli_hip.flash_attn_fwd(q, k, v, out=o, variant=var)
        e.record()
        e.synchronize()
        ms = s.elapsed_time(e) / 20
        out[f"v{var}_TFLOP/s"] = round(flops / ms / 1e9, 1)
        if var == 80:
            stamps = torch.zeros(256 * 4 * 32, dtype=torch.int32, device="cuda")
            assert lib.pli_diag_v13_clock(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, H, N,
                                          stamps.data_ptr()) == 0
            st = stamps.cpu().numpy().view(np.uint32).reshape(-1, 32)[:, :8].astype(np.uint64)
            t0 = st[:, 0] | (st[:, 1] << 32)
            r0 = st[:, 2] | (st[:, 3] << 32)
            t1 = st[:, 4] | (st[:, 5] << 32)
            r1 = st[:, 6] | (st[:, 7] << 32)
            dt, dr = (t1 - t0).astype(np.float64), (r1 - r0).astype(np.float64)
            ghz = dt.sum() / dr.sum() * 0.1
            tiles = B * H * (N // 64) * (N // 64) / 1024  # wave-tiles per wave (one wave per SIMD)
            out.update({"clock_GHz": round(float(ghz), 3), "cycles_per_wave_tile": round(float(dt.mean() / tiles), 1),
                        "wave_us_mean": round(float(dr.mean() / 100), 1),
                        "wave_us_min_max": [round(float(dr.min() / 100), 1), round(float(dr.max() / 100), 1)]})
            # by XCD (workgroup w runs on XCD w % 8): clock, wave time, and the
            # span from the first wave's start to each XCD's last exit
            wg = np.arange(len(dt)) // 4
            start = float(r0.min())
            xcd = {}
            for x in range(8):
                m = wg % 8 == x
                xcd[x] = {"GHz": round(float(dt[m].sum() / dr[m].sum() * 0.1), 3),
                          "wave_us_mean": round(float(dr[m].mean() / 100), 1),
                          "wave_us_max": round(float(dr[m].max() / 100), 1),
                          "end_us_max": round(float((r1[m].max() - start) / 100), 1)}
            out["by_xcd"] = xcd
            out["span_us"] = round(float((r1.max() - start) / 100), 1)
    print(json.dumps(out), flush=True)
