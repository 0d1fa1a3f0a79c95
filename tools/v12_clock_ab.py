#!/usr/bin/env python3
"""In-kernel clock of timing-only attn_fwd_v12 builds (GPU box): for each
diagnostic library in $DIAG_LIBS, >= 2 s of back-to-back clock-stamped
launches of that same build (attn_fwd_v12<STAMP 2>: s_memtime /
s_memrealtime at each wave's entry and exit only, persistent grid of 256) on
random bench-config data, then the last launch's clock and cycles per
wave-tile.  Libraries interleaved over $ROUNDS rounds (rule 24)."""
import ctypes
import json
import os
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBS = os.environ["DIAG_LIBS"].split()
ROUNDS = int(os.environ.get("ROUNDS", "2"))
B, H, N, D = 8, 32, 4096, 128
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn(B, H, N, D, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
o = torch.empty_like(q)
fns = []
for p in LIBS:
    lib = ctypes.CDLL(os.path.join(ROOT, p))
    f = lib.pli_diag_v12_stamps
    f.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int] * 3 + [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int,
                                                                 ctypes.c_int]
    fns.append(f)
wave_tiles_per_simd = (B * H * (N // 64) * (N // 64)) / 1024
for rnd in range(ROUNDS):
    for p, f in zip(LIBS, fns):
        buf = (ctypes.c_ulonglong * 24)()
        t_end = time.perf_counter() + 2.0
        n = 0
        while time.perf_counter() < t_end:
            assert f(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, H, N, buf, 256, 2) == 0
            n += 1
        dt, dr, waves = buf[0], buf[1], buf[23]
        ghz = dt / dr * 0.1
        wave_us = dr / waves / 100.0
        cyc = ghz * 1e3 * wave_us / wave_tiles_per_simd
        print(json.dumps({"lib": os.path.basename(p), "round": rnd, "launches": n, "clock_GHz": round(ghz, 4),
                          "wave_lifetime_us": round(wave_us, 1), "cycles_per_wave_tile": round(cyc, 1),
                          "TFLOP/s_from_wave_lifetime": round(4 * B * H * N * N * D / (wave_us * 1e-6) / 1e12, 1)}),
              flush=True)
