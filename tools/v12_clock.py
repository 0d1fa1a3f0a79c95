#!/usr/bin/env python3
"""In-kernel clock of attn_fwd_v12 (the flash default) under sustained load
(MI355X_MICROARCH.md 'DVFS give-back' item 6; cdna_hip_programming.md rule 28),
GPU box: >= 2 s of back-to-back product launches (libpli_hip.so, variant 71) on
random bench-config data, then the diagnostic build's clock-stamped launch
(tools/libpli_diag.so, attn_fwd_v12<STAMP 2>: s_memtime / s_memrealtime at each
wave's entry and exit only) -> clock = sum(dtime) / sum(drealtime) x 100 MHz.
Splits the kernel's TFLOP/s into cycles per wave-tile x clock.  The MFMA
probe's clocks (both shapes) are measured in the same process for reference."""
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "physics-llm-inference_amd"), ROOT]
import pli_hip  # noqa: E402
from ch03.roofline import measure_mfma_peak_detail  # noqa: E402

lib = ctypes.CDLL(os.environ.get("DIAG_LIB") or os.path.join(ROOT, "tools", "libpli_diag.so"))
lib.pli_diag_v12_stamps.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int] * 3 + [
    ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int, ctypes.c_int]
B, H, N, D = 8, 32, 4096, 128
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn(B, H, N, D, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
o = torch.empty_like(q)
flops = 4 * B * H * N * N * D
res = {}
for rep in range(2):
    t_end = time.perf_counter() + 2.5
    while time.perf_counter() < t_end:
        for _ in range(20):
            pli_hip.flash_attn_fwd(q, k, v, out=o)
        torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        pli_hip.flash_attn_fwd(q, k, v, out=o)
    e.record()
    e.synchronize()
    ms = s.elapsed_time(e) / 20
    buf = (ctypes.c_ulonglong * 24)()
    assert lib.pli_diag_v12_stamps(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, H, N, buf, 256, 2) == 0
    dt, dr, tiles, waves = buf[0], buf[1], buf[22], buf[23]
    ghz = dt / dr * 0.1
    per_wave_us = dr / waves / 100.0
    # every SIMD runs one wave; a wave-tile = 64 query rows x 64 keys
    wave_tiles_per_simd = (B * H * (N // 64) * (N // 64)) / 1024
    res[f"rep{rep}"] = {"kernel_ms_events": ms, "TFLOP/s": flops / ms / 1e9, "clock_GHz": ghz,
                        "wave_lifetime_us": per_wave_us,
                        "cycles_per_wave_tile": ghz * ms * 1e6 / wave_tiles_per_simd,
                        "mfma_floor_cycles": 64 * 32 + 8 * 16}
    print(json.dumps(res[f"rep{rep}"]), flush=True)
for shape in ("32x32x16", "16x16x32"):
    res[f"probe_{shape}"] = measure_mfma_peak_detail(shape)
    print(shape, json.dumps(res[f"probe_{shape}"]), flush=True)
print(json.dumps(res))
