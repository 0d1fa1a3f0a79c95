#!/usr/bin/env python3
"""Cycle anatomy of attn_fwd_w4p from its s_memtime-stamped build (flash
variant 46) at the bench config: per wave, per 64-key tile, the shader cycles
of phase 1 (QK^T || softmax finish), between phases (rescale + hazard pad),
phase 2 (PV || softmax start) and the barrier (vmcnt(0) + s_barrier), plus
prologue / epilogue per wave.  Also times variants 44 and 46 with events."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "physics-llm-inference_amd"), ROOT]
import torch  # noqa: E402

import pli_hip  # noqa: E402

lib = pli_hip.lib()
lib.pli_debug_w4_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
g = torch.Generator(device="cuda").manual_seed(0)
B, H, S, D = 8, 32, 4096, 128
q, k, v = (torch.randn(B, H, S, D, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
o = torch.empty_like(q)
buf = (ctypes.c_ulonglong * 8)()
STAMPED = {46}
for var in [int(a) for a in sys.argv[1:]] or [44, 46]:
    for _ in range(3):
        pli_hip.flash_attn_fwd(q, k, v, out=o, variant=var)
    torch.cuda.synchronize()
    lib.pli_debug_w4_stamps(buf, 1)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        pli_hip.flash_attn_fwd(q, k, v, out=o, variant=var)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 5
    print(f"variant {var}: {ms:.3f} ms  {2**41 / ms / 1e9:.0f} TFLOP/s", flush=True)
    if var in STAMPED:
        lib.pli_debug_w4_stamps(buf, 1)
        w, tiles = buf[6], buf[7]
        names = ["phase1", "between", "phase2", "barrier", "prologue", "epilogue"]
        per_tile = {n: buf[i] / tiles for i, n in enumerate(names[:4])}
        tot = sum(per_tile.values())
        print("  waves", w, "tiles/wave", tiles / w)
        print("  cycles per wave-tile:", {n: round(x) for n, x in per_tile.items()}, "sum", round(tot),
              f"-> {tot / 64:.1f} cyc/MFMA")
        print("  per wave:", {n: round(buf[i] / w) for i, n in enumerate(names) if i >= 4})
