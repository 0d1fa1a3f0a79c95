#!/usr/bin/env python3
"""Cycle anatomy of attn_fwd_v12 (flash variant 70) from the diagnostic build
(tools/build_diag.sh -> tools/libpli_diag.so; GPU box): s_memtime sums per
wave per tile at the bench config."""
import ctypes
import json
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.environ.get("DIAG_LIB") or os.path.join(ROOT, "tools", "libpli_diag.so"))
lib.pli_diag_v12_stamps.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int] * 3 + [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int, ctypes.c_int]
SEGS = ["kfrag_wait", "phaseQ", "dma_wait", "barrier", "phaseP", "defer_max", "loop+first_softmax", "tail",
        "seam_ozero_kreads", "seam_vmcnt0", "seam_barrier_q", "seam_QK0", "loop_exit", "unused",
        "epi_loadq", "epi_tailB", "epi_PV", "epi_l", "epi_storeA", "epi_storeB"]
B, H, N = 8, 32, 4096
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn(B, H, N, 128, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
o = torch.empty_like(q)
buf = (ctypes.c_ulonglong * 24)()
for grid in (0, 256):  # 0: one block per workgroup (variant 70); 256: persistent (71)
    for _ in range(6):
        assert lib.pli_diag_v12_stamps(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, H, N, buf, grid, 1) == 0
    vals = list(buf)
    tiles, waves = vals[22], vals[23]
    per = {SEGS[i]: vals[i] / tiles for i in range(20)}
    tot = sum(per.values())
    print(json.dumps({"lib": os.path.basename(os.environ.get("DIAG_LIB", "libpli_diag.so")), "grid": grid or "all",
                      "waves": waves, "tiles_per_wave": tiles / max(1, waves),
                      "cycles_per_wave_tile": {a: round(b, 1) for a, b in per.items()}, "total": round(tot, 1),
                      "mfma_floor": 64 * 32 + 8 * 16}), flush=True)
