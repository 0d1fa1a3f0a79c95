#!/usr/bin/env python3
"""Cycle anatomy of the v7 flash body from the diagnostic build
(tools/build_diag.sh -> tools/libpli_diag.so, s_memtime stamps; GPU box).

    python tools/flash_stamps.py [sub ...]     (0: PRE 1, 1: PRE 0, 2/3: staggered)

Per wave and tile: mean cycles of each segment (stamps are fenced by
sched_barriers, so read SHARES, not the absolute length)."""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libpli_diag.so"))
lib.pli_diag_flash_stamps.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int] * 4 + [ctypes.POINTER(ctypes.c_ulonglong)]
SEGS = ["loads/dma_issue", "qk_mfma+max", "exp", "rescale_chk+pack", "pv_issue", "lds_store", "barrier"]

B, H, N, D = 8, 32, 4096, 128
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn(B, H, N, D, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
o = torch.empty_like(q)
buf = (ctypes.c_ulonglong * 16)()
for sub in [int(a) for a in sys.argv[1:]] or [0, 1]:
    for _ in range(8):  # warm: clocks settle under back-to-back launches
        rc = lib.pli_diag_flash_stamps(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, H, N, sub, buf)
        assert rc == 0, rc
    vals = list(buf)
    tiles, waves = vals[8], vals[9]
    per = {SEGS[i]: vals[i] / tiles for i in range(7)}
    tot = sum(per.values())
    print(json.dumps({"sub": sub, "waves": waves, "tiles_per_wave": tiles / max(1, waves),
                      "cycles_per_wave_tile": {k2: round(v2, 1) for k2, v2 in per.items()},
                      "total": round(tot, 1),
                      "share": {k2: round(v2 / tot, 3) for k2, v2 in per.items()}}), flush=True)
