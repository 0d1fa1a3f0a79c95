#!/usr/bin/env python3
"""Where a v13 block seam spends its cycles (GPU box, diagnostic build
tools/libpli_diag.so): >= 2 s of back-to-back product launches, then one
stamped launch whose waves sum, per seam point (tools/v13/kernel.py
Gen.seam_stamp), the cycles since the previous point: the tile loop, the tail
(PV of the last tile), the epilogue (normalise + O stores), the next block's
parameters, its common code (O / l zero, wait for Q and tiles 0 / 1, barrier)
and its first tile (QK, exact row max, exps, second barrier).  Prints the
per-block means over waves at $N (default 4096)."""
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
N = int(os.environ.get("N", "4096"))
B, H, D = max(1, 8 * 4096 * 4096 // (N * N)), 32, 128  # the bench's FLOPs at every N
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn(B, H, N, D, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
o = torch.empty_like(q)
names = ["loop", "tail", "epilogue", "next_params", "common_wait", "first_tile"]
for rep in range(2):
    t_end = time.perf_counter() + 2.0
    while time.perf_counter() < t_end:
        for _ in range(20):
            pli_hip.flash_attn_fwd(q, k, v, out=o, variant=80)
        torch.cuda.synchronize()
    stamps = torch.zeros(256 * 4 * 32, dtype=torch.int32, device="cuda")
    assert lib.pli_diag_v13_clock(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, H, N,
                                  stamps.data_ptr()) == 0
    st = stamps.cpu().numpy().view(np.uint32).reshape(-1, 32).astype(np.uint64)
    t0, t1 = st[:, 0] | (st[:, 1] << 32), st[:, 4] | (st[:, 5] << 32)
    r0, r1 = st[:, 2] | (st[:, 3] << 32), st[:, 6] | (st[:, 7] << 32)
    total = (t1 - t0).astype(np.float64)
    blocks = B * H * (-(-N // 256)) / 256  # per workgroup
    seams = {n: float(st[:, 16 + i].astype(np.float64).mean() / blocks) for i, n in enumerate(names)}
    out = {"N": N, "B": B, "H": H, "blocks_per_wg": blocks, "clock_GHz": round(float(total.sum() / (r1 - r0).sum() * 0.1), 3),
           "wave_cycles_mean": round(float(total.mean())), "per_block_cycles": {k_: round(v_) for k_, v_ in seams.items()},
           "tiles_per_block": N // 64,
           "loop_cycles_per_tile": round(seams["loop"] / max(1, N // 64 - 2), 1)}
    print(json.dumps(out), flush=True)
