#!/usr/bin/env python3
"""Seam ablations with clocks (GPU box; round-6 verdict item 1).  For each
stamped diagnostic library in $DIAG_LIBS (tools/build_diag.sh with
STAMP_ARGS=abl=... and DIAG_OUT=...), interleaved over $ROUNDS rounds:

  * >= $RAMP s of back-to-back *stamped* launches of that build (so the
    clock settles on the build's own power draw, guide item 6);
  * $ITERS stamped launches timed with HIP events -> TF/s;
  * from the last launch's stamps: the in-kernel clock (sum of d s_memtime /
    sum of d s_memrealtime x 100 MHz), the mean wave cycles, and the per-block
    cycles of each seam section (tools/v13/kernel.py Gen.seam_stamp: loop,
    tail, epilogue, next_params, common_wait, first_tile).

$GRIDS (comma list, default "0") also runs each library at smaller
persistent grids (multiples of 8; 0 = one workgroup per CU): fewer CUs at a
seam together, the same per-CU work order.  Prints one JSON line per (lib,
grid, round)."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBS = os.environ.get("DIAG_LIBS", "tools/libpli_diag.so").split()
ROUNDS, ITERS = int(os.environ.get("ROUNDS", "2")), int(os.environ.get("ITERS", "10"))
RAMP = float(os.environ.get("RAMP", "2.0"))
GRIDS = [int(x) for x in os.environ.get("GRIDS", "0").split(",")]
N = int(os.environ.get("N", "4096"))
B, H, D = max(1, 8 * 4096 * 4096 // (N * N)), 32, 128
NAMES = ["loop", "tail", "epilogue", "next_params", "common_wait", "first_tile"]

libs = []
for p in LIBS:
    lib = ctypes.CDLL(p if os.path.isabs(p) else os.path.join(ROOT, p))
    lib.pli_diag_v13_clock.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int] * 3 + [ctypes.c_void_p]
    lib.pli_diag_v13_set_grid.argtypes = [ctypes.c_int]
    libs.append(lib)
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn(B, H, N, D, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
o = torch.empty_like(q)
cus = torch.cuda.get_device_properties(0).multi_processor_count
stamps = torch.zeros(cus * 4 * 32, dtype=torch.int32, device="cuda")
flops = 4 * B * H * N * N * D


def launch(lib):
    assert lib.pli_diag_v13_clock(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, H, N,
                                  stamps.data_ptr()) == 0


for rnd in range(ROUNDS):
    for li, lib in enumerate(libs):
        for grid in GRIDS:
            lib.pli_diag_v13_set_grid(grid)
            G = grid or cus // 8 * 8
            t_end = time.perf_counter() + RAMP
            while time.perf_counter() < t_end:
                launch(lib)
            t0 = time.perf_counter()
            for _ in range(ITERS):
                launch(lib)  # (each launch synchronizes inside the diag entry)
            ms = (time.perf_counter() - t0) / ITERS * 1e3
            st = stamps.cpu().numpy().view(np.uint32).reshape(-1, 32)[:4 * G].astype(np.uint64)
            t0s, t1s = st[:, 0] | (st[:, 1] << 32), st[:, 4] | (st[:, 5] << 32)
            r0s, r1s = st[:, 2] | (st[:, 3] << 32), st[:, 6] | (st[:, 7] << 32)
            dt, dr = (t1s - t0s).astype(np.float64), (r1s - r0s).astype(np.float64)
            blocks = B * H * (-(-N // 256)) / G
            seams = {n: float(st[:, 16 + i].astype(np.float64).mean() / blocks) for i, n in enumerate(NAMES)}
            seam_total = sum(v_ for k_, v_ in seams.items() if k_ != "loop")
            span_us = float((r1s.max() - r0s.min()) / 100)
            print(json.dumps({
                "lib": LIBS[li], "grid": G, "round": rnd, "N": N, "B": B,
                "host_ms_per_launch": round(ms, 4),
                "TF/s_span": round(flops / (span_us * 1e-6) / 1e12, 1),
                "clock_GHz": round(float(dt.sum() / dr.sum() * 0.1), 3),
                "wave_cycles_mean": round(float(dt.mean())),
                "blocks_per_wg": blocks,
                "per_block_cycles": {k_: round(v_) for k_, v_ in seams.items()},
                "seam_cycles_per_block": round(seam_total),
                "loop_cycles_per_tile": round(seams["loop"] / max(1, N // 64 - 2), 1),
                "span_us": round(span_us, 1)}), flush=True)
