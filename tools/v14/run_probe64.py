#!/usr/bin/env python3
"""GPU box: time the head-dim-64 ping-pong probe variants (tools/v14/probe64.py),
interleaved in one process after a 1 s ramp.  Prints one JSON line per
variant: cycles per period per SIMD (two 64 x 64 wave-tiles at D = 64; the
MFMA floor is 72 x 2 x 16 = 2304 for the pair), the implied clock and the
equivalent TF/s (attn_fwd_v13's D = 64 form: 1109-1185 TF/s on the bench)."""
import ctypes
import json
import os
import statistics
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "build", os.environ.get("PP_LIB", "libpp64_probe.so")))
lib.pp64_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                          ctypes.c_float, ctypes.c_float, ctypes.c_void_p]
names = os.environ.get("PP_NAMES", "").split()
n = lib.pp64_count()
NIT, GRID, ROUNDS = int(os.environ.get("NIT", "512")), 256, int(os.environ.get("ROUNDS", "6"))
buf = (torch.randn(16 << 20, device="cuda", dtype=torch.float32) * 1.0).to(torch.bfloat16)
out = torch.zeros(8192, dtype=torch.int32, device="cuda")
stream = torch.cuda.current_stream()
c = 64 ** -0.5 * 1.4426950408889634


def launch(v):
    assert lib.pp64_launch(v, buf.data_ptr(), out.data_ptr(), NIT, GRID, c, 24.0, ctypes.c_void_p(stream.cuda_stream)) == 0


t_end = time.perf_counter() + 1.0
while time.perf_counter() < t_end:
    for v in range(n):
        launch(v)
    torch.cuda.synchronize()
res = {v: {"ms": [], "cyc": [], "cycA": [], "cycB": [], "waitC": [], "waitM": []} for v in range(n)}
for r in range(ROUNDS):
    for v in range(n):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(stream)
        for _ in range(5):
            launch(v)
        e.record(stream)
        e.synchronize()
        res[v]["ms"].append(s.elapsed_time(e) / 5)
        cyc = out[:2048].view(GRID, 8).double().cpu() / NIT
        res[v]["cyc"].append(cyc.mean().item())
        res[v]["cycA"].append(cyc[:, :4].mean().item())
        res[v]["cycB"].append(cyc[:, 4:].mean().item())
        res[v]["waitC"].append((out[4096:6144].double().cpu() / NIT).mean().item())
        res[v]["waitM"].append((out[6144:8192].double().cpu() / NIT).mean().item())
flop = 4 * 2 * (2 * 64 * 64 * 64 * 2) * GRID * NIT  # per CU per period: 4 SIMDs x 2 waves x 64x64 tile at D 64, QK + PV
for v in range(n):
    ms = statistics.median(res[v]["ms"])
    cyc = statistics.median(res[v]["cyc"])
    print(json.dumps({"variant": names[v] if v < len(names) else v, "cycles_per_period": round(cyc, 1),
                      "cycA": round(statistics.median(res[v]["cycA"]), 1),
                      "cycB": round(statistics.median(res[v]["cycB"]), 1),
                      "wait_after_C": round(statistics.median(res[v]["waitC"]), 1),
                      "wait_after_M": round(statistics.median(res[v]["waitM"]), 1),
                      "ms": round(ms, 4), "clock_GHz": round(cyc * NIT / (ms * 1e6), 3),
                      "TF/s": round(flop / (ms * 1e-3) / 1e12, 1)}), flush=True)
