#!/usr/bin/env python3
"""GPU box: does the flash bench line depend on what ran before it?  One
process: (1) fresh, W warmup + K timed flash launches (bench.py's timing);
(2) bench.py's calibration legs; (3) again W + K.  Prints TF/s of (1) and
(3) and the per-launch times of the first 30 launches of (1)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "physics-llm-inference_amd"), ROOT]
import torch  # noqa: E402

import pli_hip  # noqa: E402

W, K = int(os.environ.get("W", "5")), int(os.environ.get("K", "20"))
B, H, S, D = 8, 32, 4096, 128
gen = torch.Generator(device="cuda").manual_seed(1234)
q, k, v = (torch.randn(B, H, S, D, device="cuda", dtype=torch.bfloat16, generator=gen) for _ in range(3))
o = torch.empty_like(q)
flops = 4 * B * H * S * S * D


def timed():
    for _ in range(W):
        pli_hip.flash_attn_fwd(q, k, v, out=o)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        pli_hip.flash_attn_fwd(q, k, v, out=o)
    torch.cuda.synchronize()
    return flops * K / (time.perf_counter() - t0) / 1e12


first = timed()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(31)]
ev[0].record()
for i in range(30):
    pli_hip.flash_attn_fwd(q, k, v, out=o)
    ev[i + 1].record()
torch.cuda.synchronize()
per = [round(flops / (ev[i].elapsed_time(ev[i + 1]) * 1e-3) / 1e12, 1) for i in range(30)]
import bench  # noqa: E402
t0 = time.perf_counter()
cal = bench.calibrate()
cal_s = time.perf_counter() - t0
after = timed()
print(json.dumps({"fresh_TF/s": first, "after_calibration_TF/s": after, "calibration_s": cal_s,
                  "next_30_launches_TF/s": per, "W": W, "K": K}))
