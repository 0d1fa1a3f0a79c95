"""Time the flash fallback bodies where v13 does not apply -- D = 64 bf16
(v10 / v7 exact by the default route) and fp16 at D = 128 / 64 -- at the
bench's B8 H32 S4096 with torch SDPA beside them, plain and causal.  One
JSON line per case (events over 10 launches after 3 warm-up)."""
from __future__ import annotations

import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "physics-llm-inference_amd"))
import pli_hip  # noqa: E402


def ms(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    B, H, S = 8, 32, 4096
    # ~2 s of back-to-back launches so the clock leaves its idle state first
    x = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    for _ in range(200):
        x @ x
    torch.cuda.synchronize()
    for D, dt in ((64, torch.bfloat16), (128, torch.float16), (64, torch.float16)):
        g = torch.Generator(device="cuda").manual_seed(D)
        q, k, v = (torch.randn(B, H, S, D, device="cuda", dtype=dt, generator=g) for _ in range(3))
        out = torch.empty_like(q)
        for causal in (False, True):
            f = 4 * B * H * S * S * D / (2 if causal else 1)
            t = ms(lambda: pli_hip.flash_attn_fwd(q, k, v, causal=causal, out=out))
            ts = ms(lambda: F.scaled_dot_product_attention(q, k, v, is_causal=causal))
            print(json.dumps({"D": D, "dtype": str(dt).split(".")[-1], "causal": causal, "ms": round(t, 4),
                              "TFLOP/s": round(f / t / 1e9, 1), "sdpa_TFLOP/s": round(f / ts / 1e9, 1)}), flush=True)
        del q, k, v, out


if __name__ == "__main__":
    main()
