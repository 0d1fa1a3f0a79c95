"""Time pli_hip.flash_attn_fwd at the bench shape (B8 H32 S4096 D128 bf16)
with the default scale and with explicit scales, to show which route each
takes on hardware: v13 (~1.6 ms) for any scale > 0 since round 4; the old
c <= 1 gate sent scale 1.0 to variant 21.  Variant 21 forced is timed
beside it for reference.  Output: one JSON line per case."""
from __future__ import annotations

import json
import os
import sys

import torch

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
    B, H, S, D = 8, 32, 4096, 128
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = (torch.randn(B, H, S, D, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
    out = torch.empty_like(q)
    flops = 4 * B * H * S * S * D
    for causal in (False, True):
        for scale in (None, 1.0, 0.25):
            t = ms(lambda: pli_hip.flash_attn_fwd(q, k, v, scale=scale, causal=causal, out=out))
            f = flops / (2 if causal else 1)
            print(json.dumps({"causal": causal, "scale": scale, "ms": round(t, 4), "TFLOP/s": round(f / t / 1e9, 1)}),
                  flush=True)
        t = ms(lambda: pli_hip.flash_attn_fwd(q, k, v, scale=1.0, causal=causal, out=out, variant=21), n=3)
        print(json.dumps({"causal": causal, "scale": 1.0, "variant": 21, "ms": round(t, 4)}), flush=True)


if __name__ == "__main__":
    main()
