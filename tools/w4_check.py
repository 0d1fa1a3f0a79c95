#!/usr/bin/env python3
"""Max |O_variant - O_21| for flash variants over a few shapes (GPU box)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "physics-llm-inference_amd"), ROOT]
import torch  # noqa: E402

import pli_hip  # noqa: E402

variants = [int(a) for a in sys.argv[1:]]
for (B, H, N, causal) in [(1, 4, 1024, False), (1, 4, 2048, False), (1, 8, 4096, False), (2, 32, 4096, False),
                          (8, 32, 4096, False), (1, 8, 4096, True)]:
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = (torch.randn(B, H, N, 128, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
    ref = pli_hip.flash_attn_fwd(q, k, v, causal=causal, variant=21).float()
    res = []
    for var in variants:
        o = pli_hip.flash_attn_fwd(q, k, v, causal=causal, variant=var).float()
        d = (o - ref).abs()
        bad = (d > 1e-2).nonzero()
        res.append(f"{var}:{d.max().item():.1e}" + (f"(n{bad.shape[0]} bh{tuple(bad[0, :2].tolist())} row{bad[0, 2].item()})" if bad.shape[0] else ""))
    print((B, H, N, causal), " ".join(res), flush=True)
