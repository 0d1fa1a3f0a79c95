#!/usr/bin/env python3
"""A few launches of the default GEMM at 4096^3 NN and NT and 8192^3 NT for
rocprofv3 --pmc passes (GPU box): LDS bank conflicts, LDS / MFMA / VALU
instruction counts, MFMA busy cycles per kernel."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "physics-llm-inference_amd"), ROOT]
import pli_hip  # noqa: E402

for (n, tb) in ((4096, False), (4096, True), (8192, True)):
    a = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
    c = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        pli_hip.gemm(a, b, trans_b=tb, out=c)
    torch.cuda.synchronize()
print("ok")
