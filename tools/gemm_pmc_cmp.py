#!/usr/bin/env python3
"""GPU box, under rocprofv3 --pmc: three launches each of the default GEMM
and of torch (hipBLASLt) at 8192^3 NT on the same bf16 data, for
stall-counter comparisons of the two main loops (tools/gemm_pmc_cmp.sh)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "physics-llm-inference_amd"), ROOT]
import pli_hip  # noqa: E402

n = int(os.environ.get("N", "8192"))
a = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
b = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
c = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
for _ in range(3):
    pli_hip.gemm(a, b, trans_b=True, out=c)
for _ in range(3):
    torch.mm(a, b.t(), out=c)
torch.cuda.synchronize()
print("ok")
