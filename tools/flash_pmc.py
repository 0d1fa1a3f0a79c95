#!/usr/bin/env python3
"""Flash prefill launches of the given kernel variants (bench workload,
B=8 H=32 S=4096 D=128 bf16; PLI_PMC_D=64 / PLI_PMC_DTYPE=fp16 for the other
legs) for rocprofv3 --pmc passes:

    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace \\
        -d gpurun_out/pmc -o run -- python tools/flash_pmc.py 21 30

Each variant runs `reps` times after one warm-up; rows of the counter CSV are
told apart by dispatch order (variants in argv order)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "physics-llm-inference_amd"), ROOT]

import torch  # noqa: E402

import pli_hip  # noqa: E402

variants = [int(a) for a in sys.argv[1:]] or [21]
reps = int(os.environ.get("PLI_PMC_REPS", "3"))
causal = os.environ.get("PLI_PMC_CAUSAL", "0") == "1"
D = int(os.environ.get("PLI_PMC_D", "128"))
dt = torch.float16 if os.environ.get("PLI_PMC_DTYPE", "bf16") == "fp16" else torch.bfloat16
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn(8, 32, 4096, D, device="cuda", dtype=dt, generator=g)
           for _ in range(3))
out = torch.empty_like(q)
for var in variants:
    for _ in range(reps + 1):
        pli_hip.flash_attn_fwd(q, k, v, causal=causal, out=out, variant=var)
    torch.cuda.synchronize()
print("variants", variants, "reps", reps + 1, "causal", causal, "D", D, "dtype", dt)
