#!/usr/bin/env python3
"""Workload for the rocprofv3 --pmc passes (tools/gpu_pmc.sh): a few launches
of each shipped hot-path kernel at its bench shape, nothing else, so each
kernel's counters come from dispatches of one known grid.

  flash    attn_fwd_v13 (default) and attn_fwd_v13c (causal default), B8 S4096 H32 D128;
           attn_fwd_v13h (fp16), attn_fwd_v13_d64 / v13h_d64 (head dim 64) at B8 S4096 H32
  flash12  attn_fwd_v12 (variant 71) and v12 causal (74), the round-3 kernels
  gemm     gemm_w5 4096^3 NN and NT (pli_gemm default routes)
  gemv     gemv_vec 4096^2 (W rotated over 24 copies)
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "physics-llm-inference_amd"), ROOT]
import pli_hip  # noqa: E402

N_LAUNCH = int(os.environ.get("PMC_LAUNCHES", "3"))
if os.environ.get("PMC_SET") == "gemm8k":
    # TP=1 8192^3 NT: gemm_w5 (one-tile form at K = 8192) beside hipBLASLt
    n = 8192
    g = torch.Generator(device="cuda").manual_seed(0)
    a = torch.randn(n, n, device="cuda", dtype=torch.bfloat16, generator=g)
    w = torch.randn(n, n, device="cuda", dtype=torch.bfloat16, generator=g)
    c = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
    for _ in range(N_LAUNCH):
        pli_hip.gemm(a, w, trans_b=True, out=c)
        torch.nn.functional.linear(a, w)
    torch.cuda.synchronize()
    print("pmc workload done", flush=True)
    sys.exit(0)
if os.environ.get("PMC_SET") == "causal":
    # causal walks side by side: 83 (pair walk, persistent) and 84 (one block
    # per workgroup, heaviest first) -- told apart by their grid sizes
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = (torch.randn(8, 32, 4096, 128, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
    o = torch.empty_like(q)
    for _ in range(N_LAUNCH):
        for var in (83, 84):
            pli_hip.flash_attn_fwd(q, k, v, out=o, causal=True, variant=var)
    torch.cuda.synchronize()
    print("pmc workload done", flush=True)
    sys.exit(0)
g = torch.Generator(device="cuda").manual_seed(0)
B, H, S, D = 8, 32, 4096, 128
q, k, v = (torch.randn(B, H, S, D, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
o = torch.empty_like(q)
for _ in range(N_LAUNCH):
    pli_hip.flash_attn_fwd(q, k, v, out=o)
    pli_hip.flash_attn_fwd(q, k, v, out=o, causal=True)
    pli_hip.flash_attn_fwd(q, k, v, out=o, variant=71)
    pli_hip.flash_attn_fwd(q, k, v, out=o, causal=True, variant=74)
torch.cuda.synchronize()
del q, k, v, o
# fp16 D = 128 and head dim 64 (bf16 / fp16) on their default routes
# (attn_fwd_v13h, attn_fwd_v13_d64, attn_fwd_v13h_d64 since round 5)
for dt, hd in ((torch.float16, 128), (torch.bfloat16, 64), (torch.float16, 64)):
    q, k, v = (torch.randn(B, H, S, hd, device="cuda", dtype=dt, generator=g) for _ in range(3))
    o = torch.empty_like(q)
    for _ in range(N_LAUNCH):
        pli_hip.flash_attn_fwd(q, k, v, out=o)
    torch.cuda.synchronize()
    del q, k, v, o
n = 4096
a = torch.randn(n, n, device="cuda", dtype=torch.bfloat16, generator=g)
b = torch.randn(n, n, device="cuda", dtype=torch.bfloat16, generator=g)
c = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
for _ in range(N_LAUNCH):
    pli_hip.gemm(a, b, out=c)                 # NN
    pli_hip.gemm(a, b, trans_b=True, out=c)   # NT
torch.cuda.synchronize()
ws = [torch.randn(n, n, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(24)]
x = torch.randn(n, device="cuda", dtype=torch.bfloat16, generator=g)
y = torch.empty(n, device="cuda", dtype=torch.bfloat16)
for _ in range(N_LAUNCH):
    for w in ws:
        pli_hip.gemv(w, x, out=y)
torch.cuda.synchronize()
print("pmc workload done", flush=True)
