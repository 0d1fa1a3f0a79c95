#!/usr/bin/env python3
"""Sustained NT/NN GEMM throughput (20 back-to-back launches per sample,
variants interleaved over rounds, median) against torch (hipBLASLt), at the
ch09 shard / ch03 shapes.  PLI_GEMM_VARIANTS (default 0,12,2)."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "physics-llm-inference_amd"), ROOT]
import torch  # noqa: E402

import pli_hip  # noqa: E402


def ev(fn, n):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / n


variants = [int(v) for v in os.environ.get("PLI_GEMM_VARIANTS", "0,12,2").split(",")]
shapes = [(8192, 8192, 8192, True), (8192, 8192, 4096, True), (8192, 8192, 2048, True),
          (8192, 8192, 1024, True), (4096, 4096, 4096, True), (4096, 4096, 4096, False),
          (8192, 8192, 8192, False), (4096, 14336, 4096, True)]
for (m, n, k, tb) in shapes:
    a = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
    b = (torch.randn(n, k, device="cuda", dtype=torch.bfloat16) if tb
         else torch.randn(k, n, device="cuda", dtype=torch.bfloat16)) * k ** -0.5
    c = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
    fns = {f"v{v}": (lambda v=v: pli_hip.gemm(a, b, trans_b=tb, out=c, variant=v)) for v in variants}
    fns["torch"] = (lambda: torch.nn.functional.linear(a, b)) if tb else (lambda: torch.mm(a, b))
    for f in fns.values():
        f()
    res = {kk: [] for kk in fns}
    for _ in range(4):
        for kk, f in fns.items():
            res[kk].append(ev(f, 20))
    tf = {kk: round(2 * m * n * k / statistics.median(v) / 1e9) for kk, v in res.items()}
    print(f"{m}x{n}x{k} {'NT' if tb else 'NN'} sustained TF/s:", tf, flush=True)
