#!/usr/bin/env python3
"""GPU box: the reference's own GEMM benchmark configurations
(ch03/gemm_benchmark.py __main__: M = batch x seq in {16384, 32768, 65536,
4096}, N = K = 4096, torch.mm at fp16, i.e. NN) through pli_hip.gemm and
torch.mm (hipBLASLt), interleaved in one process; also bf16 and the NT
(F.linear) layout.  One JSON line per (shape, dtype, layout): median TF/s of
ROUNDS rounds of ITERS back-to-back launches, the route taken, and the max
relative difference between the two products."""
import json
import os
import statistics

import torch

import pli_hip

ROUNDS, ITERS = int(os.environ.get("ROUNDS", "6")), int(os.environ.get("ITERS", "10"))
SHAPES = [(16384, 4096, 4096), (32768, 4096, 4096), (65536, 4096, 4096), (4096, 4096, 4096)]
for dt in (torch.float16, torch.bfloat16):
    for (m, n, k) in SHAPES:
        for layout in ("nn", "nt"):
            g = torch.Generator(device="cuda").manual_seed(m)
            a = torch.randn(m, k, device="cuda", generator=g).to(dt)
            b = torch.randn(k, n, device="cuda", generator=g).to(dt) if layout == "nn" else \
                torch.randn(n, k, device="cuda", generator=g).to(dt)
            c = torch.empty(m, n, device="cuda", dtype=dt)
            ours = (lambda: pli_hip.gemm(a, b, out=c)) if layout == "nn" else \
                (lambda: pli_hip.gemm(a, b, trans_b=True, out=c))
            ref = (lambda: torch.mm(a, b)) if layout == "nn" else (lambda: torch.nn.functional.linear(a, b))
            ours()
            route = pli_hip.last_route()
            r = ref()
            diff = ((c.float() - r.float()).abs().max() / r.float().abs().max()).item()
            res = {"ours": [], "torch": []}
            for _ in range(3):
                ours(), ref()
            torch.cuda.synchronize()
            for _ in range(ROUNDS):
                for name, f in (("ours", ours), ("torch", ref)):
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    for _ in range(ITERS):
                        f()
                    e.record()
                    torch.cuda.synchronize()
                    res[name].append(2 * m * n * k * ITERS / (s.elapsed_time(e) * 1e-3) / 1e12)
            print(json.dumps({"m": m, "n": n, "k": k, "dtype": str(dt).split(".")[-1], "layout": layout,
                              "route": route, "TF/s": statistics.median(res["ours"]),
                              "torch_TF/s": statistics.median(res["torch"]), "max_rel_diff": diff}), flush=True)
