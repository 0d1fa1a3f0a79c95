#!/usr/bin/env python3
"""GPU box: interleaved in-process A/B of GEMM builds (cdna_hip_programming.md
rule 24).  Every library in $LIBS is loaded with ctypes side by side; each
round times $ITERS back-to-back pli_gemm_variant calls (variant $VARIANT,
$VARIANTS, default 40) per library and variant and layout on random bf16 data, libraries
interleaved; prints median / min TF/s per (library, layout) and whether the
output is bitwise equal to the first library's.  $SHAPES: MxNxK,...;
$LAYOUTS: nt,nn; torch (hipBLASLt) is timed beside them."""
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBS = os.environ.get("LIBS", "physics-llm-inference_amd/pli_hip/libpli_hip.so").split()
ROUNDS, ITERS = int(os.environ.get("ROUNDS", "6")), int(os.environ.get("ITERS", "10"))
VARIANTS = [int(v) for v in os.environ.get("VARIANTS", os.environ.get("VARIANT", "40")).split(",")]
LAYOUTS = os.environ.get("LAYOUTS", "nt,nn").split(",")
SHAPES = [tuple(int(x) for x in s.split("x")) for s in os.environ.get("SHAPES", "4096x4096x4096").split(",")]
fns = []
for p in LIBS:
    lib = ctypes.CDLL(os.path.join(ROOT, p) if not os.path.isabs(p) else p)
    f = lib.pli_gemm_variant
    f.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int] * 3 + [ctypes.c_int64] * 3 + [ctypes.c_int] * 2 + \
        [ctypes.c_void_p, ctypes.c_int]
    f.restype = ctypes.c_int
    fns.append(f)
stream = torch.cuda.current_stream()
for (m, n, k) in SHAPES:
    a = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
    bt = torch.randn(n, k, device="cuda", dtype=torch.bfloat16)
    bn = torch.randn(k, n, device="cuda", dtype=torch.bfloat16)
    arms = [(li, lay, v) for lay in LAYOUTS for li in range(len(LIBS)) for v in VARIANTS] + \
        [(-1, lay, None) for lay in LAYOUTS]
    outs = [torch.empty(m, n, device="cuda", dtype=torch.bfloat16) for _ in arms]

    def call(i):
        li, lay, var = arms[i]
        b = bt if lay == "nt" else bn
        if li < 0:
            torch.mm(a, b.t() if lay == "nt" else b, out=outs[i])
            return
        rc = fns[li](a.data_ptr(), b.data_ptr(), outs[i].data_ptr(), None, m, n, k, k, k if lay == "nt" else n, n,
                     1 if lay == "nt" else 0, 2, ctypes.c_void_p(stream.cuda_stream), var)
        assert rc == 0, (LIBS[li], rc)

    for i in range(len(arms)):
        for _ in range(5):
            call(i)
    torch.cuda.synchronize()
    res = {i: [] for i in range(len(arms))}
    for _ in range(ROUNDS):
        for i in range(len(arms)):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(stream)
            for _ in range(ITERS):
                call(i)
            e.record(stream)
            e.synchronize()
            res[i].append(2 * m * n * k / (s.elapsed_time(e) / ITERS * 1e-3) / 1e12)
    for i, (li, lay, var) in enumerate(arms):
        first = arms.index((0, lay, VARIANTS[0]))
        print(json.dumps({"lib": LIBS[li] if li >= 0 else "torch", "layout": lay, "shape": [m, n, k],
                          "variant": var,
                          "TF/s_median": round(statistics.median(res[i]), 1), "TF/s_min": round(min(res[i]), 1),
                          "TF/s_max": round(max(res[i]), 1),
                          "bitwise_eq_first": bool(torch.equal(outs[i], outs[first]))}), flush=True)
