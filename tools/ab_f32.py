#!/usr/bin/env python3
"""GPU box: interleaved in-process A/B of the fp32 GEMM (pli_gemm, PLI_F32 ->
gemm_f32_mfma, the ch05 tiled-matmul demo's kernel) across the libraries in
$LIBS at $SHAPES (MxNxK, NN and NT); median TF/s per library and whether the
output is bitwise equal to the first library's."""
import ctypes
import json
import os
import statistics

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBS = os.environ.get("LIBS", "physics-llm-inference_amd/pli_hip/libpli_hip.so").split()
SHAPES = [tuple(int(x) for x in s.split("x")) for s in os.environ.get("SHAPES", "2048x2048x2048").split(",")]
ROUNDS, ITERS = int(os.environ.get("ROUNDS", "6")), int(os.environ.get("ITERS", "10"))
fns = []
for p in LIBS:
    lib = ctypes.CDLL(os.path.join(ROOT, p))
    f = lib.pli_gemm
    f.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int] * 3 + [ctypes.c_int64] * 3 + [ctypes.c_int] * 2 + [ctypes.c_void_p]
    f.restype = ctypes.c_int
    fns.append(f)
stream = torch.cuda.current_stream()
for (m, n, k) in SHAPES:
    a = torch.randn(m, k, device="cuda")
    for tb in (0, 1):
        b = torch.randn(n, k, device="cuda") if tb else torch.randn(k, n, device="cuda")
        outs = [torch.empty(m, n, device="cuda") for _ in fns]

        def call(i):
            rc = fns[i](a.data_ptr(), b.data_ptr(), outs[i].data_ptr(), None, m, n, k, k, k if tb else n, n, tb, 0,
                        ctypes.c_void_p(stream.cuda_stream))
            assert rc == 0
        for i in range(len(fns)):
            for _ in range(5):
                call(i)
        torch.cuda.synchronize()
        res = {i: [] for i in range(len(fns))}
        for _ in range(ROUNDS):
            for i in range(len(fns)):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record(stream)
                for _ in range(ITERS):
                    call(i)
                e.record(stream)
                e.synchronize()
                res[i].append(2 * m * n * k / (s.elapsed_time(e) / ITERS * 1e-3) / 1e12)
        for i in range(len(fns)):
            print(json.dumps({"lib": LIBS[i], "shape": [m, n, k], "nt": tb,
                              "TF/s_median": statistics.median(res[i]),
                              "bitwise_eq_first": bool(torch.equal(outs[i], outs[0]))}), flush=True)
