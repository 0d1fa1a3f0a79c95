#!/usr/bin/env python3
"""GPU box: interleaved in-process A/B of flash builds (cdna_hip_programming.md
rule 24).  Every library in $LIBS (space-separated .so paths) is loaded with
ctypes side by side; each round times $ITERS back-to-back launches of its
pli_flash_attn_fwd_variant (variant $VARIANT, default -1 = the default
kernel) on the bench config (random data), libraries interleaved, after a
warm-up; prints the median / min TF/s per library and whether its output is
bitwise equal to the first library's.  $CAUSAL=1 times the causal form,
$SCALE sets the softmax scale (default 1/sqrt(D)), $DTYPE bf16 / fp16."""
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBS = os.environ.get("LIBS", "tools/ab/libpli_base.so physics-llm-inference_amd/pli_hip/libpli_hip.so").split()
ROUNDS, ITERS = int(os.environ.get("ROUNDS", "8")), int(os.environ.get("ITERS", "20"))
VARIANTS = [int(v) for v in os.environ.get("VARIANTS", os.environ.get("VARIANT", "-1")).split(",")]
CAUSAL = int(os.environ.get("CAUSAL", "0"))
SCALE = float(os.environ.get("SCALE", "0"))  # softmax scale (0: 1/sqrt(D))
SHAPES = [tuple(int(x) for x in sh.split(",")) for sh in os.environ.get("SHAPE", "8,32,4096,128").split(";")]
libs = []
for p in LIBS:
    lib = ctypes.CDLL(os.path.join(ROOT, p) if not os.path.isabs(p) else p)
    f = lib.pli_flash_attn_fwd_variant
    f.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int] * 6 + [ctypes.c_void_p, ctypes.c_float, ctypes.c_int,
                                                                 ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    f.restype = ctypes.c_int
    libs.append(f)
# (library, variant) arms, interleaved round by round
arms = [(li, var) for li in range(len(LIBS)) for var in VARIANTS]
stream = torch.cuda.current_stream()
DT = {"bf16": (2, torch.bfloat16), "fp16": (1, torch.float16)}[os.environ.get("DTYPE", "bf16")]  # PLI_BF16 / PLI_FP16
for (B, H, N, D) in SHAPES:
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = (torch.randn(B, H, N, D, device="cuda", dtype=DT[1], generator=g) for _ in range(3))
    outs = [torch.empty_like(q) for _ in arms]
    st = (ctypes.c_int64 * 12)(*(int(x) for t in (q, k, v, q) for x in t.stride()[:3]))

    def call(a):
        li, var = arms[a]
        rc = libs[li](q.data_ptr(), k.data_ptr(), v.data_ptr(), outs[a].data_ptr(), B, H, H, N, N, D, st,
                      SCALE or D ** -0.5, CAUSAL, DT[0], ctypes.c_void_p(stream.cuda_stream), var)
        assert rc == 0, (LIBS[li], var, rc)

    pairs = N * (N + 1) // 2 if CAUSAL else N * N
    flops = 4 * B * H * D * pairs
    for a in range(len(arms)):
        for _ in range(30):
            call(a)
    torch.cuda.synchronize()
    res = {a: [] for a in range(len(arms))}
    for r in range(ROUNDS):
        for a in range(len(arms)):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(stream)
            for _ in range(ITERS):
                call(a)
            e.record(stream)
            e.synchronize()
            res[a].append(flops / (s.elapsed_time(e) / ITERS * 1e-3) / 1e12)
    ref = outs[0].float()
    for a, (li, var) in enumerate(arms):
        print(json.dumps({"lib": LIBS[li], "shape": [B, H, N, D], "variant": var, "causal": CAUSAL, "scale": SCALE or D ** -0.5,
                          "TF/s_median": statistics.median(res[a]), "TF/s_min": min(res[a]),
                          "TF/s_max": max(res[a]), "bitwise_eq_first": bool(torch.equal(outs[a], outs[0])),
                          "max_diff_first": (outs[a].float() - ref).abs().max().item()}), flush=True)
    del q, k, v, outs
