#!/usr/bin/env python3
"""GPU box: interleaved A/B of decode-attention modes / chunk targets on the
bench workload (B8, 32q/8kv heads, 32768 keys, D128 bf16, two 1 GiB caches
alternated): $MODES (comma list of pli_attn_decode_variant modes, -1 =
default) x $TARGETS (target workgroup counts, 0 = default); prints median
GB/s per arm and whether the output equals the default arm's."""
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "physics-llm-inference_amd"), ROOT]
import pli_hip  # noqa: E402

MODES = [int(x) for x in os.environ.get("MODES", "-1").split(",")]
TARGETS = [int(x) for x in os.environ.get("TARGETS", "0").split(",")]
ROUNDS, ITERS = int(os.environ.get("ROUNDS", "8")), int(os.environ.get("ITERS", "20"))
B, Hq, Hkv, n, D = 8, 32, 8, 32768, 128
caches = [(torch.randn(B, n, Hkv, D, device="cuda", dtype=torch.bfloat16),
           torch.randn(B, n, Hkv, D, device="cuda", dtype=torch.bfloat16)) for _ in range(2)]
q = torch.randn(B, 1, Hq, D, device="cuda", dtype=torch.bfloat16)
arms = [(m, t) for m in MODES for t in TARGETS]
outs = {a: torch.empty_like(q) for a in arms}
nbytes = 2 * B * n * Hkv * D * 2 + 2 * q.numel() * 2
state = {"i": 0}


def step(a, out):
    kc, vc = caches[state["i"] & 1]
    state["i"] += 1
    pli_hip.attn_decode(q, kc, vc, n, out=out, causal=False, variant=a[0], target_wgs=a[1])


for a in arms:
    for _ in range(4):
        step(a, outs[a])
torch.cuda.synchronize()
res = {a: [] for a in arms}
st = torch.cuda.current_stream()
for _ in range(ROUNDS):
    for a in arms:
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(st)
        for _ in range(ITERS):
            step(a, outs[a])
        e.record(st)
        e.synchronize()
        res[a].append(nbytes / (s.elapsed_time(e) / ITERS * 1e-3) / 1e9)
ref = caches[(state["i"] - 1) & 1]
for a in arms:
    step(a, outs[a])  # same cache for every arm
    state["i"] -= 1
torch.cuda.synchronize()
for a in arms:
    print(json.dumps({"mode": a[0], "target_wgs": a[1], "GB/s_median": round(statistics.median(res[a]), 1),
                      "GB/s_max": round(max(res[a]), 1),
                      "equal_first": bool(torch.equal(outs[a], outs[arms[0]]))}), flush=True)
