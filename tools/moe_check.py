#!/usr/bin/env python3
"""Grouped expert GEMMs (variants 1 / 2) vs a torch fp32 per-expert reference
on the same routing (GPU box)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "physics-llm-inference_amd"), ROOT]
import torch  # noqa: E402

import pli_hip  # noqa: E402
from ch09 import MoEConfig, MoELayer  # noqa: E402

torch.manual_seed(0)
cfg = MoEConfig(hidden_dim=1024, expert_dim=2048)
moe = MoELayer(cfg).cuda().bfloat16().eval()
t1, t3, t2 = moe._weight_tables()
H, I = cfg.hidden_dim, cfg.expert_dim
for T in (3, 8, 64, 100, 256):
    x = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
    logits = pli_hip.gemm(x, moe.router.gate.weight, trans_b=True)
    w, idx, pos, gather, offsets = pli_hip.moe_route(logits, cfg.num_experts_per_tok, cfg.normalize_expert_weights)
    rows = T * cfg.num_experts_per_tok
    off = offsets.cpu().tolist()
    g = gather.cpu().long()
    ref_h = torch.empty(rows, I, device="cuda")
    ref_y = torch.empty(rows, H, device="cuda")
    for e, ex in enumerate(moe.experts):
        a, b = off[e], off[e + 1]
        if a == b:
            continue
        xe = x[g[a:b].cuda()].float()
        h = torch.nn.functional.silu(xe @ ex.w1.weight.float().t()) * (xe @ ex.w3.weight.float().t())
        ref_h[a:b] = h
        ref_y[a:b] = h.bfloat16().float() @ ex.w2.weight.float().t()
    for v in (1, 2):
        h = pli_hip.gemm_grouped(x, gather, t1, offsets, rows, I, H, H, wu_table=t3, variant=v)
        y = pli_hip.gemm_grouped(h, None, t2, offsets, rows, H, I, I, variant=v)
        eh = ((h.float() - ref_h).abs() / (ref_h.abs() + 1)).max().item()
        ey = ((y.float() - ref_y).abs() / (ref_y.abs() + 1)).max().item()
        print(f"T={T} rows={rows} v{v}: h rel err {eh:.2e}, y rel err {ey:.2e}", flush=True)
