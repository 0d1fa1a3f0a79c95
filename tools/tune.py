#!/usr/bin/env python3
"""A/B kernel variants in ONE process (interleaved rounds), GPU box only.

    python tools/tune.py [leg ...]   (default: hbm gemv flash gemm)

Legs: hbm (copy ceiling), gemv / bgemv / gemvsweep (decode GEMV), flash /
flash64 (prefill variants, PLI_FLASH_VARIANTS), gemm / gemmshapes (256-tile
schedules, PLI_GEMM_VARIANTS / PLI_GEMM_SHAPES), midm (decode-batch and
few-tile NT routes), swiglu / swr (fused SwiGLU, decode-batch routes), moe /
moeg (MoE layer, grouped expert GEMM routes), decode (decode attention
modes), graph (HIP-graph decode step at batch 1 / 8 / 32).

Prints one JSON object per measurement; correctness of every variant is
checked against variant 0 (and flash against the f64 oracle on one head).
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "physics-llm-inference_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import pli_hip  # noqa: E402


def ev_ms(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def interleave(fns: dict, iters: int, rounds: int):
    res = {k: [] for k in fns}
    for _ in range(rounds):
        for k, fn in fns.items():
            res[k].append(ev_ms(fn, iters))
    return {k: (float(np.median(v)), float(np.min(v))) for k, v in res.items()}


def tune_flash(variants=None, causal=False, B=8, H=32, S=4096, D=128):
    from oracle.attention import naive_attention
    if variants is None:
        variants = tuple(int(x) for x in os.environ.get("PLI_FLASH_VARIANTS", "21,30,31").split(","))
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = (torch.randn(B, H, S, D, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
    outs = {vv: torch.empty_like(q) for vv in variants}
    for vv in variants:
        pli_hip.flash_attn_fwd(q, k, v, causal=causal, out=outs[vv], variant=vv)
    torch.cuda.synchronize()
    ref = naive_attention(*(t[0:1, 0:1].float().cpu().numpy() for t in (q, k, v)), causal=causal)
    fns = {vv: (lambda vv=vv: pli_hip.flash_attn_fwd(q, k, v, causal=causal, out=outs[vv], variant=vv))
           for vv in variants}
    t = interleave(fns, 5, int(os.environ.get("PLI_TUNE_ROUNDS", "3")))
    flops = 4 * B * H * S * S * D * (0.5 if causal else 1.0)
    for vv in variants:
        diff = (outs[vv].float() - outs[variants[0]].float()).abs().max().item()
        err = float(np.abs(outs[vv][0:1, 0:1].float().cpu().numpy() - ref).max())
        print(json.dumps({"kernel": "flash", "variant": vv, "causal": causal, "ms_med": t[vv][0],
                          "ms_min": t[vv][1], "TFLOP/s": flops / t[vv][0] / 1e9,
                          "maxdiff_vs_v0": diff, "err_vs_f64_head0": err}), flush=True)


def tune_gemv(variants=(0, 1, 2, 3, 4, 5, 6, 7, 8), m=4096, k=4096, copies=24):
    """GEMV variants, each as a HIP graph of `copies` launches over rotated
    weights (device time per launch incl. kernel boundaries, no host cost)."""
    ws = [torch.randn(m, k, device="cuda", dtype=torch.bfloat16) for _ in range(copies)]
    x = torch.randn(k, device="cuda", dtype=torch.bfloat16)
    ys = {vv: torch.empty(m, device="cuda", dtype=torch.bfloat16) for vv in variants}
    ref = (ws[0].float() @ x.float())
    graphs = {}
    for vv in variants:
        for w in ws:
            pli_hip.gemv(w, x, out=ys[vv], variant=vv)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for w in ws:
                pli_hip.gemv(w, x, out=ys[vv], variant=vv)
        graphs[vv] = gr
    t = interleave({vv: graphs[vv].replay for vv in variants}, 10, 5)
    nbytes = (m * k + m + k) * 2
    for vv in variants:
        pli_hip.gemv(ws[0], x, out=ys[vv], variant=vv)
        err = ((ys[vv].float() - ref).abs() / (ref.abs() + 1)).max().item()
        us = t[vv][0] * 1e3 / copies
        print(json.dumps({"kernel": "gemv", "variant": vv, "us_per_launch": us,
                          "GB/s": nbytes / (us * 1e-6) / 1e9, "rel_err": err}), flush=True)


def tune_gemv_sweep():
    """Per-launch time vs size: separates fixed launch/latency cost from
    streaming bandwidth (t = t0 + bytes / BW)."""
    for m in (1024, 2048, 4096, 8192, 16384):
        k = m
        copies = max(2, (768 << 20) // (m * k * 2))
        ws = [torch.randn(m, k, device="cuda", dtype=torch.bfloat16) for _ in range(copies)]
        x = torch.randn(k, device="cuda", dtype=torch.bfloat16)
        y = torch.empty(m, device="cuda", dtype=torch.bfloat16)
        st = {"i": 0}

        def f():
            pli_hip.gemv(ws[st["i"] % copies], x, out=y)
            st["i"] += 1
        for _ in range(2 * copies):
            f()
        t = interleave({"g": f}, max(4 * copies, 40), 3)["g"][0]
        nbytes = (m * k + m + k) * 2
        print(json.dumps({"kernel": "gemv_sweep", "m": m, "copies": copies, "us": t * 1e3,
                          "GB/s": nbytes / (t * 1e-3) / 1e9}), flush=True)
        del ws
    # the same launches captured in a HIP graph: device time incl. the kernel
    # boundary, without Python launch overhead
    for m in (4096, 8192):
        k = m
        copies = max(2, (768 << 20) // (m * k * 2))
        ws = [torch.randn(m, k, device="cuda", dtype=torch.bfloat16) for _ in range(copies)]
        x = torch.randn(k, device="cuda", dtype=torch.bfloat16)
        y = torch.empty(m, device="cuda", dtype=torch.bfloat16)
        for w in ws:
            pli_hip.gemv(w, x, out=y)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for w in ws:
                pli_hip.gemv(w, x, out=y)
        for _ in range(3):
            gr.replay()
        t = interleave({"g": gr.replay}, 10, 3)["g"][0] / copies
        nbytes = (m * k + m + k) * 2
        print(json.dumps({"kernel": "gemv_graph", "m": m, "copies": copies, "us": t * 1e3,
                          "GB/s": nbytes / (t * 1e-3) / 1e9}), flush=True)
        del ws
    # empty-kernel launch gap: a 1-element scale_copy back to back
    a = torch.zeros(4, device="cuda")
    b = torch.zeros(4, device="cuda")
    t = interleave({"e": lambda: pli_hip.scale_copy(a, b)}, 200, 3)["e"][0]
    print(json.dumps({"kernel": "empty_launch", "us": t * 1e3}), flush=True)


def tune_bgemv():
    """x @ W^T for decode batches: HIP (skinny <= 16, MFMA tile above) vs torch."""
    m = k = 4096
    copies = 24
    ws = [torch.randn(m, k, device="cuda", dtype=torch.bfloat16) for _ in range(copies)]
    for bsz in (1, 2, 4, 8, 16, 32, 64):
        x = torch.randn(bsz, k, device="cuda", dtype=torch.bfloat16)
        y = torch.empty(bsz, m, device="cuda", dtype=torch.bfloat16)
        graphs = {}
        for name, fn in (("hip", lambda w: pli_hip.gemm(x, w, trans_b=True, out=y)),
                         ("torch", lambda w: torch.matmul(x, w.t(), out=y))):
            for w in ws:
                fn(w)
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                for w in ws:
                    fn(w)
            graphs[name] = gr
        t = interleave({n: g.replay for n, g in graphs.items()}, 5, 3)
        nbytes = (m * k + bsz * (m + k)) * 2
        print(json.dumps({"kernel": "batched_gemv", "batch": bsz,
                          **{f"{n}_us": t[n][0] * 1e3 / copies for n in t},
                          **{f"{n}_GB/s": nbytes / (t[n][0] * 1e-3 / copies) / 1e9 for n in t}}), flush=True)


def tune_decode(configs=((1, 32, 8, 32768), (8, 32, 8, 4096), (32, 32, 8, 4096), (8, 32, 8, 32768),
                          (64, 32, 8, 2048), (1, 32, 8, 131072)), D=128,
                modes=((13, 0), (0, 0))):
    """Decode attention over a [B, S, Hkv, D] bf16 cache: HIP split-K vs the
    reference formulation (repeat_interleave + matmul + softmax + matmul,
    ch02/kv_cache.py:81-98) in torch.  Graph of `copies` launches over rotated
    caches (> 1 GiB total, past the 256 MiB MALL)."""
    import math
    for B, H, Hkv, n in configs:
        kv_bytes = 2 * B * n * Hkv * D * 2
        copies = max(2, min(16, math.ceil((1 << 30) / kv_bytes)))
        ks = [torch.randn(B, n, Hkv, D, device="cuda", dtype=torch.bfloat16) for _ in range(copies)]
        vs = [torch.randn(B, n, Hkv, D, device="cuda", dtype=torch.bfloat16) for _ in range(copies)]
        q = torch.randn(B, 1, H, D, device="cuda", dtype=torch.bfloat16)
        out = torch.empty_like(q)

        def ref(k, v):
            qt = q.transpose(1, 2)
            kt = k.transpose(1, 2).repeat_interleave(H // Hkv, dim=1)
            vt = v.transpose(1, 2).repeat_interleave(H // Hkv, dim=1)
            sc = torch.matmul(qt, kt.transpose(-2, -1)) / math.sqrt(D)
            return torch.matmul(torch.softmax(sc, dim=-1), vt)

        fns = {f"hip{m}_{tg}": (lambda k, v, m=m, tg=tg: pli_hip.attn_decode(
            q, k, v, n, out=out, causal=False, variant=m, target_wgs=tg)) for m, tg in modes}
        if kv_bytes * (H // Hkv) * 2 < (24 << 30):
            fns["torch_ref"] = ref
        graphs = {}
        for name, fn in fns.items():
            for k, v in zip(ks, vs):
                fn(k, v)
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                for k, v in zip(ks, vs):
                    fn(k, v)
            graphs[name] = gr
        t = interleave({nm: g.replay for nm, g in graphs.items()}, 3, 3)
        fns[f"hip{modes[0][0]}_{modes[0][1]}"](ks[-1], vs[-1])
        ref_out = ref(ks[-1], vs[-1]).transpose(1, 2)
        err = (ref_out.float() - out.float()).abs().max().item()
        nbytes = kv_bytes + 2 * q.numel() * 2
        print(json.dumps({"kernel": "attn_decode", "B": B, "Hq": H, "Hkv": Hkv, "n_kv": n, "D": D,
                          "splits_ws_MB": pli_hip.attn_decode_workspace_bytes(B, H, Hkv, 1, n, D) / 2**20,
                          **{f"{nm}_us": t[nm][0] * 1e3 / copies for nm in t},
                          **{f"{nm}_GB/s": nbytes / (t[nm][0] * 1e-3 / copies) / 1e9 for nm in t},
                          "maxdiff_vs_torch": err}), flush=True)
        del ks, vs, graphs
        torch.cuda.empty_cache()


def tune_swiglu():
    """Fused SwiGLU (one launch) vs unfused: torch (2 hipBLASLt GEMMs + silu*mul)
    and HIP (2 pli_gemm + torch silu*mul), at TensorParallelConfig's defaults
    (hidden 4096, intermediate 14336 = TP1; 1792 = the TP8 shard).  Weights
    rotated over > 1 GiB for the decode sizes.  Graph-timed."""
    import math
    import torch.nn.functional as F
    H = 4096
    for inter in (14336, 1792):
        wbytes = 2 * inter * H * 2
        copies = max(2, min(12, math.ceil((1 << 30) / wbytes)))
        wg = [torch.randn(inter, H, device="cuda", dtype=torch.bfloat16) * H ** -0.5 for _ in range(copies)]
        wu = [torch.randn(inter, H, device="cuda", dtype=torch.bfloat16) * H ** -0.5 for _ in range(copies)]
        for m in tuple(int(v) for v in os.environ.get("PLI_SWIGLU_M", "1,8,32,128,4096").split(",")):
            x = torch.randn(m, H, device="cuda", dtype=torch.bfloat16)
            out = torch.empty(m, inter, device="cuda", dtype=torch.bfloat16)
            fns = {"fused": lambda a, b: pli_hip.gemm_swiglu(x, a, b, out=out),
                   "fused_nosplit": lambda a, b: pli_hip.gemm_swiglu(x, a, b, out=out, split_k=False),
                   "hip_unfused": lambda a, b: torch.mul(F.silu(pli_hip.gemm(x, a, trans_b=True)),
                                                         pli_hip.gemm(x, b, trans_b=True), out=out),
                   "torch": lambda a, b: torch.mul(F.silu(x @ a.t()), x @ b.t(), out=out)}
            graphs = {}
            for nm, fn in fns.items():
                for a, b in zip(wg, wu):
                    fn(a, b)
                torch.cuda.synchronize()
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr):
                    for a, b in zip(wg, wu):
                        fn(a, b)
                graphs[nm] = gr
            t = interleave({nm: g.replay for nm, g in graphs.items()}, 3, 3)
            fns["torch"](wg[-1], wu[-1])
            ref = out.float().clone()
            fns["fused"](wg[-1], wu[-1])
            err = ((out.float() - ref).abs().max() / (ref.abs().max() + 1e-6)).item()
            flops = 2 * 2 * m * inter * H
            nbytes = wbytes + (m * H + m * inter) * 2
            print(json.dumps({"kernel": "swiglu", "m": m, "inter": inter,
                              **{f"{nm}_us": t[nm][0] * 1e3 / copies for nm in t},
                              **{f"{nm}_TFLOP/s": flops / (t[nm][0] * 1e-3 / copies) / 1e12 for nm in t},
                              **{f"{nm}_GB/s": nbytes / (t[nm][0] * 1e-3 / copies) / 1e9 for nm in t},
                              "rel_diff_vs_torch": err}), flush=True)
        del wg, wu
        torch.cuda.empty_cache()


def tune_graph(batches=(1, 8, 32), prompt=512, steps=32):
    """ch02 decode step of a Llama-shaped model (vocab 32000, hidden 2048,
    16 layers, 32/8 heads, intermediate 5632, bf16): per-token latency of
    eager steps (host-length caches) vs one HIP-graph launch per step
    (ch08.DecodeStepGraph, device-length caches)."""
    import time
    from ch02 import CachedTransformerModel
    from ch08 import DecodeStepGraph
    torch.manual_seed(0)
    model = CachedTransformerModel(32000, 2048, 16, 32, 8, 5632).cuda().bfloat16().eval()
    for B in batches:
        ids = torch.randint(0, 32000, (B, prompt), device="cuda")
        tok = torch.randint(0, 32000, (B, 1), device="cuda")
        res = {}
        with torch.no_grad():
            for mode in ("eager", "eager_devlen", "graph"):
                if mode == "graph":
                    g = DecodeStepGraph(model, B, prompt + steps + 8, torch.bfloat16)
                    g.prefill(ids)
                    fn = lambda: g.step(tok)  # noqa: E731
                else:
                    caches = model.create_caches(B, prompt + steps + 8, torch.device("cuda"),
                                                 torch.bfloat16, device_pos=(mode == "eager_devlen"))
                    model(ids, caches)
                    fn = lambda: model(tok, caches, start_pos=caches[0].seq_len)  # noqa: E731
                fn()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(steps - 1):
                    fn()
                torch.cuda.synchronize()
                res[mode] = (time.perf_counter() - t0) / (steps - 1) * 1e3
        print(json.dumps({"kernel": "decode_step", "batch": B, "prompt": prompt,
                          **{f"{k}_ms_per_token": v for k, v in res.items()},
                          **{f"{k}_tok/s": B / (v * 1e-3) for k, v in res.items()}}), flush=True)


def tune_moe(tokens=(1, 8, 32, 128)):
    """ch09 MoE layer at MoEConfig's defaults (hidden 4096, 8 experts x 14336,
    top-2), bf16: the HIP path (route + 2 grouped GEMMs + combine) vs the
    reference's masked per-expert loop, same device and weights.  GB/s over
    the weights of the experts actually selected."""
    import time
    from ch09 import MoEConfig, MoELayer
    torch.manual_seed(0)
    cfg = MoEConfig()
    moe = MoELayer(cfg).cuda().bfloat16().eval()

    def ref_forward(x):  # ch09/moe_layer.py:58-83 on the same weights (torch ops)
        x_flat = x.view(-1, cfg.hidden_dim)
        logits = (x_flat @ moe.router.gate.weight.t()).float()  # fp32 routing: no bf16 top-k flips
        w = torch.softmax(logits, dim=-1)
        tw, ti = torch.topk(w, cfg.num_experts_per_tok, dim=-1)
        tw = tw / tw.sum(-1, keepdim=True)
        out = torch.zeros_like(x_flat)
        for e in range(cfg.num_experts):
            mask = (ti == e).any(dim=-1)
            if not mask.any():
                continue
            ex = moe.experts[e]
            xe = x_flat[mask]
            ye = (torch.nn.functional.silu(xe @ ex.w1.weight.t()) * (xe @ ex.w3.weight.t())) @ ex.w2.weight.t()
            for kk in range(cfg.num_experts_per_tok):
                em = ti[:, kk] == e
                cm = mask & em
                if cm.any():
                    out[cm] += tw[cm, kk].unsqueeze(-1).to(x.dtype) * ye[em[mask]]
        return out.view_as(x)

    per_expert = 3 * cfg.hidden_dim * cfg.expert_dim * 2
    if os.environ.get("PLI_MOE_T"):
        tokens = tuple(int(v) for v in os.environ["PLI_MOE_T"].split(","))
    for T in tokens:
        x = torch.randn(1, T, cfg.hidden_dim, device="cuda", dtype=torch.bfloat16)
        with torch.no_grad():
            y = moe(x)
            yr = ref_forward(x)
            active = int(torch.unique(moe.router(x.view(-1, cfg.hidden_dim))[1]).numel())
            res = {}
            for name, fn in (("hip", lambda: moe(x)), ("reference", lambda: ref_forward(x))):
                fn()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(10):
                    fn()
                torch.cuda.synchronize()
                res[name] = (time.perf_counter() - t0) / 10 * 1e3
        err = ((y.float() - yr.float()).norm() / yr.float().norm()).item()
        print(json.dumps({"kernel": "moe_layer", "tokens": T, "active_experts": active,
                          **{f"{k}_us": v * 1e3 for k, v in res.items()},
                          **{f"{k}_GB/s": active * per_expert / (v * 1e-3) / 1e9 for k, v in res.items()},
                          **{f"{k}_TFLOP/s": 2 * T * cfg.num_experts_per_tok * 3 * cfg.hidden_dim
                             * cfg.expert_dim / (v * 1e-3) / 1e12 for k, v in res.items()},
                          "rel_diff": err}), flush=True)


def tune_hbm():
    for nbytes in (1 << 28, 1 << 30):
        n = nbytes // 4
        src = torch.randn(n, device="cuda")
        dst = torch.empty_like(src)
        t = interleave({"copy": lambda: pli_hip.scale_copy(src, dst)}, 20, 3)["copy"][0]
        t_torch = interleave({"c": lambda: dst.copy_(src)}, 20, 3)["c"][0]
        print(json.dumps({"kernel": "scale_copy", "bytes": nbytes, "GB/s": 2 * nbytes / (t * 1e-3) / 1e9,
                          "torch_copy_GB/s": 2 * nbytes / (t_torch * 1e-3) / 1e9}), flush=True)


def tune_gemm():
    for n in (4096, 8192):
        a = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
        b = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
        c = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
        vs = [int(v) for v in os.environ.get("PLI_GEMM_VARIANTS", "2,5,6,7,8").split(",")]
        fns = {}
        for v in vs:
            fns[f"hip_nn_v{v}"] = (lambda v=v: pli_hip.gemm(a, b, out=c, variant=v))
            fns[f"hip_nt_v{v}"] = (lambda v=v: pli_hip.gemm(a, b, trans_b=True, out=c, variant=v))
        fns["torch_nn"] = lambda: torch.mm(a, b)
        fns["torch_nt"] = lambda: torch.mm(a, b.t())
        t = interleave(fns, 5, int(os.environ.get("PLI_TUNE_ROUNDS", "3")))
        for kname, (med, mn) in t.items():
            print(json.dumps({"kernel": "gemm", "n": n, "impl": kname, "ms_med": med,
                              "TFLOP/s": 2 * n ** 3 / med / 1e9}), flush=True)


def tune_gemm_shapes():
    """256-tile schedule / rasterization variants over the callers' shapes."""
    shapes = [(4096, 4096, 4096), (8192, 8192, 8192), (16384, 4096, 4096), (4096, 14336, 4096),
              (4096, 4096, 14336), (8192, 1024, 8192), (8192, 8192, 1024), (2048, 2048, 2048),
              (1024, 1024, 1024), (512, 4096, 4096), (4096, 512, 4096), (1024, 8192, 8192)]
    if os.environ.get("PLI_GEMM_SHAPES"):
        shapes = [tuple(int(x) for x in sh.split("x")) for sh in os.environ["PLI_GEMM_SHAPES"].split(",")]
    vs = [int(v) for v in os.environ.get("PLI_GEMM_VARIANTS", "2,13,12,14").split(",")]
    for (m, n, k) in shapes:
        a = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
        bt = torch.randn(n, k, device="cuda", dtype=torch.bfloat16)
        bn = torch.randn(k, n, device="cuda", dtype=torch.bfloat16)
        c = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        fns = {}
        for v in vs:
            fns[f"nt_v{v}"] = (lambda v=v: pli_hip.gemm(a, bt, trans_b=True, out=c, variant=v))
            fns[f"nn_v{v}"] = (lambda v=v: pli_hip.gemm(a, bn, out=c, variant=v))
        fns["nt_torch"] = lambda: torch.mm(a, bt.t())
        fns["nn_torch"] = lambda: torch.mm(a, bn)
        # every variant against torch's product (relative to |ref| + 1)
        errs = {}
        for lay, bb, tb in (("nt", bt, True), ("nn", bn, False)):
            ref = torch.mm(a, bb.t() if tb else bb).float()
            for v in vs:
                o = pli_hip.gemm(a, bb, trans_b=tb, variant=v).float()
                errs[f"{lay}_v{v}"] = round(((o - ref).abs() / (ref.abs() + 1)).max().item(), 4)
        t = interleave(fns, 5, int(os.environ.get("PLI_TUNE_ROUNDS", "3")))
        row = {kname: round(2 * m * n * k / med / 1e9, 1) for kname, (med, mn) in t.items()}
        print(json.dumps({"kernel": "gemm_shapes", "m": m, "n": n, "k": k, "TFLOP/s": row, "max_rel_err": errs}),
              flush=True)


def tune_midm():
    """Decode-batch / TP-shard NT GEMMs at M = 17..256: the split-K path with
    256 / 512 / 128 target workgroups (0 / 22 / 24, workspace from the
    wrapper), the mid-M kernel (20), the small-M kernel (21), torch F.linear."""
    shapes = [(m, n, k) for (n, k) in ((8192, 8192), (4096, 4096), (8192, 1024), (14336, 4096))
              for m in (17, 32, 64, 128, 256)]
    if os.environ.get("PLI_GEMM_SHAPES"):
        shapes = [tuple(int(x) for x in sh.split("x")) for sh in os.environ["PLI_GEMM_SHAPES"].split(",")]
    for (m, n, k) in shapes:
        x = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(n, k, device="cuda", dtype=torch.bfloat16) * k ** -0.5
        ref = torch.nn.functional.linear(x.float(), w.float())
        outs = {v: torch.empty(m, n, device="cuda", dtype=torch.bfloat16) for v in (0, 20, 21, 25, 26, 27)}
        fns = {f"v{v}": (lambda v=v: pli_hip.gemm(x, w, trans_b=True, out=outs[v], variant=v)) for v in outs}
        fns["torch"] = lambda: torch.nn.functional.linear(x, w)
        errs = {}
        for v in outs:
            fns[f"v{v}"]()
            errs[f"v{v}"] = round(((outs[v].float() - ref).abs() / (ref.abs() + 1)).max().item(), 4)
        t = interleave(fns, 10, int(os.environ.get("PLI_TUNE_ROUNDS", "3")))
        print(json.dumps({"kernel": "midm", "m": m, "n": n, "k": k,
                          "us": {kk: round(med * 1e3, 1) for kk, (med, mn) in t.items()},
                          "weight_TB/s": {kk: round(n * k * 2 / med / 1e9, 2) for kk, (med, mn) in t.items()},
                          "err": errs}), flush=True)


def tune_moe_grouped():
    """The two grouped expert GEMMs of the ch09 MoE layer (MoEConfig defaults)
    on the same routing: variant 1 (weight-streaming / 256-row tile routes)
    vs 2 (LDS-staged grouped kernel); GB/s over the active experts' weights."""
    from ch09 import MoEConfig, MoELayer
    torch.manual_seed(0)
    cfg = MoEConfig()
    moe = MoELayer(cfg).cuda().bfloat16().eval()
    t1, t3, t2 = moe._weight_tables()
    H, I = cfg.hidden_dim, cfg.expert_dim
    tokens = tuple(int(v) for v in os.environ.get("PLI_MOE_T", "1,8,32,64,128,256,512").split(","))
    for T in tokens:
        x = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
        with torch.no_grad():
            logits = pli_hip.gemm(x, moe.router.gate.weight, trans_b=True)
            w, _, pos, gather, offsets = pli_hip.moe_route(logits, cfg.num_experts_per_tok,
                                                           cfg.normalize_expert_weights)
        rows = T * cfg.num_experts_per_tok
        active = int((offsets[1:] - offsets[:-1] > 0).sum().item())
        outs = {}

        def run(v):
            h = pli_hip.gemm_grouped(x, gather, t1, offsets, rows, I, H, H, wu_table=t3, variant=v)
            return pli_hip.gemm_grouped(h, None, t2, offsets, rows, H, I, I, variant=v)
        for v in (1, 2):
            outs[v] = run(v).float()
        diff = (outs[1] - outs[2]).abs().max().item() / (outs[1].abs().max().item() + 1e-6)
        t = interleave({v: (lambda v=v: run(v)) for v in (1, 2)}, 5, 3)
        wbytes = active * 3 * H * I * 2
        print(json.dumps({"kernel": "moe_grouped", "tokens": T, "active_experts": active,
                          "us": {f"v{v}": round(t[v][0] * 1e3, 1) for v in t},
                          "weight_TB/s": {f"v{v}": round(wbytes / t[v][0] / 1e9, 2) for v in t},
                          "rel_diff_v1_v2": diff}), flush=True)


def tune_swiglu_routes():
    """SwiGLU decode-batch routes on the same shapes: default, forced split-K
    (variant 1), never split (2), torch (2 GEMMs + silu * mul)."""
    import torch.nn.functional as F
    shapes = [tuple(int(x) for x in sh.split("x")) for sh in os.environ.get(
        "PLI_SWIGLU_SHAPES", "32x5632x2048,64x5632x2048,128x5632x2048,32x14336x4096,32x1792x4096,128x1792x4096").split(",")]
    for (m, n, k) in shapes:
        x = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
        wg = torch.randn(n, k, device="cuda", dtype=torch.bfloat16) * k ** -0.5
        wu = torch.randn(n, k, device="cuda", dtype=torch.bfloat16) * k ** -0.5
        out = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        fns = {"default": lambda: pli_hip.gemm_swiglu(x, wg, wu, out=out),
               "split": lambda: pli_hip.gemm_swiglu(x, wg, wu, out=out, variant=1),
               "nosplit": lambda: pli_hip.gemm_swiglu(x, wg, wu, out=out, variant=2),
               "torch": lambda: torch.mul(F.silu(x @ wg.t()), x @ wu.t(), out=out)}
        t = interleave(fns, 10, 3)
        print(json.dumps({"kernel": "swiglu_routes", "m": m, "n": n, "k": k,
                          "us": {kk: round(v[0] * 1e3, 1) for kk, v in t.items()}}), flush=True)


if __name__ == "__main__":
    what = sys.argv[1:] or ["hbm", "gemv", "flash", "gemm"]
    if "hbm" in what:
        tune_hbm()
    if "gemv" in what:
        tune_gemv()
    if "bgemv" in what:
        tune_bgemv()
    if "gemvsweep" in what:
        tune_gemv_sweep()
    if "flash" in what:
        tune_flash()
        tune_flash(causal=True)
    if "flash64" in what:
        tune_flash(D=64, H=64)
    if "gemm" in what:
        tune_gemm()
    if "midm" in what:
        tune_midm()
    if "moeg" in what:
        tune_moe_grouped()
    if "swr" in what:
        tune_swiglu_routes()
    if "gemmshapes" in what:
        tune_gemm_shapes()
    if "decode" in what:
        tune_decode()
    if "swiglu" in what:
        tune_swiglu()
    if "graph" in what:
        tune_graph()
    if "moe" in what:
        tune_moe()
