#!/usr/bin/env python3
"""Generate golden vectors by running the REFERENCE itself (build container only).

Usage:  python tests/golden/make_golden.py [--ref /root/reference]

Imports the reference chapter packages from ``--ref`` (read-only, never copied)
and records, for seeded inputs, what the reference computes:

* ``flash_*.npz``   -- ``ch06.flash_attention_forward`` in the input dtype (the
  reference's own output) and ``ch06.naive_attention`` run in float64 on the
  same rounded inputs (the exact answer the kernels are held to);
* ``softmax.npz``  -- ``ch06.online_softmax`` / ``standard_softmax`` /
  ``online_softmax_with_output`` on fixed inputs, float64;
* ``mha.npz``      -- ``ch01.MultiHeadAttention(512, 8)`` built under
  ``torch.manual_seed(0)``: weight hashes and fp32 outputs (causal and not);
* ``tp.npz``       -- ``ch09`` Column/RowParallelLinear seeded weights + outputs;
* ``gqa.npz``      -- ``ch01.GroupedQueryAttention`` and the ``ch02`` cached
  attention modules (``GQAWithCache`` over ``KVCache``, ``CachedGQA`` over
  ``LayerKVCache``): seeded weights, a prompt, single-token decode steps and
  a 3-token chunk (bottom-right causal mask), fp32;
* ``kv_cache.json`` -- ``ch02.calculate_kv_cache_size`` over a small grid;
* ``moe.npz``      -- ``ch09`` MoELayer (hidden 256, experts 8 x 512, top-2)
  and its Router with seeded weights, fp32;
* ``ffn.npz``      -- ``ch01`` NaiveFFN / SwiGLUFFN / FusedSwiGLUFFN and the
  ``ch09`` TensorParallelMLP (world 1) with seeded weights, fp32;
* ``analytic.json`` -- exact values of the reference cost models
  (ch03 roofline / flops / bytes, ch06 memory + flops, ch09 comm models).

Inputs come from ``np.random.RandomState(seed)`` (portable), so the fixtures
hold outputs and input hashes only; ``tests/`` regenerates the inputs.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))  # repo root (oracle)

from oracle.numerics import array_hash, bf16_bits, seeded_normal  # noqa: E402

# (name, B, H, N, D, dtype, seed)  -- SURVEY.md §8(c) case list
FLASH_CASES = [
    ("b2h4n128d64_fp32", 2, 4, 128, 64, "fp32", 11),
    ("b2h4n128d64_fp16", 2, 4, 128, 64, "fp16", 12),
    ("b2h4n128d64_bf16", 2, 4, 128, 64, "bf16", 13),
    ("b1h8n512d64_fp16", 1, 8, 512, 64, "fp16", 14),
    ("b1h2n256d128_bf16", 1, 2, 256, 128, "bf16", 15),
    ("b1h2n200d64_bf16", 1, 2, 200, 64, "bf16", 16),   # ragged last tile
    ("b1h2n200d128_fp32", 1, 2, 200, 128, "fp32", 17),  # ragged, fp32
]


def torch_dtype(name):
    import torch
    return {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}[name]


def qkv_inputs(B, H, N, D, dtype, seed):
    shape = (B, H, N, D)
    return [seeded_normal(shape, seed * 10 + i, dtype) for i in range(3)]


def _compact(x, dt):
    """Lossless storage of dtype-representable float32 values."""
    if dt == "fp16":
        return x.astype(np.float16)
    if dt == "bf16":
        return bf16_bits(x)
    return x.astype(np.float32)


def gen_flash(ref_ch06, out_dir):
    import torch
    for name, B, H, N, D, dt, seed in FLASH_CASES:
        q, k, v = qkv_inputs(B, H, N, D, dt, seed)
        tq, tk, tv = (torch.from_numpy(a).to(torch_dtype(dt)) for a in (q, k, v))
        flash = ref_ch06.flash_attention_forward(tq, tk, tv).float().numpy()
        naive_dt = ref_ch06.naive_attention(tq, tk, tv).float().numpy()
        naive64 = ref_ch06.naive_attention(
            torch.from_numpy(q).double(), torch.from_numpy(k).double(),
            torch.from_numpy(v).double()).numpy()
        np.savez_compressed(
            os.path.join(out_dir, f"flash_{name}.npz"),
            shape=np.array([B, H, N, D]), seed=np.array(seed), dtype=np.array(dt),
            hash_q=np.array(array_hash(q)), hash_k=np.array(array_hash(k)),
            hash_v=np.array(array_hash(v)),
            # reference flash output, stored losslessly in its own dtype
            ref_flash=_compact(flash, dt),
            ref_naive_dtype_maxerr=np.array(np.abs(naive_dt - naive64).max()),
            # float64 reference rounded to float32 (7 significant digits)
            ref_naive_f64=naive64.astype(np.float32))
        print(f"flash {name}: max|flash-naive64| = {np.abs(flash - naive64).max():.3e}")


def gen_softmax(ref_ch06, out_dir):
    import torch
    x1 = np.array([1.0, 2.0, 3.0, 4.0, 5.0], dtype=np.float32)
    x2 = np.array([1000.0, 1001.0, 1002.0], dtype=np.float32)
    x3 = seeded_normal((4, 8, 64), 21)
    x4 = seeded_normal((2, 4, 32), 22)
    v4 = seeded_normal((2, 4, 32, 16), 23)
    d = {}
    for key, x in (("x1", x1), ("x2", x2), ("x3", x3)):
        t = torch.from_numpy(x).double()
        d[f"{key}_online"] = ref_ch06.online_softmax(t).numpy()
        d[f"{key}_standard"] = ref_ch06.standard_softmax(t).numpy()
    o, den = ref_ch06.online_softmax_with_output(torch.from_numpy(x4).double(),
                                                 torch.from_numpy(v4).double())
    d["x4_o"], d["x4_d"] = o.numpy(), den.numpy()
    d["hash_x3"] = np.array(array_hash(x3))
    d["hash_x4"] = np.array(array_hash(x4))
    d["hash_v4"] = np.array(array_hash(v4))
    np.savez_compressed(os.path.join(out_dir, "softmax.npz"), **d)
    print("softmax: ok")


def gen_mha(ref_ch01, out_dir):
    import torch
    B, S, hidden, heads = 1, 128, 512, 8
    torch.manual_seed(0)
    mha = ref_ch01.MultiHeadAttention(hidden, heads)
    x = seeded_normal((B, S, hidden), 31)
    with torch.no_grad():
        y_c = mha(torch.from_numpy(x), causal=True).numpy()
        y_n = mha(torch.from_numpy(x), causal=False).numpy()
    d = {f"hash_{n}": np.array(array_hash(p.detach().numpy()))
         for n, p in mha.named_parameters()}
    d["param_order"] = np.array([n for n, _ in mha.named_parameters()])
    d.update(y_causal=y_c, y_noncausal=y_n, hash_x=np.array(array_hash(x)))
    np.savez_compressed(os.path.join(out_dir, "mha.npz"), **d)
    print("mha: ok")


def gen_gqa(ref_ch01, ref_ch02, out_dir):
    import torch
    hidden, heads, kv_heads = 512, 8, 2
    d = {}
    torch.manual_seed(1)
    gqa = ref_ch01.GroupedQueryAttention(hidden, heads, kv_heads)
    x = seeded_normal((1, 64, hidden), 41)
    with torch.no_grad():
        d["gqa_causal"] = gqa(torch.from_numpy(x), causal=True).numpy()
        d["gqa_noncausal"] = gqa(torch.from_numpy(x), causal=False).numpy()
    d.update({f"gqa_hash_{n}": np.array(array_hash(p.detach().numpy()))
              for n, p in gqa.named_parameters()})
    # the same token stream through both cached modules: prompt 40, two decode
    # steps, then a 3-token chunk
    steps = [seeded_normal((2, 40, hidden), 42), seeded_normal((2, 1, hidden), 43),
             seeded_normal((2, 1, hidden), 44), seeded_normal((2, 3, hidden), 45)]
    torch.manual_seed(2)
    gwc = ref_ch02.GQAWithCache(hidden, heads, kv_heads)
    cache = ref_ch02.KVCache.create(2, 64, kv_heads, hidden // heads, torch.device("cpu"),
                                    torch.float32)
    torch.manual_seed(3)
    cg = ref_ch02.CachedGQA(hidden, heads, kv_heads)
    lc = ref_ch02.LayerKVCache(k=torch.zeros(2, 64, kv_heads, hidden // heads),
                               v=torch.zeros(2, 64, kv_heads, hidden // heads), seq_len=0)
    pos = 0
    with torch.no_grad():
        for i, xs in enumerate(steps):
            d[f"gwc_step{i}"] = gwc(torch.from_numpy(xs), kv_cache=cache)[0].numpy()
            d[f"cg_step{i}"] = cg(torch.from_numpy(xs), cache=lc, start_pos=pos).numpy()
            pos += xs.shape[1]
        d["gwc_nocache"] = gwc(torch.from_numpy(steps[0]), kv_cache=None)[0].numpy()
    d["cache_len"] = np.array([cache.seq_len, lc.seq_len])
    d.update({f"gwc_hash_{n}": np.array(array_hash(p.detach().numpy()))
              for n, p in gwc.named_parameters()})
    d.update({f"cg_hash_{n}": np.array(array_hash(p.detach().numpy()))
              for n, p in cg.named_parameters()})
    np.savez_compressed(os.path.join(out_dir, "gqa.npz"), **d)
    grid = [(b, s, l, h, hd, dt) for b in (1, 8) for s in (2048, 32768) for l in (1, 32)
            for h in (2, 8) for hd in (64, 128) for dt in ("float16", "float32")]
    kv = [[list(g), ref_ch02.calculate_kv_cache_size(*g[:5], dtype=getattr(torch, g[5]))]
          for g in grid]
    with open(os.path.join(out_dir, "kv_cache.json"), "w") as f:
        json.dump(kv, f, indent=0)
    print("gqa / kv_cache: ok")


def gen_ffn(ref_ch01, ref_ch09, out_dir):
    import importlib

    import torch
    hidden, inter = 256, 512
    x = seeded_normal((2, 16, hidden), 51)
    d = {}
    for seed, name in ((5, "NaiveFFN"), (6, "SwiGLUFFN"), (7, "FusedSwiGLUFFN")):
        torch.manual_seed(seed)
        m = getattr(ref_ch01, name)(hidden, inter)
        with torch.no_grad():
            d[name] = m(torch.from_numpy(x)).numpy()
        d.update({f"{name}_hash_{n}": np.array(array_hash(p.detach().numpy()))
                  for n, p in m.named_parameters()})
    torch.manual_seed(8)
    tpm = importlib.import_module("ch09.tensor_parallel")  # not re-exported by ch09/__init__
    mlp = tpm.TensorParallelMLP(tpm.TensorParallelConfig(
        world_size=1, rank=0, hidden_dim=hidden, intermediate_dim=inter))
    with torch.no_grad():
        d["TensorParallelMLP"] = mlp(torch.from_numpy(x)).numpy()
    d.update({f"TensorParallelMLP_hash_{n}": np.array(array_hash(p.detach().numpy()))
              for n, p in mlp.named_parameters()})
    np.savez_compressed(os.path.join(out_dir, "ffn.npz"), **d)
    print("ffn: ok")


def gen_moe(out_dir):
    import importlib

    import torch
    ml = importlib.import_module("ch09.moe_layer")
    cfg = ml.MoEConfig(hidden_dim=256, expert_dim=512, num_experts=8, num_experts_per_tok=2)
    torch.manual_seed(9)
    moe = ml.MoELayer(cfg)
    x = seeded_normal((2, 8, 256), 61)
    with torch.no_grad():
        y = moe(torch.from_numpy(x)).numpy()
        w, idx, logits = moe.router(torch.from_numpy(x).view(-1, 256))
    d = {"y": y, "router_w": w.numpy(), "router_idx": idx.numpy(), "router_logits": logits.numpy()}
    d.update({f"hash_{n}": np.array(array_hash(p.detach().numpy())) for n, p in moe.named_parameters()})
    np.savez_compressed(os.path.join(out_dir, "moe.npz"), **d)
    print("moe: ok")


def gen_tp(ref_ch09, out_dir):
    import torch
    d = {}
    torch.manual_seed(1)
    col = ref_ch09.ColumnParallelLinear(256, 1024, world_size=4, rank=0, bias=True)
    torch.manual_seed(2)
    row = ref_ch09.RowParallelLinear(1024, 256, world_size=4, rank=1, bias=True)
    x_col = seeded_normal((8, 256), 41)
    x_row = seeded_normal((8, 256), 42)
    with torch.no_grad():
        d["col_y"] = col(torch.from_numpy(x_col)).numpy()
        d["row_y"] = row(torch.from_numpy(x_row)).numpy()
    d["col_w_hash"] = np.array(array_hash(col.weight.detach().numpy()))
    d["row_w_hash"] = np.array(array_hash(row.weight.detach().numpy()))
    d["col_w_shape"] = np.array(col.weight.shape)
    d["row_w_shape"] = np.array(row.weight.shape)
    np.savez_compressed(os.path.join(out_dir, "tp.npz"), **d)
    print("tp: ok")


def gen_analytic(ref, out_dir):
    import torch
    ch03, ch06, ch09 = ref["ch03"], ref["ch06"], ref["ch09"]
    from ch03 import roofline as rl  # reference module (sys.path)
    from ch06 import flash_attention as fa
    from ch09 import nccl_primitives as npm
    from ch09 import tensor_parallel as tp
    out = {"gemm": [], "gemv": [], "roofline": [], "attn": [], "comm": [], "tp": [],
           "transition": []}
    for (m, n, k) in [(1, 1, 1), (1024, 1024, 1024), (512, 1024, 2048), (4096, 4096, 4096),
                      (8192, 8192, 1024)]:
        for dt in ("float16", "float32", "bfloat16"):
            tdt = getattr(torch, dt)
            out["gemm"].append({"m": m, "n": n, "k": k, "dtype": dt,
                                "flops": ch03.gemm_flops(m, n, k),
                                "bytes": ch03.gemm_bytes(m, n, k, tdt)})
            out["gemv"].append({"m": m, "k": k, "dtype": dt,
                                "flops": ch03.gemv_flops(m, k),
                                "bytes": ch03.gemv_bytes(m, k, tdt)})
    for hw in ("RTX_3090", "RTX_4090", "A100_80GB", "H100_SXM"):
        spec = getattr(rl, hw)
        row = {"hw": hw, "peak": spec.peak_tflops, "bw": spec.memory_bandwidth_gbps,
               "name": spec.name, "ridge": rl.ridge_point(spec), "points": []}
        for ai in (0.5, 1.0, 10.0, 38.0, 100.0, 153.0, 295.0, 1000.0):
            row["points"].append({"ai": ai, "tput": rl.roofline_throughput(ai, spec),
                                  "cb": rl.is_compute_bound(ai, spec)})
        out["roofline"].append(row)
        out["transition"].append({"hw": hw, "batch": ch03.find_transition_batch_size(
            4096, 4096, spec.peak_tflops, spec.memory_bandwidth_gbps)})
    out["ai"] = {
        "gemm_4096": rl.gemm_arithmetic_intensity(4096, 4096, 4096),
        "gemv_4096": rl.gemv_arithmetic_intensity(4096, 4096),
        "bgemv": [rl.batched_gemv_arithmetic_intensity(b, 4096, 4096) for b in (1, 4, 16, 64, 256, 512)],
        "basic": rl.arithmetic_intensity(1000, 100),
    }
    for (B, H, N, D) in [(1, 8, 1024, 64), (1, 32, 4096, 128), (8, 32, 4096, 128), (2, 4, 200, 64)]:
        st = ch06.attention_memory_bytes(B, H, N, D, 2)
        fm = fa.flash_attention_memory_bytes(B, H, N, D)
        out["attn"].append({"B": B, "H": H, "N": N, "D": D,
                            "flops": ch06.attention_flops(B, H, N, D),
                            "ai": ch06.attention_arithmetic_intensity(N, D),
                            "mem": {"qk": st.qk_bytes, "softmax": st.softmax_bytes,
                                    "output": st.output_bytes, "total": st.total_bytes,
                                    "total_mb": st.total_mb},
                            "flash_mem": fm})
    for ws in (2, 4, 8):
        ar = npm.simulate_all_reduce(npm.AllReduceConfig(world_size=ws, data_size_mb=10.0))
        ag = npm.simulate_all_gather(npm.AllGatherConfig(world_size=ws, data_size_per_gpu_mb=10.0))
        ring = npm.compute_ring_all_reduce_time(100 * 1024 * 1024, ws)
        out["comm"].append({"ws": ws, "ar": ar, "ag": ag, "ring": ring})
    out["overlap"] = [npm.compute_communication_overlap_potential(c, m)
                      for c, m in ((1000, 100), (100, 1000), (500, 200))]
    for ws in (1, 2, 4, 8):
        out["tp"].append({"ws": ws, **tp.compute_tp_memory_savings(4096, 14336, ws)})
    with open(os.path.join(out_dir, "analytic.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("analytic: ok")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=HERE)
    args = ap.parse_args()
    sys.path.insert(0, args.ref)
    sys.dont_write_bytecode = True
    import importlib
    ref = {n: importlib.import_module(n) for n in ("ch01", "ch02", "ch03", "ch06", "ch09")}
    gen_flash(ref["ch06"], args.out)
    gen_softmax(ref["ch06"], args.out)
    gen_mha(ref["ch01"], args.out)
    gen_tp(ref["ch09"], args.out)
    gen_gqa(ref["ch01"], ref["ch02"], args.out)
    gen_ffn(ref["ch01"], ref["ch09"], args.out)
    gen_moe(args.out)
    gen_analytic(ref, args.out)


if __name__ == "__main__":
    main()
