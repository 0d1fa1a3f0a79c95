"""GPU parity of decode attention over a KV cache (pli_attn_decode) and of the
ch01 GQA / ch02 cached modules that use it.

Oracle: oracle.attention.naive_attention in float64 on the same rounded
inputs (GQA head mapping h // (H/Hkv), bottom-right causal mask = the
reference's triu(..., diagonal=n_kv - n_q + 1), ch02/kv_cache.py:91-95).
Tolerance 1e-2 for bf16/fp16 outputs, 1e-3 for fp32 (north_star).  Module
outputs in fp32 are held to the reference's own outputs (gqa.npz).
"""
from __future__ import annotations

import zlib

import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import attention as oatt
from oracle.numerics import seeded_normal

pytestmark = pytest.mark.gpu
TDT = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}
TOL = {"fp32": 1e-3, "fp16": 1e-2, "bf16": 1e-2}

# B, Hq, Hkv, Sq, n_kv, S_max, D, dtype, causal
CASES = [
    (1, 32, 8, 1, 4096, 4200, 128, "bf16", False),   # split-K over many chunks
    (4, 8, 2, 1, 333, 400, 64, "fp16", False),       # ragged chunk, G=4
    (2, 16, 16, 1, 1, 8, 128, "bf16", False),        # one cached token, G=1
    (1, 8, 1, 1, 77, 80, 128, "bf16", False),        # G=8
    (2, 32, 2, 1, 1000, 1024, 64, "bf16", False),    # G=16: a full 16-row tile
    (1, 8, 2, 3, 50, 64, 128, "bf16", True),         # 3-token chunk, bottom-right mask
    (1, 4, 4, 4, 4, 4, 64, "bf16", True),            # prompt == cache
    (2, 8, 2, 2, 9000, 9000, 128, "fp16", True),     # 2-token chunk, long cache
    (1, 8, 2, 8, 2048, 2048, 128, "bf16", True),     # 32 rows/kv head: prefill kernel
    (1, 8, 2, 1, 300, 320, 128, "fp32", False),      # fp32: generic kernel
    (1, 4, 2, 1, 129, 130, 80, "bf16", False),       # head_dim 80: generic kernel
    (16, 32, 8, 1, 2048, 2048, 128, "bf16", False),  # batch grid, 1 chunk per head
]


def _case_id(c):
    return "b{}h{}kv{}sq{}n{}s{}d{}_{}{}".format(*c[:8], "_causal" if c[8] else "")


@pytest.mark.parametrize("mode", [None, 2, 9, 11, 13])
@pytest.mark.parametrize("case", CASES, ids=_case_id)
def test_decode_vs_oracle(case, mode):
    import pli_hip
    B, H, Hkv, Sq, n_kv, S_max, D, dt, causal = case
    seed = zlib.crc32(repr(case).encode()) % 1000
    q = seeded_normal((B, Sq, H, D), seed, dt)
    kc = seeded_normal((B, S_max, Hkv, D), seed + 1, dt)
    vc = seeded_normal((B, S_max, Hkv, D), seed + 2, dt)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda().to(TDT[dt])
    out = pli_hip.attn_decode(dev(q), dev(kc), dev(vc), n_kv, causal=causal, variant=mode)
    assert out.shape == (B, Sq, H, D) and out.dtype == TDT[dt]
    ref = oatt.naive_attention(q.transpose(0, 2, 1, 3), kc[:, :n_kv].transpose(0, 2, 1, 3),
                               vc[:, :n_kv].transpose(0, 2, 1, 3), causal=causal)
    got = out.float().cpu().numpy().transpose(0, 2, 1, 3).astype(np.float64)
    assert np.isfinite(got).all()
    err = np.abs(got - ref).max()
    assert err <= TOL[dt], f"max |err| {err:.3e}"


def test_decode_reads_cache_in_place_and_ignores_stale_tail():
    """Positions >= n_kv hold garbage (huge values): they must not leak in."""
    import pli_hip
    B, H, Hkv, S_max, D, n_kv = 2, 16, 4, 512, 128, 300
    q = seeded_normal((B, 1, H, D), 5, "bf16")
    kc = seeded_normal((B, S_max, Hkv, D), 6, "bf16")
    vc = seeded_normal((B, S_max, Hkv, D), 7, "bf16")
    kc[:, n_kv:] = 300.0
    vc[:, n_kv:] = 1e4
    dev = lambda a: torch.from_numpy(a).cuda().bfloat16()
    out = pli_hip.attn_decode(dev(q), dev(kc), dev(vc), n_kv)
    ref = oatt.naive_attention(q.transpose(0, 2, 1, 3), kc[:, :n_kv].transpose(0, 2, 1, 3),
                               vc[:, :n_kv].transpose(0, 2, 1, 3))
    assert np.abs(out.float().cpu().numpy().transpose(0, 2, 1, 3) - ref).max() <= 1e-2


def test_decode_split_invariance():
    """Split-K must not change the answer: the same head computed with many
    chunks (B=1) and with one chunk (as part of a big batch) agree."""
    import pli_hip
    H, Hkv, D, n = 32, 8, 128, 8192
    q = torch.randn(1, 1, H, D, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(1, n, Hkv, D, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(1, n, Hkv, D, device="cuda", dtype=torch.bfloat16)
    assert pli_hip.attn_decode_workspace_bytes(1, H, Hkv, 1, n, D) > 0
    assert pli_hip.attn_decode_workspace_bytes(128, H, Hkv, 1, n, D) == 0
    one = pli_hip.attn_decode(q, k, v, n)
    big = pli_hip.attn_decode(q.expand(128, 1, H, D).contiguous(), k.expand(128, n, Hkv, D),
                              v.expand(128, n, Hkv, D), n)
    diff = (big.float() - one.float()).abs().max().item()
    assert diff <= 2 ** -7, diff


def test_decode_graph_capture():
    """The decode call is capturable (no host sync, workspace from the graph pool)."""
    import pli_hip
    q = torch.randn(1, 1, 32, 128, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(1, 4096, 8, 128, device="cuda", dtype=torch.bfloat16)
    v = torch.randn_like(k)
    ref = pli_hip.attn_decode(q, k, v, 4000)
    out = torch.empty_like(ref)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        pli_hip.attn_decode(q, k, v, 4000, out=out)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


# ------------------------------------------------------------ modules ---
def test_gqa_module_matches_reference_on_gpu():
    from ch01 import GroupedQueryAttention
    g = load_golden("gqa.npz")
    torch.manual_seed(1)
    m = GroupedQueryAttention(512, 8, 2).cuda()
    x = torch.from_numpy(seeded_normal((1, 64, 512), 41)).cuda()
    with torch.no_grad():
        for causal, key in ((True, "gqa_causal"), (False, "gqa_noncausal")):
            y = m(x, causal=causal).cpu().numpy()
            np.testing.assert_allclose(y, g[key], rtol=1e-3, atol=1e-3)


def test_cached_modules_match_reference_stream_on_gpu():
    from ch02 import CachedGQA, GQAWithCache, KVCache, LayerKVCache
    g = load_golden("gqa.npz")
    torch.manual_seed(2)
    gwc = GQAWithCache(512, 8, 2).cuda()
    torch.manual_seed(3)
    cg = CachedGQA(512, 8, 2).cuda()
    cache = KVCache.create(2, 64, 2, 64, torch.device("cuda"), torch.float32)
    lc = LayerKVCache(k=torch.zeros(2, 64, 2, 64, device="cuda"),
                      v=torch.zeros(2, 64, 2, 64, device="cuda"))
    pos = 0
    with torch.no_grad():
        for i, (shape, seed) in enumerate([((2, 40), 42), ((2, 1), 43), ((2, 1), 44), ((2, 3), 45)]):
            x = torch.from_numpy(seeded_normal((*shape, 512), seed)).cuda()
            np.testing.assert_allclose(gwc(x, kv_cache=cache)[0].cpu().numpy(), g[f"gwc_step{i}"],
                                       rtol=1e-3, atol=1e-3)
            np.testing.assert_allclose(cg(x, cache=lc, start_pos=pos).cpu().numpy(),
                                       g[f"cg_step{i}"], rtol=1e-3, atol=1e-3)
            pos += shape[1]


def test_cached_model_bf16_decode_tracks_fp32():
    """A bf16 model on the decode kernel follows the fp32 CPU model through a
    prompt and 8 decode steps (same weights, same tokens)."""
    from ch02 import CachedTransformerModel
    torch.manual_seed(0)
    cpu = CachedTransformerModel(1000, 512, 2, 8, 2, 1024)
    gpu = CachedTransformerModel(1000, 512, 2, 8, 2, 1024)
    gpu.load_state_dict(cpu.state_dict())
    gpu = gpu.cuda().bfloat16()
    cc = cpu.create_caches(2, 64, torch.device("cpu"), torch.float32)
    gc = gpu.create_caches(2, 64, torch.device("cuda"), torch.bfloat16)
    ids = torch.randint(0, 1000, (2, 24))
    with torch.no_grad():
        steps = [ids] + [torch.randint(0, 1000, (2, 1)) for _ in range(8)]
        pos = 0
        for t in steps:
            a = cpu(t, cc, start_pos=pos)
            b = gpu(t.cuda(), gc, start_pos=pos).float().cpu()
            pos += t.shape[1]
            rel = (a - b).norm() / a.norm()
            assert rel < 3e-2, float(rel)
    assert all(c.seq_len == 32 for c in gc)
