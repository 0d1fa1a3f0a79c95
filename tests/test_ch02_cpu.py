"""CPU checks of the GQA / KV-cache mirrors against fixtures made by the
reference itself (tests/golden/make_golden.py: gqa.npz, kv_cache.json).

The mirrors must build the reference's weights from the same seed (parameter
names, shapes and creation order), append to the cache exactly as the
reference does, and -- on CPU, where they keep the reference math -- give its
outputs for a prompt, single-token decode steps and a 3-token chunk.  The
restated assertions of the reference's own ch02 tests
(ch02/test_ch02.py:21-205) are at the bottom; that file itself imports
ch01.transformer (out of scope), so it is not run unmodified.
"""
from __future__ import annotations

import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_golden
from oracle.numerics import array_hash, seeded_normal

HIDDEN, HEADS, KV = 512, 8, 2
STEPS = [((2, 40), 42), ((2, 1), 43), ((2, 1), 44), ((2, 3), 45)]


@pytest.fixture(scope="module")
def g():
    return load_golden("gqa.npz")


def _hashes(mod, prefix, g):
    for n, p in mod.named_parameters():
        assert array_hash(p.detach().numpy()) == str(g[f"{prefix}_hash_{n}"]), n


def test_gqa_mirror_matches_reference(g):
    from ch01 import GroupedQueryAttention
    torch.manual_seed(1)
    m = GroupedQueryAttention(HIDDEN, HEADS, KV)
    _hashes(m, "gqa", g)
    x = torch.from_numpy(seeded_normal((1, 64, HIDDEN), 41))
    with torch.no_grad():
        np.testing.assert_allclose(m(x, causal=True).numpy(), g["gqa_causal"], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(m(x, causal=False).numpy(), g["gqa_noncausal"], rtol=1e-5,
                                   atol=1e-5)
    assert m.kv_cache_size_per_token() == 2 * KV * 64 * 2


def test_cached_modules_match_reference_stream(g):
    from ch02 import CachedGQA, GQAWithCache, KVCache, LayerKVCache
    torch.manual_seed(2)
    gwc = GQAWithCache(HIDDEN, HEADS, KV)
    torch.manual_seed(3)
    cg = CachedGQA(HIDDEN, HEADS, KV)
    _hashes(gwc, "gwc", g)
    _hashes(cg, "cg", g)
    hd = HIDDEN // HEADS
    cache = KVCache.create(2, 64, KV, hd, torch.device("cpu"), torch.float32)
    lc = LayerKVCache(k=torch.zeros(2, 64, KV, hd), v=torch.zeros(2, 64, KV, hd), seq_len=0)
    pos = 0
    with torch.no_grad():
        for i, (shape, seed) in enumerate(STEPS):
            x = torch.from_numpy(seeded_normal((*shape, HIDDEN), seed))
            y, ret = gwc(x, kv_cache=cache)
            assert ret is cache
            np.testing.assert_allclose(y.numpy(), g[f"gwc_step{i}"], rtol=1e-5, atol=1e-5)
            np.testing.assert_allclose(cg(x, cache=lc, start_pos=pos).numpy(), g[f"cg_step{i}"],
                                       rtol=1e-5, atol=1e-5)
            pos += shape[1]
        y0, none = gwc(torch.from_numpy(seeded_normal((2, 40, HIDDEN), 42)), kv_cache=None)
        assert none is None
        np.testing.assert_allclose(y0.numpy(), g["gwc_nocache"], rtol=1e-5, atol=1e-5)
    assert [cache.seq_len, lc.seq_len] == list(g["cache_len"])


def test_calculate_kv_cache_size_matches_reference():
    from ch02 import calculate_kv_cache_size
    with open(os.path.join(GOLDEN, "kv_cache.json")) as f:
        rows = json.load(f)
    for args, want in rows:
        got = calculate_kv_cache_size(*args[:5], dtype=getattr(torch, args[5]))
        assert got == want, args


# ---- restated from the reference's ch02/test_ch02.py (shapes / cache lengths)
def test_reference_ch02_contracts():
    from ch02 import (CachedGQA, CachedTransformerModel, GQAWithCache, KVCache, LayerKVCache,
                      cached_generate)
    c = KVCache.create(2, 100, 4, 64, torch.device("cpu"), torch.float32)
    assert c.k_cache.shape == (2, 100, 4, 64) and c.seq_len == 0
    k, v = torch.randn(2, 10, 4, 64), torch.randn(2, 10, 4, 64)
    kf, vf = c.update(k, v)
    assert kf.shape == (2, 10, 4, 64) and c.seq_len == 10 and torch.equal(kf, k)
    kf, _ = c.update(torch.randn(2, 1, 4, 64), torch.randn(2, 1, 4, 64))
    assert kf.shape == (2, 11, 4, 64)
    assert c.memory_bytes() == 2 * 100 * 4 * 64 * 4 * 2
    lc = LayerKVCache(k=torch.zeros(2, 50, 2, 32), v=torch.zeros(2, 50, 2, 32))
    kf, _ = lc.update(torch.ones(2, 5, 2, 32), torch.ones(2, 5, 2, 32))
    assert kf.shape == (2, 5, 2, 32) and lc.seq_len == 5
    attn = GQAWithCache(hidden_dim=256, num_heads=8, num_kv_heads=2)
    assert attn(torch.randn(2, 1, 256), kv_cache=None)[0].shape == (2, 1, 256)
    cg = CachedGQA(hidden_dim=256, num_heads=8, num_kv_heads=2)
    cache = LayerKVCache(k=torch.zeros(2, 100, 2, 32), v=torch.zeros(2, 100, 2, 32))
    cg(torch.randn(2, 10, 256), cache=cache, start_pos=0)
    assert cg(torch.randn(2, 1, 256), cache=cache, start_pos=10).shape == (2, 1, 256)
    assert cache.seq_len == 11
    model = CachedTransformerModel(1000, 256, 2, 8, 2, 512)
    caches = model.create_caches(2, 100, torch.device("cpu"), torch.float32)
    assert model(torch.randint(0, 1000, (2, 10)), caches=caches).shape == (2, 10, 1000)
    assert model(torch.randint(0, 1000, (2, 1)), caches=caches, start_pos=10).shape == (2, 1, 1000)
    assert all(c.seq_len == 11 for c in caches)
    ids = torch.randint(0, 1000, (1, 5))
    out, t = cached_generate(model, ids, max_new_tokens=10)
    assert out.shape == (1, 15) and torch.equal(out[:, :5], ids)
    assert len(t["decode_ms"]) == 9 and t["total_ms"] >= t["prefill_ms"]


def test_ch08_graph_runner_without_gpu():
    """The reference's CUDAGraphRunner contract on a host without a device:
    capture reports False, run_graph None (ch08/cuda_graph.py:37-41, 69-70)."""
    from ch08 import CUDAGraphRunner, GraphConfig
    cfg = GraphConfig()
    assert cfg.batch_sizes == [1, 2, 4, 8, 16, 32] and cfg.max_seq_len == 2048
    r = CUDAGraphRunner(cfg, model_fn=lambda x: x)
    if not torch.cuda.is_available():
        assert r.capture_graph(1, (8,)) is False
    assert r.run_graph(3, torch.zeros(3, 8)) is None and r.get_captured_batch_sizes() in ([], [1])
