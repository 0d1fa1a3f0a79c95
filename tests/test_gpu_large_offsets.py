"""Operands whose byte extents cross 2^31 / 2^32 (huge strides, small compute):
the kernels address a head's rows / a tile's rows by 32-bit per-lane offsets
from a 64-bit base, and each fast route states the extent it takes
(flash_v13.hip attn_v13_ok: a Q / O head's rows below 2^32 bytes; gemm_w5.hip:
256 rows of A / B below 2^31 bytes); past that the dispatch must fall back to a
kernel that is still correct.  Every case runs once just inside and once just
outside such a bound and is checked against fp32 torch math on contiguous
copies of the same data (1e-2 absolute for attention on randn inputs, 2^-7
relative to the row scale for the bf16 GEMM / GEMV outputs)."""
from __future__ import annotations

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
MB2 = 1 << 20  # row stride in elements: 2 MiB per bf16 row


def big_rows(n, h, d, dtype=torch.bfloat16, seed=0):
    """[1, h, n, d] view whose rows sit 2 MiB apart ([n, h, 2^20 / h] storage)"""
    g = torch.Generator(device=DEV).manual_seed(seed)
    s = torch.empty(n, h, MB2 // h, device=DEV, dtype=dtype)
    s[:, :, :d] = torch.randn(n, h, d, device=DEV, dtype=torch.float32, generator=g).to(dtype)
    return s[:, :, :d].permute(1, 0, 2).unsqueeze(0)


def attn_ref(q, k, v, causal):
    s = (q.float() @ k.float().transpose(-1, -2).repeat_interleave(q.shape[1] // k.shape[1], 1)) * q.shape[-1] ** -0.5
    if causal:
        nq, nk = s.shape[-2:]
        s = s.masked_fill(torch.ones(nq, nk, dtype=torch.bool, device=DEV).triu(nk - nq + 1), float("-inf"))
    return torch.softmax(s, -1) @ v.float().repeat_interleave(q.shape[1] // k.shape[1], 1)


# Nq rows at 2 MiB: 1500 -> 2.9 GiB of Q / O rows (v13, offsets past 2^31),
# 2100 -> 4.1 GiB (past v13's 2^32 bound: the fallback route)
@pytest.mark.parametrize("causal", (False, True))
@pytest.mark.parametrize("nq,d,dtype", [(1500, 128, torch.bfloat16), (2100, 128, torch.bfloat16),
                                        (1500, 64, torch.float16)])
def test_flash_rows_past_2g(nq, d, dtype, causal):
    import pli_hip
    q = big_rows(nq, 2, d, dtype, seed=1)
    o = big_rows(nq, 2, d, dtype, seed=2)
    g = torch.Generator(device=DEV).manual_seed(3)
    nk = nq + 37
    k = torch.randn(1, 1, nk, d, device=DEV, generator=g).to(dtype)
    v = torch.randn(1, 1, nk, d, device=DEV, generator=g).to(dtype)
    out = pli_hip.flash_attn_fwd(q, k, v, causal=causal, out=o)
    assert out.data_ptr() == o.data_ptr()
    # Nk = Nq + 37 (ragged): the v13 ragged bodies inside the 2^32 bound, v7 / v10 past it
    want = ("attn_fwd_v13" + ("h" if dtype == torch.float16 else "") + ("rc" if causal else "r") +
            ("_d64" if d == 64 else "")) if nq < 2048 else "attn_fwd_v7"
    assert pli_hip.last_route() == want
    ref = attn_ref(q.contiguous(), k, v, causal)
    err = (out.float() - ref).abs().max().item()
    assert err <= 1e-2, f"Nq {nq} D {d} causal {causal}: max |err| {err:.3e}"
    del q, o


def gemm_check(c, ref):
    scale = ref.abs().amax(dim=1, keepdim=True).clamp_min(1e-3)
    err = ((c.float() - ref).abs() / scale).max().item()
    assert err <= 2.0 ** -7, f"max rel err {err:.3e}"


# A [512, 128] at row stride lda: a tile's 256 rows x lda x 2 B against
# gemm_w5's 2^31 (M 512 x N 16384: the 128 tiles of 256^2 its default route needs)
@pytest.mark.parametrize("lda", ((1 << 22) - 64, (1 << 22) + 64))
@pytest.mark.parametrize("trans_b", (False, True))
def test_gemm_a_rows_past_2g(lda, trans_b):
    import pli_hip
    g = torch.Generator(device=DEV).manual_seed(5)
    s = torch.empty(512, lda, device=DEV, dtype=torch.bfloat16)
    s[:, :128] = torch.randn(512, 128, device=DEV, generator=g).to(torch.bfloat16)
    a = s[:, :128]
    n = 16384
    b = torch.randn(n, 128, device=DEV, generator=g).to(torch.bfloat16)
    if trans_b:
        c = pli_hip.gemm(a, b, trans_b=True)
        ref = a.float() @ b.float().t()
    else:
        bt = b.t().contiguous()
        c = pli_hip.gemm(a, bt)
        ref = a.float() @ bt.float()
    assert (pli_hip.last_route() == "gemm_w5") == (lda < (1 << 22)), pli_hip.last_route()
    gemm_check(c, ref)


# NN B [128, 32768] at row stride ldb: 64 k-rows x ldb x 2 B against 2^31 (M 512)
@pytest.mark.parametrize("ldb", ((1 << 24) - 64, (1 << 24) + 64))
def test_gemm_nn_b_rows_past_2g(ldb):
    import pli_hip
    g = torch.Generator(device=DEV).manual_seed(6)
    n = 32768
    s = torch.empty(128, ldb, device=DEV, dtype=torch.bfloat16)
    s[:, :n] = torch.randn(128, n, device=DEV, generator=g).to(torch.bfloat16)
    b = s[:, :n]
    a = torch.randn(512, 128, device=DEV, generator=g).to(torch.bfloat16)
    c = pli_hip.gemm(a, b)
    assert (pli_hip.last_route() == "gemm_w5") == (ldb < (1 << 24)), pli_hip.last_route()
    gemm_check(c, a.float() @ b.float())


def test_gemv_rows_past_4g():
    """W [2304, 4096] at 2 MiB rows: 4.5 GiB between the first and last row"""
    import pli_hip
    g = torch.Generator(device=DEV).manual_seed(7)
    m, k = 2304, 4096
    s = torch.empty(m, MB2, device=DEV, dtype=torch.bfloat16)
    s[:, :k] = torch.randn(m, k, device=DEV, generator=g).to(torch.bfloat16)
    w = s[:, :k]
    x = torch.randn(k, device=DEV, generator=g).to(torch.bfloat16)
    y = pli_hip.gemv(w, x)
    ref = w.float() @ x.float()
    err = ((y.float() - ref).abs() / ref.abs().max()).max().item()
    assert err <= 2.0 ** -7, f"max rel err {err:.3e}"


def test_decode_cache_batches_past_2g():
    """[B, S_max, Hkv, D] caches with 2^20 positions: batch b starts at b x 2
    GiB; 5000 valid keys, the last batch past 4 GiB"""
    import pli_hip
    g = torch.Generator(device=DEV).manual_seed(8)
    B, S, Hkv, D, n_kv = 3, 1 << 20, 8, 128, 5000
    kc = torch.empty(B, S, Hkv, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.empty_like(kc)
    kc[:, :n_kv] = torch.randn(B, n_kv, Hkv, D, device=DEV, generator=g).to(torch.bfloat16)
    vc[:, :n_kv] = torch.randn(B, n_kv, Hkv, D, device=DEV, generator=g).to(torch.bfloat16)
    q = torch.randn(B, 1, 32, D, device=DEV, generator=g).to(torch.bfloat16)
    out = pli_hip.attn_decode(q, kc, vc, n_kv)
    kk = kc[:, :n_kv].permute(0, 2, 1, 3)
    vv = vc[:, :n_kv].permute(0, 2, 1, 3)
    ref = attn_ref(q.permute(0, 2, 1, 3), kk, vv, False).permute(0, 2, 1, 3)
    err = (out.float() - ref).abs().max().item()
    assert err <= 1e-2, f"max |err| {err:.3e}"


def sampled_ref(q, k, v, rows, causal):
    """fp32 attention of the given query rows only (each row over all keys)"""
    G = q.shape[1] // k.shape[1]
    nq, nk = q.shape[2], k.shape[2]
    qs = q[:, :, rows].float()
    kf = k.float().repeat_interleave(G, 1)
    s = (qs @ kf.transpose(-1, -2)) * q.shape[-1] ** -0.5
    if causal:
        lim = rows.to(DEV)[:, None] + (nk - nq)
        s = s.masked_fill(torch.arange(nk, device=DEV)[None, :] > lim, float("-inf"))
    return torch.softmax(s, -1) @ v.float().repeat_interleave(G, 1)


# long prefill on the v13 programs (whole and ragged key tiles, causal, fp16 D64)
@pytest.mark.parametrize("shape,dtype,causal", [
    ((1, 4, 1, 32768, 32768, 128), torch.bfloat16, False),
    ((1, 4, 1, 32768, 32768, 128), torch.bfloat16, True),
    ((1, 4, 2, 32813, 32813, 128), torch.bfloat16, True),
    ((1, 2, 2, 65536, 65536, 64), torch.float16, False),
    ((1, 2, 1, 65536 + 7, 65536 + 7, 64), torch.float16, True),
], ids=lambda p: str(p) if not isinstance(p, tuple) else "b{}h{}kv{}q{}k{}d{}".format(*p))
def test_flash_long_sequences(shape, dtype, causal):
    import pli_hip
    B, H, Hkv, Nq, Nk, D = shape
    g = torch.Generator(device=DEV).manual_seed(sum(shape))
    q = torch.randn(B, H, Nq, D, device=DEV, generator=g).to(dtype)
    k = torch.randn(B, Hkv, Nk, D, device=DEV, generator=g).to(dtype)
    v = torch.randn(B, Hkv, Nk, D, device=DEV, generator=g).to(dtype)
    out = pli_hip.flash_attn_fwd(q, k, v, causal=causal)
    rows = torch.cat([torch.arange(0, 70), torch.randint(70, Nq - 70, (300,), generator=torch.Generator().manual_seed(1)),
                      torch.arange(Nq - 70, Nq)])
    ref = sampled_ref(q, k, v, rows, causal)
    err = (out[:, :, rows.to(DEV)].float() - ref).abs().max().item()
    assert err <= 1e-2, f"{shape} causal {causal}: max |err| {err:.3e}"


# a chunk of new rows over a cache-long key stream: the causal walk packs the
# key-tile count into 16 bits (flash_v13.hip attn_v13_ok: cdiv(Nk, 64) <=
# 0xFFFF), so 65535 tiles run v13 and one tile more the fallback
@pytest.mark.parametrize("causal", (False, True))
@pytest.mark.parametrize("nk", (65535 * 64, 65535 * 64 + 64, 65535 * 64 - 13))
def test_flash_four_million_keys(nk, causal):
    import pli_hip
    g = torch.Generator(device=DEV).manual_seed(nk % 1000)
    q = torch.randn(1, 2, 128, 128, device=DEV, generator=g).to(torch.bfloat16)
    k = torch.randn(1, 1, nk, 128, device=DEV, generator=g).to(torch.bfloat16)
    v = torch.randn(1, 1, nk, 128, device=DEV, generator=g).to(torch.bfloat16)
    out = pli_hip.flash_attn_fwd(q, k, v, causal=causal)
    tiles = -(-nk // 64)
    want = "attn_fwd_v13" + ("rc" if causal and nk % 64 else "r" if nk % 64 else "c" if causal else "")
    if causal and tiles > 0xFFFF:
        want = "attn_fwd_v12"  # the causal v12 body (Nk % 64 == 0, bf16 D 128)
    assert pli_hip.last_route() == want
    rows = torch.arange(128)
    ref = sampled_ref(q, k, v, rows, causal)
    err = (out.float() - ref).abs().max().item()
    assert err <= 1e-2, f"Nk {nk} causal {causal}: max |err| {err:.3e}"
