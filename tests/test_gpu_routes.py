"""Which kernel each call runs (pli_last_route): the dispatch tables that
DESIGN.md §0 / §3 and include/pli.h state, checked on the device.  Flash:
csrc/flash_attn.hip launch_mfma -> attn_v13_ok (flash_v13.hip) -> v12
(attn_v12_ok) -> v7 / v10 -> the generic kernel; each routed call is also
checked against fp32 torch attention, so a route is only "taken" when its
result is right."""
from __future__ import annotations

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def v13(dtype, D, causal, ragged):
    return ("attn_fwd_v13" + ("h" if dtype == torch.float16 else "") +
            ("rc" if ragged and causal else "r" if ragged else "c" if causal else "") + ("_d64" if D == 64 else ""))


BF, FP = torch.bfloat16, torch.float16
# (B, H, Hkv, Nq, Nk, D, dtype, causal, expected route)
FLASH = [
    *[(2, 4, 2, 256, 256, D, dt, c, v13(dt, D, c, False)) for D in (128, 64) for dt in (BF, FP) for c in (False, True)],
    *[(2, 4, 2, 200, 200, D, dt, c, v13(dt, D, c, True)) for D in (128, 64) for dt in (BF, FP) for c in (False, True)],
    (1, 8, 8, 128, 1024, 128, BF, True, "attn_fwd_v13c"),      # chunked prefill, offset 896
    (1, 8, 8, 100, 1000, 128, BF, True, "attn_fwd_v13rc"),     # offset 900, ragged
    (1, 8, 2, 1, 777, 64, FP, True, "attn_fwd_v13hrc_d64"),    # one query row
    (2, 4, 4, 64, 64, 128, BF, False, "attn_fwd_v12"),          # Nk = 64: v12
    (2, 4, 4, 64, 64, 128, BF, True, "attn_fwd_v12"),
    (2, 4, 4, 64, 64, 128, FP, False, "attn_fwd_v7"),           # v12 is bf16 only
    (2, 4, 4, 40, 40, 128, BF, False, "attn_fwd_v7"),           # Nk < 64
    (2, 4, 4, 300, 200, 128, BF, True, "attn_fwd_v7"),          # causal Nq > Nk
    (2, 4, 4, 128, 256, 96, BF, False, "attn_fwd_generic"),     # head dim 96
    (2, 4, 4, 128, 256, 128, torch.float32, False, "attn_fwd_generic"),
    (2, 4, 4, 128, 0, 128, BF, False, "attn_fwd_generic"),      # no keys: O = 0
]


@pytest.mark.parametrize("case", FLASH, ids=lambda c: "b{}h{}kv{}q{}k{}d{}-{}-causal{}".format(
    *c[:6], str(c[6]).split(".")[-1], int(c[7])))
def test_flash_route(case):
    import pli_hip
    B, H, Hkv, Nq, Nk, D, dt, causal, want = case
    g = torch.Generator(device=DEV).manual_seed(Nq + Nk + D)
    q = torch.randn(B, H, Nq, D, device=DEV, generator=g).to(dt)
    k = torch.randn(B, Hkv, Nk, D, device=DEV, generator=g).to(dt)
    v = torch.randn(B, Hkv, Nk, D, device=DEV, generator=g).to(dt)
    out = pli_hip.flash_attn_fwd(q, k, v, causal=causal)
    assert pli_hip.last_route() == want
    G = H // Hkv
    s = (q.float() @ k.float().repeat_interleave(G, 1).transpose(-1, -2)) * D ** -0.5
    if causal:
        s = s.masked_fill(torch.ones(Nq, Nk, dtype=torch.bool, device=DEV).triu(Nk - Nq + 1), float("-inf"))
    ref = torch.softmax(s, -1) @ v.float().repeat_interleave(G, 1) if Nk else torch.zeros_like(q, dtype=torch.float32)
    ref = torch.nan_to_num(ref)  # (causal Nq > Nk: rows with no key are 0 here and NaN in torch)
    assert (out.float() - ref).abs().max().item() <= 1e-2


def test_gemm_and_decode_routes():
    import pli_hip
    g = torch.Generator(device=DEV).manual_seed(3)
    a = torch.randn(4096, 4096, device=DEV, generator=g).to(BF)
    b = torch.randn(4096, 4096, device=DEV, generator=g).to(BF)
    pli_hip.gemm(a, b)
    assert pli_hip.last_route() == "gemm_w5"                      # 4096^3 NN: the 256^2 one-wave-per-SIMD tile
    pli_hip.gemm(a[:1], b, trans_b=True)
    assert pli_hip.last_route() == "gemv_vec"                     # M = 1, no bias: the GEMV
    x = torch.randn(8, 4096, device=DEV, generator=g).to(BF)
    pli_hip.gemm(x, b, trans_b=True, bias=b[0])
    assert pli_hip.last_route() in ("gemm_smallm_nt", "gemm_skinny_nt")
    f = torch.randn(2048, 2048, device=DEV, generator=g)
    pli_hip.gemm(f, f)
    assert pli_hip.last_route() == "gemm_f32_mfma"
    pli_hip.gemm(a[:, :0], b[:0])
    assert pli_hip.last_route() == "gemm_generic"                 # K = 0: C = 0
    pli_hip.gemm(a[:0], b)
    assert pli_hip.last_route() == ""                             # empty output: nothing launched
    pli_hip.gemv(a, a[0])
    assert pli_hip.last_route() == "gemv_vec"
    q = torch.randn(8, 1, 32, 128, device=DEV, generator=g).to(BF)
    kc = torch.randn(8, 32768, 8, 128, device=DEV, generator=g).to(BF)
    pli_hip.attn_decode(q, kc, kc, 32768)
    assert pli_hip.last_route() == "attn_decode_chunk+attn_decode_combine"
    pli_hip.attn_decode(q, kc, kc, 0)
    assert pli_hip.last_route() == "attn_fwd_generic"             # empty cache: O = 0


# (M, N, K, trans_b, bias, expected route or prefix): csrc/gemm.hip gemm_dispatch
# through the Python wrapper (which passes a split-K workspace when one is needed)
GEMM = [
    (1, 4096, 4096, True, True, "gemm_skinny_nt"),                          # M = 1 with a bias
    (16, 2048, 2048, True, False, "gemm_smallm_nt"),                        # short K, M <= 32
    (64, 8192, 1024, True, False, "gemm_midm_nt"),                          # the TP-8 row shard at M 64
    (128, 8192, 8192, True, False, "gemm_splitk_lds_nt+gemm_splitk_reduce"),  # decode batch, deep K
    (1024, 4096, 4096, True, False, "gemm_splitk_lds_nt"),                  # few tiles: 128-row slabs
    (384, 384, 256, False, False, "gemm_mfma"),                             # below the 2 x 2 grid of 256^2
    (8192, 8192, 1024, True, False, "gemm_w5"),                             # 1024 tiles
    (4096, 4096, 4096, False, True, "gemm_w5"),                             # NN with a bias
]


@pytest.mark.parametrize("case", GEMM, ids=lambda c: "m{}n{}k{}-nt{}-bias{}".format(*c[:5]))
def test_gemm_route(case):
    import pli_hip
    M, N, K, nt, bias, want = case
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    a = torch.randn(M, K, device=DEV, generator=g).to(BF)
    b = torch.randn(N, K, device=DEV, generator=g).to(BF) if nt else torch.randn(K, N, device=DEV, generator=g).to(BF)
    bi = torch.randn(N, device=DEV, generator=g).to(BF) if bias else None
    c = pli_hip.gemm(a, b, trans_b=nt, bias=bi)
    route = pli_hip.last_route()
    assert route == want or (want.endswith("_nt") and route.startswith(want + "+")), route
    ref = a.float() @ (b.float().t() if nt else b.float()) + (bi.float() if bias else 0)
    scale = ref.abs().amax(dim=1, keepdim=True).clamp_min(1e-3)
    assert ((c.float() - ref).abs() / scale).max().item() <= 2.0 ** -7
