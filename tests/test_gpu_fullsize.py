"""Every kernel variant the dispatch tables can select, at the BASELINE /
bench sizes (not only the small parity cases): GEMM tile variants at 4096^3
(NN, NT) and 8192^3 NT, GEMV variants at 4096^2 and a 32000 x 4096 LM head,
decode-attention modes at the bench's 1 GiB cache.  The oracle is the f64
restatement on sampled rows / (batch, head) pairs, so each case stays within
seconds of host time."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import attention as oatt
from oracle import linear as olin
from oracle.numerics import seeded_normal

pytestmark = pytest.mark.gpu
DEV = "cuda"
LIN_TOL = {"fp16": 4e-3, "bf16": 1e-2}


def _bf16(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV).to(torch.bfloat16)


def _rows_close(out_rows, ref, what):
    out = out_rows.astype(np.float64)
    bound = LIN_TOL["bf16"] * (np.abs(ref) + 1.0)
    bad = np.abs(out - ref) > bound
    assert not bad.any(), f"{what}: {bad.sum()} elements beyond tol, max err {np.abs(out - ref).max():.3e}"


@pytest.fixture(scope="module")
def gemm4096():
    a = seeded_normal((4096, 4096), 61, "bf16")
    b = seeded_normal((4096, 4096), 62, "bf16")
    return a, b, _bf16(a), _bf16(b)


# 1: 128^2 tile, 2: 256^2 one-phase, 3: phased SCHED 0, 4: setprio, 5-8:
# phased SCHED 1/3/5/7, 9-11: grouped one-phase, 12-15: grouped phased,
# 40: gemm_w4v, 41: gemm_w5, 43: gemm_w5 persistent (41 / 43: the large-shape defaults since round 3)
@pytest.mark.parametrize("variant", [None, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 40, 41, 43])
@pytest.mark.parametrize("tb", [False, True])
def test_gemm_variants_4096_cube(gemm4096, variant, tb):
    import pli_hip
    a, b, da, db = gemm4096
    c = pli_hip.gemm(da, db, trans_b=tb, variant=variant).float().cpu().numpy()
    rows = np.random.RandomState(variant or 0).choice(4096, 24, replace=False)
    ref = olin.linear(a[rows], b) if tb else olin.gemm(a[rows], b)
    _rows_close(c[rows], ref, f"4096^3 tb={tb} v{variant}")


@pytest.mark.parametrize("variant", [None, 3, 7, 9, 13, 40, 41, 43])
def test_gemm_variants_8192_cube_nt(variant):
    """The ch09 TP=1 shape of the bench (x [8192, 8192] . W^T)."""
    import pli_hip
    x = seeded_normal((8192, 8192), 63, "bf16")
    w = seeded_normal((8192, 8192), 64, "bf16") * np.float32(8192 ** -0.5)
    from oracle.numerics import round_to_bf16
    w = round_to_bf16(w)
    y = pli_hip.gemm(_bf16(x), _bf16(w), trans_b=True, variant=variant).float().cpu().numpy()
    rows = np.random.RandomState(7).choice(8192, 16, replace=False)
    _rows_close(y[rows], olin.linear(x[rows], w), f"8192^3 NT v{variant}")


@pytest.mark.parametrize("variant", [None] + list(range(17)))
@pytest.mark.parametrize("m,k", [(4096, 4096), (32000, 4096)])
def test_gemv_variants_full_size(variant, m, k):
    import pli_hip
    w = seeded_normal((m, k), 65, "bf16") * np.float32(k ** -0.5)
    from oracle.numerics import round_to_bf16
    w = round_to_bf16(w)
    x = seeded_normal((k,), 66, "bf16")
    y = pli_hip.gemv(_bf16(w), _bf16(x), variant=variant).float().cpu().numpy()
    _rows_close(y, olin.gemv(w, x), f"gemv {m}x{k} v{variant}")


@pytest.mark.parametrize("mode", [None, 2, 9, 11, 13])
def test_decode_modes_bench_config(mode):
    """bench.py's decode attention: B=8, Hq=32, Hkv=8, one new token over a
    32768-token bf16 cache (1 GiB); (batch, head) pairs 0/0, 3/17, 7/31 vs f64."""
    import pli_hip
    B, H, Hkv, S, D = 8, 32, 8, 32768, 128
    g = torch.Generator(device=DEV).manual_seed(11)
    q = torch.randn(B, 1, H, D, device=DEV, dtype=torch.bfloat16, generator=g)
    kc = torch.randn(B, S, Hkv, D, device=DEV, dtype=torch.bfloat16, generator=g)
    vc = torch.randn(B, S, Hkv, D, device=DEV, dtype=torch.bfloat16, generator=g)
    out = pli_hip.attn_decode(q, kc, vc, S, causal=False, variant=mode).float().cpu().numpy()
    for b, h in ((0, 0), (3, 17), (7, 31)):
        hk = h // (H // Hkv)
        qq = q[b, :, h].float().cpu().numpy()[None, None]
        kk = kc[b, :, hk].float().cpu().numpy()[None, None]
        vv = vc[b, :, hk].float().cpu().numpy()[None, None]
        ref = oatt.naive_attention(qq, kk, vv)[0, 0]
        err = np.abs(out[b, :, h] - ref).max()
        assert err <= 1e-2, f"mode {mode} (b{b}, h{h}): max |err| {err:.3e}"
