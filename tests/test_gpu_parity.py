"""GPU parity: the HIP kernels (through the C ABI) against the pinned oracle.

Tolerances (north_star): 1e-3 for fp32, 1e-2 for bf16/fp16 outputs of the
attention path, measured against the float64 oracle on the same rounded
inputs.  GEMV/GEMM outputs grow like sqrt(K), so their bound is relative:
|err| <= tol * (|ref| + 1) with the per-dtype tol below (output rounding to
bf16 alone is 2^-9 relative).
"""
from __future__ import annotations

import glob
import os
import zlib

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_golden
from oracle import attention as oatt
from oracle import linear as olin
from oracle.numerics import bf16_from_bits, seeded_normal
from stress_cases import STRESS, prescaled_q, stress_inputs

pytestmark = pytest.mark.gpu

TDT = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}
ATTN_TOL = {"fp32": 1e-3, "fp16": 1e-2, "bf16": 1e-2}
LIN_TOL = {"fp32": 1e-4, "fp16": 4e-3, "bf16": 1e-2}
DEV = "cuda"


def dev(a, dt):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV).to(TDT[dt])


def assert_attn_close(out, ref, dt, what=""):
    out = out.float().cpu().numpy().astype(np.float64)
    err = np.abs(out - ref).max()
    assert np.isfinite(out).all(), f"{what}: non-finite output"
    assert err <= ATTN_TOL[dt], f"{what}: max |err| {err:.3e} > {ATTN_TOL[dt]}"
    return err


def assert_lin_close(out, ref, dt, what=""):
    out = out.float().cpu().numpy().astype(np.float64)
    bound = LIN_TOL[dt] * (np.abs(ref) + 1.0)
    bad = np.abs(out - ref) > bound
    assert not bad.any(), f"{what}: {bad.sum()} elements beyond tol, max err {np.abs(out - ref).max():.3e}"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    import pli_hip
    assert pli_hip.available(), "libpli_hip.so must load on the GPU box"
    yield


# ------------------------------------------------------------- attention ---
@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "flash_*.npz"))),
                         ids=os.path.basename)
def test_flash_golden(path):
    """HIP flash vs the reference naive attention in f64 (fixture), and no
    worse than the reference's own flash output."""
    from ch06 import flash_attention_forward
    g = load_golden(os.path.basename(path))
    B, H, N, D = (int(x) for x in g["shape"])
    dt, seed = str(g["dtype"]), int(g["seed"])
    q, k, v = (seeded_normal((B, H, N, D), seed * 10 + i, dt) for i in range(3))
    out = flash_attention_forward(dev(q, dt), dev(k, dt), dev(v, dt))
    assert out.dtype == TDT[dt] and tuple(out.shape) == (B, H, N, D)
    ref = g["ref_naive_f64"].astype(np.float64)
    err = assert_attn_close(out, ref, dt, os.path.basename(path))
    ref_flash = bf16_from_bits(g["ref_flash"]) if dt == "bf16" else g["ref_flash"].astype(np.float32)
    assert err <= np.abs(ref_flash - ref).max() + ATTN_TOL[dt] / 2


CASES = [
    # B, H, Hkv, Nq, Nk, D, dtype, causal
    (1, 4, 4, 1024, 1024, 128, "bf16", False),
    (2, 4, 4, 333, 333, 128, "bf16", False),
    (1, 3, 3, 257, 257, 64, "fp16", False),
    (2, 4, 4, 256, 256, 128, "bf16", True),
    (1, 2, 2, 200, 200, 64, "bf16", True),
    (1, 8, 2, 384, 384, 128, "bf16", True),    # GQA 4:1
    (1, 8, 2, 130, 130, 64, "fp16", False),    # GQA, ragged
    (1, 4, 4, 64, 300, 128, "bf16", True),     # Nq < Nk: bottom-right causal
    (1, 2, 2, 1, 77, 64, "bf16", False),       # single query row
    (1, 2, 2, 100, 100, 32, "fp32", True),     # generic kernel, odd head_dim
    (1, 2, 2, 150, 150, 128, "fp32", False),
    (1, 2, 2, 96, 96, 80, "bf16", False),      # generic kernel for bf16 (D=80)
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "b{}h{}kv{}q{}k{}d{}_{}{}".format(*c[:7], "_causal" if c[7] else ""))
def test_flash_vs_oracle(case):
    import pli_hip
    B, H, Hkv, Nq, Nk, D, dt, causal = case
    seed = zlib.crc32(repr(case).encode()) % 1000
    q = seeded_normal((B, H, Nq, D), seed, dt)
    k = seeded_normal((B, Hkv, Nk, D), seed + 1, dt)
    v = seeded_normal((B, Hkv, Nk, D), seed + 2, dt)
    out = pli_hip.flash_attn_fwd(dev(q, dt), dev(k, dt), dev(v, dt), causal=causal)
    ref = oatt.naive_attention(q, k, v, causal=causal)
    assert_attn_close(out, ref, dt, str(case))


# every MFMA variant (alternates A/B-tested by tools/tune.py) on the MFMA-eligible cases
MFMA_VARIANTS = (21, 50, 51, 54, 55, 60, 70, 71, 72, 73, 74, 80, 81, 82)



@pytest.mark.parametrize("variant", MFMA_VARIANTS)
@pytest.mark.parametrize("case", [c for c in CASES if c[6] != "fp32" and c[5] in (64, 128)],
                         ids=lambda c: "b{}h{}kv{}q{}k{}d{}_{}{}".format(*c[:7], "_causal" if c[7] else ""))
def test_flash_variants_vs_oracle(case, variant):
    import pli_hip
    B, H, Hkv, Nq, Nk, D, dt, causal = case
    seed = zlib.crc32(repr(case).encode()) % 1000
    q = seeded_normal((B, H, Nq, D), seed, dt)
    k = seeded_normal((B, Hkv, Nk, D), seed + 1, dt)
    v = seeded_normal((B, Hkv, Nk, D), seed + 2, dt)
    out = pli_hip.flash_attn_fwd(dev(q, dt), dev(k, dt), dev(v, dt), causal=causal, variant=variant)
    ref = oatt.naive_attention(q, k, v, causal=causal)
    assert_attn_close(out, ref, dt, f"{case} variant {variant}")

def test_flash_strided_views_and_out_param():
    """Non-contiguous [B,H,S,hd] views (the MHA layout) read/written in place."""
    import pli_hip
    B, S, H, D = 2, 192, 4, 128
    x = seeded_normal((3, B, S, H, D), 5, "bf16")
    t = dev(x, "bf16")
    q, k, v = (t[i].transpose(1, 2) for i in range(3))
    o = torch.empty(B, S, H, D, dtype=torch.bfloat16, device=DEV)
    pli_hip.flash_attn_fwd(q, k, v, causal=True, out=o.transpose(1, 2))
    ref = oatt.naive_attention(*(x[i].transpose(0, 2, 1, 3) for i in range(3)), causal=True)
    assert_attn_close(o.transpose(1, 2), ref, "bf16", "strided")


# variants whose Q is prescaled by scale*log2(e) and rounded to the 16-bit
# input type before the MFMA (the rest scale the f32 scores exactly)
PRESCALED = (50, 54)
DEFAULT_VARIANT = 80  # attn_fwd_v13 since round 4 (71 = v12 where v13 does not apply)


DEFAULT_CAUSAL_VARIANT = 83  # attn_fwd_v13c since round 4 (74 = v12 causal otherwise)


def test_flash_default_variants():
    import pli_hip
    q, k, v = (dev(x, "bf16") for x in stress_inputs("late"))
    assert torch.equal(pli_hip.flash_attn_fwd(q, k, v), pli_hip.flash_attn_fwd(q, k, v, variant=DEFAULT_VARIANT))
    assert torch.equal(pli_hip.flash_attn_fwd(q, k, v, causal=True),
                       pli_hip.flash_attn_fwd(q, k, v, causal=True, variant=DEFAULT_CAUSAL_VARIANT))


@pytest.mark.parametrize("variant", MFMA_VARIANTS)
@pytest.mark.parametrize("name", STRESS)
def test_flash_stress(variant, name):
    """Adversarial inputs (tests/stress_cases.py) that force the rescale
    branch at chosen tiles, underflow against a zero max, or rescale in many
    tiles.  Bound: 2^-8 * max|v| -- the bf16 rounding of the P weights fed to
    the PV MFMA (2^-9 relative) plus the bf16 rounding of the output (2^-9),
    each at most 2^-9 * max|v| when a few keys dominate a row (on random
    inputs the suite's 1e-2 holds with a wide margin; here every variant,
    the round-1 kernel included, lands near 1.0e-2).  Exact-scaling variants
    are held to that against the f64 oracle.  Prescaled variants are held to
    it against the f64 oracle given the same bf16-rounded Q*scale*log2(e) (the
    kernel's arithmetic, every branch included), and, against the exact
    answer, to no worse than the reference's own bf16 flash path on the same
    input (tests/golden/stress_flash.npz, recorded from the reference)."""
    import pli_hip
    q, k, v = stress_inputs(name)
    out = pli_hip.flash_attn_fwd(dev(q, "bf16"), dev(k, "bf16"), dev(v, "bf16"), variant=variant)
    o64 = out.float().cpu().numpy().astype(np.float64)
    assert np.isfinite(o64).all(), f"stress {name}: non-finite output"
    tol = 2.0 ** -8 * float(np.abs(v).max())
    exact = oatt.naive_attention(q, k, v)
    err = np.abs(o64 - exact).max()
    if variant in PRESCALED:
        own = np.abs(o64 - oatt.naive_attention(prescaled_q(q, q.shape[-1] ** -0.5), k, v)).max()
        assert own <= tol, f"stress {name} (prescaled oracle): {own:.3e} > {tol:.3e}"
        ref_err = float(load_golden("stress_flash.npz")[f"{name}_ref_err"])
        assert err <= ref_err, f"stress {name}: {err:.3e} > reference bf16 flash {ref_err:.3e}"
    else:
        assert err <= tol, f"stress {name}: {err:.3e} > {tol:.3e}"


@pytest.mark.parametrize("variant", [None, 21, 50, 51, 54, 55, 60, 70, 71, 81])
def test_flash_full_config_properties(variant):
    """B=8 S=4096 H=32 D=128 bf16 (the bench config): v = 1 gives exactly 1;
    two heads checked against the f64 oracle; key permutation invariance."""
    import pli_hip
    B, H, N, D = 8, 32, 4096, 128
    g = torch.Generator(device=DEV).manual_seed(0)
    q, k, v = (torch.randn(B, H, N, D, device=DEV, dtype=torch.bfloat16, generator=g) for _ in range(3))
    out = pli_hip.flash_attn_fwd(q, k, v, variant=variant)
    ones = pli_hip.flash_attn_fwd(q, k, torch.ones_like(v), variant=variant)
    assert (ones.float() - 1).abs().max().item() <= 2 ** -8  # one bf16 ulp below 1
    for (b, h) in ((0, 0), (3, 17), (7, 31)):
        ref = oatt.naive_attention(*(t[b:b + 1, h:h + 1].float().cpu().numpy() for t in (q, k, v)))
        assert_attn_close(out[b:b + 1, h:h + 1], ref, "bf16", f"full b{b} h{h}")
    perm = torch.randperm(N, device=DEV, generator=g)
    out_p = pli_hip.flash_attn_fwd(q[:, :2], k[:, :2, perm], v[:, :2, perm], variant=variant)
    assert (out_p.float() - out[:, :2].float()).abs().max().item() <= 1e-2
    # full-tensor agreement with the round-1 kernel (independent softmax code)
    if variant is None:
        base = pli_hip.flash_attn_fwd(q, k, v, variant=21)
        assert (base.float() - out.float()).abs().max().item() <= 1.6e-2
    # attn_fwd_v12 (70, 71) runs attn_fwd_v10's arithmetic in the same
    # order: bitwise equal to 55 over the whole tensor; the default (v13,
    # variant 80) and its one-block-per-workgroup form 81 bitwise equal
    if variant in (70, 71):
        assert torch.equal(out, pli_hip.flash_attn_fwd(q, k, v, variant=55))
    if variant in (None, 81):
        assert torch.equal(out, pli_hip.flash_attn_fwd(q, k, v, variant=80))


@pytest.mark.parametrize("shape", [(4, 16, 4, 2048, 1024), (4, 32, 8, 1024, 128), (4, 32, 8, 1024, 192),
                                   (3, 40, 8, 1000, 320), (2, 4, 1, 2048, 192)])
def test_flash_v12_persistent_seams(shape):
    """Variant 71 walks more than one block per workgroup once the grid
    exceeds one workgroup per CU; the K/V stream then crosses block seams
    (blocks of 2 and 3 tiles, ragged Nq, GQA).  Bitwise equal to 55 and to
    the non-persistent form 70; the rescale path forced by scaled-up Q."""
    import pli_hip
    B, H, Hkv, Nq, Nk = shape
    g = torch.Generator(device=DEV).manual_seed(sum(shape))
    q = torch.randn(B, H, Nq, 128, device=DEV, dtype=torch.bfloat16, generator=g)
    k = torch.randn(B, Hkv, Nk, 128, device=DEV, dtype=torch.bfloat16, generator=g)
    v = torch.randn(B, Hkv, Nk, 128, device=DEV, dtype=torch.bfloat16, generator=g)
    for qq in (q, q * 4):
        a = pli_hip.flash_attn_fwd(qq, k, v, variant=55)
        assert torch.equal(a, pli_hip.flash_attn_fwd(qq, k, v, variant=71)), f"{shape}: 71 != 55"
        assert torch.equal(a, pli_hip.flash_attn_fwd(qq, k, v, variant=70)), f"{shape}: 70 != 55"


@pytest.mark.parametrize("variant", [None, 55, 21])
def test_flash_full_config_causal(variant):
    """Causal at the bench config (the ch01 MHA / GQA semantics): rows 0,
    1000 and 4095 of three heads against the f64 oracle (row i sees keys
    0..i), v = 1 gives 1, and the default agrees with the 8-wave kernel."""
    import pli_hip
    B, H, N, D = 8, 32, 4096, 128
    g = torch.Generator(device=DEV).manual_seed(5)
    q, k, v = (torch.randn(B, H, N, D, device=DEV, dtype=torch.bfloat16, generator=g) for _ in range(3))
    out = pli_hip.flash_attn_fwd(q, k, v, causal=True, variant=variant).float().cpu().numpy()
    ones = pli_hip.flash_attn_fwd(q, k, torch.ones_like(v), causal=True, variant=variant)
    assert (ones.float() - 1).abs().max().item() <= 2 ** -8
    for (b, h) in ((0, 0), (3, 17), (7, 31)):
        qq, kk, vv = (t[b:b + 1, h:h + 1].float().cpu().numpy() for t in (q, k, v))
        for i in (0, 1000, 4095):
            ref = oatt.naive_attention(qq[:, :, i:i + 1], kk[:, :, :i + 1], vv[:, :, :i + 1])
            err = np.abs(out[b, h, i] - ref[0, 0, 0]).max()
            assert err <= 1e-2, f"causal b{b} h{h} row {i}: {err:.3e}"
    if variant is None:
        base = pli_hip.flash_attn_fwd(q, k, v, causal=True, variant=55).float().cpu().numpy()
        assert np.abs(base - out).max() <= 1.6e-2


def test_mha_hip_matches_reference_golden():
    from ch01 import MultiHeadAttention
    g = load_golden("mha.npz")
    torch.manual_seed(0)
    mha = MultiHeadAttention(512, 8).to(DEV)
    x = torch.from_numpy(seeded_normal((1, 128, 512), 31)).to(DEV)
    with torch.no_grad():
        for causal, key in ((True, "y_causal"), (False, "y_noncausal")):
            y = mha(x, causal=causal).cpu().numpy()
            np.testing.assert_allclose(y, g[key], rtol=1e-3, atol=1e-4)


def test_ch06_reference_gpu_cases():
    """ch06/test_ch06.py:158-189 restated: fp16 flash vs naive (torch) on device."""
    from ch06 import flash_attention_forward, naive_attention
    torch.manual_seed(0)
    for (B, H, N, D), tol in (((2, 4, 128, 64), 0.01), ((1, 8, 512, 64), 0.02)):
        q, k, v = (torch.randn(B, H, N, D, device=DEV, dtype=torch.float16) for _ in range(3))
        torch.testing.assert_close(flash_attention_forward(q, k, v), naive_attention(q, k, v),
                                   rtol=tol, atol=tol)


# ------------------------------------------------------------------ GEMV ---
@pytest.mark.parametrize("m,k,dt", [(4096, 4096, "bf16"), (4096, 4096, "fp16"), (1000, 4096, "fp32"),
                                    (333, 1000, "bf16"), (128, 4104, "bf16"), (64, 37, "bf16"),
                                    (7, 8192, "fp16"), (8192, 8192, "bf16"),
                                    # tall W (M >= 16384: 2-rows-per-wave variant): LM head, odd M
                                    (32000, 2048, "bf16"), (16385, 520, "fp16"),
                                    # short rows (<= 128 chunks: 2 rows x 2 chunks per lane)
                                    (8192, 1024, "bf16"), (1001, 512, "fp32"), (3, 1024, "fp16")])
def test_gemv_vs_oracle(m, k, dt):
    import pli_hip
    w = seeded_normal((m, k), m + k, dt)
    x = seeded_normal((k,), m * 3 + 1, dt)
    y = pli_hip.gemv(dev(w, dt), dev(x, dt))
    assert_lin_close(y, olin.gemv(w, x), dt, f"gemv {m}x{k} {dt}")


def test_gemv_strided_rows():
    import pli_hip
    w = seeded_normal((256, 1024), 3, "bf16")
    wt = dev(w, "bf16")[:, :1000]  # ldw 1024 > k 1000
    x = seeded_normal((1000,), 4, "bf16")
    y = pli_hip.gemv(wt, dev(x, "bf16"))
    assert_lin_close(y, olin.gemv(w[:, :1000], x), "bf16", "strided gemv")


# ------------------------------------------------------------------ GEMM ---
@pytest.mark.parametrize("m,n,k,dt,tb", [
    (512, 512, 512, "bf16", False), (512, 512, 512, "bf16", True),
    (300, 264, 200, "bf16", False), (300, 264, 200, "fp16", True),
    (129, 72, 64, "bf16", True), (64, 64, 64, "fp32", False), (100, 60, 70, "fp32", True),
    (8, 4096, 4096, "bf16", True), (1, 256, 512, "bf16", False), (77, 77, 13, "bf16", False),
    # decode batches (skinny NT path, M <= 16)
    (1, 4096, 4096, "bf16", True), (3, 264, 520, "bf16", True), (5, 1000, 4096, "fp16", True),
    (16, 512, 8192, "bf16", True), (12, 96, 64, "fp16", True),
    # small-M MFMA NT path (M <= 128, K % 512 == 0, N % 16 == 0)
    (8, 4096, 4096, "fp16", True), (17, 1024, 1024, "bf16", True), (33, 528, 2048, "bf16", True),
    (64, 4096, 4096, "bf16", True), (100, 256, 512, "fp16", True), (128, 1024, 1536, "bf16", True)])
def test_gemm_vs_oracle(m, n, k, dt, tb):
    import pli_hip
    a = seeded_normal((m, k), 10 + m, dt)
    b = seeded_normal((n, k) if tb else (k, n), 20 + n, dt)
    c = pli_hip.gemm(dev(a, dt), dev(b, dt), trans_b=tb)
    ref = olin.linear(a, b) if tb else olin.gemm(a, b)
    assert_lin_close(c, ref, dt, f"gemm {m}x{n}x{k} {dt} tb={tb}")


@pytest.mark.parametrize("variant", [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15])
@pytest.mark.parametrize("m,n,k,tb,bias", [
    (512, 512, 512, False, False),
    (512, 512, 512, True, True),
    (600, 520, 256, False, False),    # ragged M and N in the last tiles
    (520, 600, 128, True, False),
    (1024, 768, 1024, False, True),   # tiles_n = 3 (XCD remap with nwg % 8 != 0)
    (256, 4096, 64, True, False),     # one K-tile
    (512, 512, 128, False, False),    # two K-tiles: pipeline drain from the start
    (768, 1024, 192, True, True),     # three K-tiles
    (2048, 2048, 4096, False, False), # long K: the steady-state vmcnt(8) path
    (2048, 2048, 4096, True, False),
])
def test_gemm_tile_variants(m, n, k, tb, bias, variant):
    """The 128x128 register-staged tile (1), the 256x256 LDS-DMA tile (2), its
    s_setprio form (4), its phased pipeline (3) and the phased pipeline with
    the staggered two-barrier schedule (5-8: SCHED 1, 3, 5, 7)."""
    import pli_hip
    dt = "bf16"
    a = seeded_normal((m, k), 3, dt)
    b = seeded_normal((n, k) if tb else (k, n), 4, dt)
    bb = seeded_normal((n,), 5, dt) if bias else None
    out = pli_hip.gemm(dev(a, dt), dev(b, dt), trans_b=tb, bias=dev(bb, dt) if bias else None,
                       variant=variant)
    ref = olin.gemm(a, b.T if tb else b)
    if bias:
        ref = ref + bb.astype(np.float64)
    assert_lin_close(out, ref, dt, f"variant {variant}")


# decode-batch / TP-shard NT paths, 16 < M <= 256: default route (workspace
# from the wrapper: LDS split-K, or mid-M / small-M for short K), direct-load
# split-K (22, 24), LDS split-K (25-27), mid-M (20), small-M (21)
@pytest.mark.parametrize("variant", [None, 20, 21, 22, 24, 25, 26, 27, 28, 29])
@pytest.mark.parametrize("m,n,k,dt,bias", [
    (17, 1024, 4096, "bf16", False),   # one 32-row chunk, 8 n-tiles x 8 slices
    (64, 512, 8192, "bf16", True),     # long K slices
    (100, 288, 4096, "fp16", False),   # ragged M chunk, N % 128 != 0 (last tile half empty)
    (128, 256, 1024, "bf16", True),    # short K: mid-M route by default
    (200, 640, 2048, "bf16", False),   # two 128-row slabs of X, the second partial
    (256, 128, 512, "fp16", True),     # one n-tile: slices fill the grid
    (520, 384, 1024, "bf16", True),    # few-tile route: 5 slabs, the last one 8 rows
    (1024, 512, 4096, "fp16", False),
])
def test_gemm_decode_batch_paths(m, n, k, dt, bias, variant):
    import pli_hip
    a = seeded_normal((m, k), 7 + m, dt)
    w = seeded_normal((n, k), 8 + n, dt)
    bb = seeded_normal((n,), 9, dt) if bias else None
    out = pli_hip.gemm(dev(a, dt), dev(w, dt), trans_b=True, bias=dev(bb, dt) if bias else None,
                       variant=variant)
    assert_lin_close(out, olin.linear(a, w, bb), dt, f"decode-batch gemm {m}x{n}x{k} v{variant}")


# M <= 4 skinny NT path (gemm_skinny_nt): chunks per lane 2 / 4 / 8 / 12 chosen
# by K; each side of every boundary
@pytest.mark.parametrize("m", [1, 3])
@pytest.mark.parametrize("k", [512, 1024, 1032, 2048, 2056, 5632])
def test_gemm_skinny_cpl_boundaries(m, k):
    """Without a bias M = 1 routes to the gemv kernel; with one (zeros, so the
    expected output is unchanged) to the skinny kernel: both vs the oracle,
    and the two routes bitwise equal (same per-lane chunk order)."""
    import pli_hip
    a = seeded_normal((m, k), 11 + k, "bf16")
    w = seeded_normal((300, k), 12 + k, "bf16")
    out = pli_hip.gemm(dev(a, "bf16"), dev(w, "bf16"), trans_b=True)
    assert_lin_close(out, olin.linear(a, w, None), "bf16", f"skinny gemm {m}x300x{k}")
    zb = torch.zeros(300, device=DEV, dtype=torch.bfloat16)
    out_b = pli_hip.gemm(dev(a, "bf16"), dev(w, "bf16"), trans_b=True, bias=zb)
    assert_lin_close(out_b, olin.linear(a, w, None), "bf16", f"skinny gemm {m}x300x{k} + bias")
    if m == 1 and k in (512, 1024, 2048, 5632):
        assert torch.equal(out, out_b), "gemv route differs from the skinny kernel"


def test_gemm_ws_abi_direct():
    """pli_gemm_ws through the C ABI: undersized workspace falls back, a
    sized one takes the split-K path; both match the oracle."""
    import ctypes
    import pli_hip
    m, n, k = 96, 512, 4096
    a, w = seeded_normal((m, k), 1, "bf16"), seeded_normal((n, k), 2, "bf16")
    at, wt = dev(a, "bf16"), dev(w, "bf16")
    ref = olin.linear(a, w)
    lib = pli_hip.lib()
    need = lib.pli_gemm_workspace_size(m, n, k, 1, 2)
    assert need > 0 and lib.pli_gemm_workspace_size(m, n, k, 0, 2) == 0
    stream = torch.cuda.current_stream().cuda_stream
    for wsb in (16, need):
        ws = torch.empty(max(wsb, 16), dtype=torch.uint8, device=DEV)
        out = torch.empty(m, n, dtype=torch.bfloat16, device=DEV)
        rc = lib.pli_gemm_ws(at.data_ptr(), wt.data_ptr(), out.data_ptr(), None, m, n, k, k, k, n, 1, 2,
                             ws.data_ptr(), wsb, ctypes.c_void_p(stream))
        assert rc == 0, pli_hip.lib().pli_last_error()
        assert_lin_close(out, ref, "bf16", f"pli_gemm_ws ws={wsb}")


@pytest.mark.parametrize("m", [192, 4, 48])
def test_gemm_bias_epilogue(m):
    import pli_hip
    a, w = seeded_normal((m, 512), 1, "bf16"), seeded_normal((144, 512), 2, "bf16")
    bias = seeded_normal((144,), 3, "bf16")
    c = pli_hip.gemm(dev(a, "bf16"), dev(w, "bf16"), trans_b=True, bias=dev(bias, "bf16"))
    assert_lin_close(c, olin.linear(a, w, bias), "bf16", "bias")


def test_batched_gemv_benchmark_api():
    """ch03.benchmark_batched_gemv runs the HIP skinny path end to end."""
    from ch03 import benchmark_batched_gemv
    r = benchmark_batched_gemv(4, 1024, 1024, dtype=torch.bfloat16, warmup=2, iterations=5)
    assert r.batch_size == 4 and r.mean_us > 0 and r.tokens_per_second > 0


def test_gemm_4096_cube_rows():
    """The ch05/ch03 config (4096^3 bf16, NN): 64 random rows vs f64."""
    import pli_hip
    m = n = k = 4096
    a, b = seeded_normal((m, k), 31, "bf16"), seeded_normal((k, n), 32, "bf16")
    c = pli_hip.gemm(dev(a, "bf16"), dev(b, "bf16")).float().cpu().numpy()
    rows = np.random.RandomState(0).choice(m, 64, replace=False)
    assert_lin_close(torch.from_numpy(c[rows]), olin.gemm(a[rows], b), "bf16", "4096^3")


@pytest.mark.parametrize("tp", [8, 4, 2])
def test_row_parallel_shard_full_config(tp):
    """ch09 TP config (BASELINE configs[4]): the per-rank
    row shard of the 8192x8192 weight at M = 8192, X [8192, 8192/tp] and
    W [8192, 8192/tp] (NT, bf16) through RowParallelLinear (the HIP GEMM),
    64 random output rows against the f64 oracle (ch09/tensor_parallel.py:43-68)."""
    from ch09 import RowParallelLinear
    M = N = K = 8192
    ks = K // tp
    r = tp - 1  # the last rank's slice
    x = seeded_normal((M, ks), 40 + tp, "bf16")
    w = seeded_normal((N, ks), 50 + tp, "bf16") * np.float32(ks ** -0.5)
    from oracle.numerics import round_to_bf16
    w = round_to_bf16(w)
    layer = RowParallelLinear(K, N, world_size=tp, rank=r).to(DEV).to(torch.bfloat16)
    assert tuple(layer.weight.shape) == (N, ks)
    layer.weight.data.copy_(dev(w, "bf16"))
    with torch.no_grad():
        y = layer(dev(x, "bf16")).float().cpu().numpy()
    rows = np.random.RandomState(tp).choice(M, 64, replace=False)
    assert_lin_close(torch.from_numpy(y[rows]), olin.linear(x[rows], w), "bf16", f"TP{tp} shard")


# ------------------------------------------------------- softmax / stream ---
@pytest.mark.parametrize("shape,dt", [((4, 8, 64), "fp32"), ((5,), "fp32"), ((33, 1000), "bf16"),
                                      ((7, 4097), "fp16")])
def test_softmax_rows(shape, dt):
    from ch06 import online_softmax, standard_softmax
    x = seeded_normal(shape, 42, dt)
    ref = oatt.standard_softmax(x)
    for fn in (online_softmax, standard_softmax):
        y = fn(dev(x, dt)).float().cpu().numpy()
        np.testing.assert_allclose(y, ref, rtol=LIN_TOL[dt] * 2, atol=1e-6 if dt == "fp32" else 2e-3)


def test_softmax_large_logits_stable():
    from ch06 import online_softmax
    x = torch.tensor([1000.0, 1001.0, 1002.0], device=DEV)
    y = online_softmax(x)
    assert torch.isfinite(y).all()
    np.testing.assert_allclose(y.cpu().numpy(), oatt.standard_softmax(x.cpu().numpy()), rtol=1e-6)


def test_online_softmax_with_output_golden():
    from ch06 import online_softmax_with_output
    g = load_golden("softmax.npz")
    x4, v4 = seeded_normal((2, 4, 32), 22), seeded_normal((2, 4, 32, 16), 23)
    o, d = online_softmax_with_output(dev(x4, "fp32"), dev(v4, "fp32"))
    np.testing.assert_allclose(o.cpu().numpy(), g["x4_o"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(d.cpu().numpy(), g["x4_d"], rtol=1e-5, atol=1e-6)


def test_scale_copy_exact():
    import pli_hip
    src = torch.randn(1 << 20, device=DEV)
    out = torch.empty_like(src)
    pli_hip.scale_copy(src, out)
    assert torch.equal(out, src * 2)
    out_s = torch.empty((1 << 20) // 32, device=DEV)
    pli_hip.scale_copy(src, out_s, stride=32)
    assert torch.equal(out_s, src[::32] * 2)


# ------------------------------------------------------------------- TP ----
def test_tensor_parallel_shards_sum_to_full_linear():
    """Row-parallel partials of 4 shards (one process) sum to F.linear; the
    chunked/overlapped path equals the plain one."""
    from ch09 import ColumnParallelLinear, RowParallelLinear, row_parallel_forward_overlapped
    ws, M, K, N = 4, 96, 512, 256
    x = seeded_normal((M, K), 1, "bf16")
    w = seeded_normal((N, K), 2, "bf16")
    total, mag = 0.0, 0.0
    for r in range(ws):
        layer = RowParallelLinear(K, N, world_size=ws, rank=r).to(DEV).to(torch.bfloat16)
        sl = slice(r * K // ws, (r + 1) * K // ws)
        layer.weight.data.copy_(dev(w[:, sl], "bf16"))
        y = layer(dev(x[:, sl], "bf16")).float()
        y2 = row_parallel_forward_overlapped(dev(x[:, sl], "bf16"), layer.weight, chunks=3).float()
        torch.testing.assert_close(y2, y, rtol=0, atol=0)
        assert_lin_close(y, olin.linear(x[:, sl], w[:, sl]), "bf16", f"partial {r}")
        y = y.cpu().numpy().astype(np.float64)
        total, mag = total + y, mag + np.abs(y)
    # each partial is rounded to bf16 before the sum: bound by sum |partial|
    err = np.abs(total - olin.row_parallel_sum(x, w, ws))
    assert np.all(err <= LIN_TOL["bf16"] * (mag + 1.0)), err.max()
    col = ColumnParallelLinear(K, 4 * N, world_size=4, rank=1, bias=True).to(DEV)
    xx = torch.from_numpy(x).to(DEV)
    yc = col(xx).cpu().numpy()
    ref = olin.linear(x, col.weight.detach().cpu().numpy(), col.bias.detach().cpu().numpy())
    np.testing.assert_allclose(yc, ref, rtol=1e-4, atol=1e-4)


def test_calibration_probes():
    """The roofline calibration kernels compute what they claim: the read
    probe touches every 16-byte chunk exactly once (XOR of all thread words ==
    XOR of the buffer); the MFMA probe's outputs are finite and non-zero."""
    import pli_hip
    g = torch.Generator(device=DEV).manual_seed(3)
    buf = torch.randint(-2 ** 31, 2 ** 31 - 1, ((1 << 20) + 4 * 37,), device=DEV, dtype=torch.int32, generator=g)
    want = np.bitwise_xor.reduce(buf.cpu().numpy().view(np.uint32))
    for mode in (0, 1):
        for blocks in (1, 8, 300, 1023):
            out = torch.zeros(blocks * 256, device=DEV, dtype=torch.int32)
            pli_hip.hbm_read_probe(buf, out, blocks, mode)
            got = np.bitwise_xor.reduce(out.cpu().numpy().view(np.uint32))
            assert got == want, (mode, blocks)
    for shape in (0, 1):
        o = torch.zeros(16 * 256, device=DEV, dtype=torch.float32)
        ck = torch.zeros(16 * 8, device=DEV, dtype=torch.int64)
        pli_hip.mfma_probe(o, 16, 64, shape, clocks=ck)
        assert torch.isfinite(o).all() and (o != 0).any()
        ck = ck.view(-1, 2).double().cpu()
        assert (ck > 0).all(), "every wave stamps its loop"
        ghz = ck[:, 0] / ck[:, 1] * 0.1
        assert ((ghz > 0.3) & (ghz < 3.0)).all(), ghz
    with pytest.raises(pli_hip.PliError):  # a CPU or non-int32 out is refused, not written
        pli_hip.hbm_read_probe(buf, torch.zeros(256, dtype=torch.int32), 1, 0)
    with pytest.raises(pli_hip.PliError):
        pli_hip.hbm_read_probe(buf, torch.zeros(256, device=DEV, dtype=torch.float32), 1, 0)


@pytest.mark.parametrize("m,n,k", [(512, 1024, 2048), (200, 96, 128), (33, 40, 72), (1, 64, 64)])
def test_gemm_f32out_vs_f64(m, n, k):
    """pli_gemm_f32out (NT, bf16 in, fp32 out): the LDS split-K route (K % 64,
    N % 32) and the one-thread-per-output route, against the f64 product of
    the same bf16 inputs; fp32 accumulation, so 1e-5 relative."""
    import pli_hip
    x, w = seeded_normal((m, k), 91, "bf16"), seeded_normal((n, k), 92, "bf16")
    y = pli_hip.gemm_f32out(dev(x, "bf16"), dev(w, "bf16")).cpu().numpy().astype(np.float64)
    ref = olin.linear(x, w)
    assert y.dtype == np.float64 and np.abs(y - ref).max() <= 1e-5 * (np.abs(ref).max() + 1)


@pytest.mark.parametrize("m,n,k", [(4096, 4096, 1024), (4096, 8192, 8192), (2200, 4096, 512)])
def test_gemm_f32out_large_w5(m, n, k):
    """pli_gemm_f32out at sizes that take gemm_w5's fp32 epilogue (128+
    tiles of 256^2; persistent for M, N multiples of 256 with K <= 4096, the
    one-tile form at K 8192 and for a ragged M): sampled rows against the f64
    product of the same bf16 inputs, fp32 accumulation so 1e-5 relative, and
    bitwise equal to the bf16 product before its rounding (pli_gemm's bf16
    output is the rounded fp32 result of the same MFMA chains)."""
    import pli_hip
    g = torch.Generator(device="cuda").manual_seed(m + n + k)
    x = torch.randn(m, k, device="cuda", dtype=torch.bfloat16, generator=g)
    w = torch.randn(n, k, device="cuda", dtype=torch.bfloat16, generator=g)
    y = pli_hip.gemm_f32out(x, w)
    assert y.dtype == torch.float32 and y.shape == (m, n)
    rows = torch.randperm(m, generator=torch.Generator().manual_seed(3))[:32].to("cuda")
    ref = x[rows].double() @ w.double().t()
    assert (y[rows].double() - ref).abs().max().item() <= 1e-5 * (ref.abs().max().item() + 1)
    assert torch.equal(y.to(torch.bfloat16), pli_hip.gemm(x, w, trans_b=True))


@pytest.mark.parametrize("tp", [2, 4, 8])
def test_row_parallel_fp32_partials_error_by_tp(tp):
    """The TP row-parallel sum at tp shards of an 8192-wide layer (M = 256):
    bf16 partials (the reference's F.linear per rank) stack tp roundings --
    where partials cancel, that breaks the 1e-2 * (|ref| + 1) bound (it did at
    tp 2 and 4 on the first run) -- fp32 partials (reduce_dtype=
    torch.float32) round once and stay within it."""
    import pli_hip
    M, N, K = 256, 8192, 8192
    g = torch.Generator(device=DEV).manual_seed(tp)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16, generator=g)
    w = (torch.randn(N, K, device=DEV, generator=g) * K ** -0.5).to(torch.bfloat16)
    ref = x.double() @ w.double().T
    ks = K // tp
    s16 = torch.zeros(M, N, device=DEV, dtype=torch.float32)
    s32 = torch.zeros(M, N, device=DEV, dtype=torch.float32)
    mag = torch.zeros(M, N, device=DEV, dtype=torch.float64)
    for r in range(tp):
        xs, wsh = x[:, r * ks:(r + 1) * ks], w[:, r * ks:(r + 1) * ks]
        p32 = pli_hip.gemm_f32out(xs, wsh)
        s16 += pli_hip.gemm(xs, wsh, trans_b=True).float()
        s32 += p32
        mag += p32.double().abs()
    e16 = (s16.to(torch.bfloat16).double() - ref).abs()
    e32 = (s32.to(torch.bfloat16).double() - ref).abs()
    # bf16's unit roundoff is u = 2^-8 (half an ulp relative to the value).
    # fp32 partials: one final bf16 rounding, u * |ref|, plus fp32 sums;
    # bf16 partials: one u * |p_i| rounding per rank's partial on top -- where
    # the partials cancel (sum << terms) that exceeds 1e-2 * (|ref| + 1), the
    # case the fp32 option exists for.  The slack covers u^2 terms and fp32
    # accumulation (~sqrt(K) * 2^-24 relative to the partials' magnitude).
    u = 2.0 ** -8
    slack = 4e-5 * (ref.abs() + mag + 1)
    assert (e32 <= u * ref.abs() + slack).all(), f"fp32 partials, tp {tp}: {e32.max().item():.3e}"
    assert (e16 <= u * (ref.abs() + mag) + slack).all(), f"bf16 partials, tp {tp}: {e16.max().item():.3e}"
    assert (e32 <= 1e-2 * (ref.abs() + 1)).all()
    assert e32.mean().item() <= e16.mean().item()
