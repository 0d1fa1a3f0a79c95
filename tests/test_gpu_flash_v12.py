"""attn_fwd_v12, the round-3 non-causal flash default (variant 71 persistent, 70 one
block per workgroup, 72 = 71 with the defer-max threshold at 0), against
references that share none of its code (cdna_hip_programming.md §5.4 rule 26):

* a float64 torch attention on the device over the WHOLE output tensor
  (scores by matmul, torch.softmax, P·V -- the reference's naive_attention,
  ch06/attention_memory.py:19-33, in f64), at every persistent-seam shape,
  plain and with Q scaled by 4 (peaky rows that take the rescale branch);
* an fp32 torch attention per head over all 256 heads of the bench config
  (B8 S4096 H32 D128);
* the threshold sweep: THR 0 (variant 72: a rescale whenever a tile raises a
  row's max) and the shipped THR 64 (8 before round 4) agree to rounding.

Bounds: 1e-2 absolute on randn inputs (north_star's bf16 bound).  On the
peaky Q x 4 inputs: 2^-8 * max|v| -- the bf16 rounding of the P weights fed
to the PV MFMA (2^-9 relative) plus that of the output (2^-9), each at most
2^-9 * max|v| when a few keys dominate a row.  For scale, the reference's own
bf16 flash (ch06/flash_attention.py:14-74) is off by 0.115-0.120 on inputs of
this kind (tests/golden/stress_flash.npz, seam2 / seam5, recorded from the
reference in the build container).
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle.numerics import seeded_normal

pytestmark = pytest.mark.gpu
DEV = "cuda"
V12 = (70, 71, 72)


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV).to(torch.bfloat16)


def torch_attention(q, k, v, dtype=torch.float64, heads_per_chunk=8, causal=False):
    """softmax(q k^T / sqrt(D)) v over [B,H,N,D] tensors in ``dtype`` on the
    device, K/V heads shared by H/Hkv query heads (GQA, ch01/gqa.py:30-34);
    causal: the bottom-right mask (row i sees keys j <= i + Nk - Nq,
    ch01/attention.py:66-67, ch02/cached_generation.py:85-91)."""
    B, H, Nq, D = q.shape
    Nk = k.shape[2]
    g = H // k.shape[1]
    out = torch.empty(B, H, Nq, D, dtype=dtype, device=q.device)
    if causal:
        i = torch.arange(Nq, device=q.device)[:, None]
        j = torch.arange(Nk, device=q.device)[None, :]
        masked = j > i + (Nk - Nq)
    for b in range(B):
        for h0 in range(0, H, heads_per_chunk):
            hs = torch.arange(h0, min(H, h0 + heads_per_chunk), device=q.device)
            qq, kk, vv = q[b, hs].to(dtype), k[b, hs // g].to(dtype), v[b, hs // g].to(dtype)
            sc = torch.matmul(qq, kk.transpose(-1, -2)) * D ** -0.5
            if causal:
                sc = sc.masked_fill(masked, float("-inf"))
            out[b, hs] = torch.matmul(torch.softmax(sc, dim=-1), vv)
    return out


def max_err(out, ref):
    o = out.to(ref.dtype)
    assert torch.isfinite(o).all(), "non-finite output"
    return (o - ref).abs().max().item()


def inputs(shape, seed):
    B, H, Hkv, Nq, Nk = shape
    q = seeded_normal((B, H, Nq, 128), seed, "bf16")
    k = seeded_normal((B, Hkv, Nk, 128), seed + 1, "bf16")
    v = seeded_normal((B, Hkv, Nk, 128), seed + 2, "bf16")
    return dev(q), dev(k), dev(v)


# (B, H, Hkv, Nq, Nk): grids beyond one workgroup per CU so the persistent
# walk crosses block seams -- blocks of 2 / 3 / 5 / 16 key tiles, ragged Nq,
# GQA -- and Nk = 64 (one key tile: the prologue's tile is also the last, no
# loop step runs, the epilogue's tailB finishes it)
SEAMS = [(4, 16, 4, 2048, 1024), (4, 32, 8, 1024, 128), (4, 32, 8, 1024, 192), (3, 40, 8, 1000, 320),
         (2, 4, 1, 2048, 192)]
NK64 = [(1, 2, 2, 1, 64), (1, 2, 2, 64, 64), (2, 4, 4, 300, 64), (1, 8, 2, 256, 64), (8, 36, 4, 256, 64)]


@pytest.mark.parametrize("qmul", (1, 4))
@pytest.mark.parametrize("shape", SEAMS + NK64, ids=lambda s: "b{}h{}kv{}q{}k{}".format(*s))
def test_v12_vs_f64_full_tensor(shape, qmul):
    """Every output element of variants 70 / 71 / 72 against the f64 device
    reference; 70 and 71 (same arithmetic, one vs many blocks per
    workgroup) bitwise equal."""
    import pli_hip
    q, k, v = inputs(shape, sum(shape) % 997)
    q = q * qmul  # exact in bf16
    ref = torch_attention(q, k, v)
    tol = 1e-2 if qmul == 1 else 2.0 ** -8 * v.abs().max().item()
    outs = {}
    for var in V12:
        outs[var] = pli_hip.flash_attn_fwd(q, k, v, variant=var)
        err = max_err(outs[var], ref)
        assert err <= tol, f"{shape} q*{qmul} variant {var}: max |err| {err:.4e} > {tol:.4e}"
    assert torch.equal(outs[70], outs[71]), f"{shape}: 70 != 71"


def test_v12_strided_bshd_views():
    """The MHA layout: q/k/v as [B,S,H,D] buffers read through [B,H,S,D]
    views and O written into a transposed view (out=), non-causal bf16 D128
    (the v12 path), against the f64 reference and the contiguous call."""
    import pli_hip
    B, S, H, D = 2, 320, 8, 128
    x = dev(seeded_normal((3, B, S, H, D), 41, "bf16"))
    q, k, v = (x[i].transpose(1, 2) for i in range(3))
    ref = torch_attention(q, k, v)
    for var in (None, 70, 71, 72):
        o = torch.full((B, S, H, D), float("nan"), dtype=torch.bfloat16, device=DEV)
        pli_hip.flash_attn_fwd(q, k, v, out=o.transpose(1, 2), variant=var)
        err = max_err(o.transpose(1, 2), ref)
        assert err <= 1e-2, f"variant {var}: strided max |err| {err:.4e}"
        contig = pli_hip.flash_attn_fwd(q.contiguous(), k.contiguous(), v.contiguous(), variant=var)
        assert torch.equal(o.transpose(1, 2), contig), f"variant {var}: strided != contiguous"


@pytest.mark.parametrize("variant", (None, 72))
def test_v12_full_config_all_heads(variant):
    """The bench config, B8 S4096 H32 D128 bf16: all 256 (batch, head) pairs
    against an fp32 torch attention per head (not SDPA), and the THR-0
    variant within rounding of the shipped one."""
    import pli_hip
    B, H, N, D = 8, 32, 4096, 128
    g = torch.Generator(device=DEV).manual_seed(0)
    q, k, v = (torch.randn(B, H, N, D, device=DEV, dtype=torch.bfloat16, generator=g) for _ in range(3))
    out = pli_hip.flash_attn_fwd(q, k, v, variant=variant)
    worst = 0.0
    for b in range(B):
        ref = torch_attention(q[b:b + 1], k[b:b + 1], v[b:b + 1], dtype=torch.float32, heads_per_chunk=4)
        err = max_err(out[b:b + 1], ref)
        worst = max(worst, err)
        assert err <= 1e-2, f"batch {b}: max |err| {err:.4e} over its 32 heads"
    print(f"variant {variant}: max |err| over all 256 heads {worst:.4e}")
    if variant == 72:
        base = pli_hip.flash_attn_fwd(q, k, v)
        assert_agree_to_rounding(out, base, v)


def assert_agree_to_rounding(a, b, v):
    """THR sweep bound: two bf16 ulps of the output plus the P rounding
    (2^-9 * max|v|) -- the two thresholds round P against different m."""
    d = (a.float() - b.float()).abs()
    bound = 2.0 ** -7 * torch.maximum(a.float().abs(), b.float().abs()) + 2.0 ** -9 * v.abs().max().float()
    bad = d > bound
    assert not bad.any(), f"{int(bad.sum())} elements beyond rounding, max |diff| {d.max().item():.4e}"


@pytest.mark.parametrize("name", ("spike", "first", "late", "all", "seam2", "seam5"))
def test_v12_threshold_sweep_stress(name):
    """cdna_hip_programming.md rule 26 (3): THR 0 (72) vs the shipped THR 64
    (71) on the adversarial inputs of tests/stress_cases.py, each of which
    forces the rescale branch at chosen tiles."""
    import pli_hip
    from stress_cases import stress_inputs
    q, k, v = (dev(x) for x in stress_inputs(name))
    assert_agree_to_rounding(pli_hip.flash_attn_fwd(q, k, v, variant=72),
                             pli_hip.flash_attn_fwd(q, k, v, variant=71), v)


def test_flash_negative_and_zero_scale():
    """A non-positive scale (allowed by the API) goes to the generic kernel:
    the MFMA bodies' running max assumes scale > 0."""
    import pli_hip
    from oracle import attention as oatt
    q, k, v = (seeded_normal((1, 2, 128, 128), 60 + i, "bf16") for i in range(3))
    for scale in (-0.125, 0.0):
        out = pli_hip.flash_attn_fwd(dev(q), dev(k), dev(v), scale=scale).double().cpu().numpy()
        ref = oatt.naive_attention(q, k, v, scale=scale)
        assert np.isfinite(out).all() and np.abs(out - ref).max() <= 1e-2, f"scale {scale}"


# causal v12 (variants 73: one block per workgroup, heaviest first; 74:
# persistent, the pair walk of query heights where the shape admits it).
# (B, H, Hkv, Nq, Nk): the pair walk (512 blocks over 256 workgroups at QB 4,
# 8 and 16), a head count the walk does not tile (one block per workgroup), bottom-right with Nq < Nk (ragged), a single query row, one key
# tile (the prologue's tile holds every diagonal)
CAUSAL_SHAPES = [(4, 32, 8, 1024, 1024), (2, 32, 32, 2048, 2048), (2, 16, 4, 4096, 4096), (3, 40, 8, 1024, 1024),
                 (2, 8, 2, 300, 512), (1, 4, 4, 1, 128), (2, 4, 4, 64, 64), (1, 8, 8, 700, 768)]


@pytest.mark.parametrize("qmul", (1, 4))
@pytest.mark.parametrize("shape", CAUSAL_SHAPES, ids=lambda s: "b{}h{}kv{}q{}k{}".format(*s))
def test_v12_causal_vs_f64_full_tensor(shape, qmul):
    """Every output element of causal 73 / 74 against the f64 device
    reference with the bottom-right mask; 73 and 74 bitwise equal (same
    arithmetic per block, only the block order differs)."""
    import pli_hip
    q, k, v = inputs(shape, sum(shape) % 991)
    q = q * qmul
    ref = torch_attention(q, k, v, causal=True)
    tol = 1e-2 if qmul == 1 else 2.0 ** -8 * v.abs().max().item()
    outs = {}
    for var in (73, 74):
        outs[var] = pli_hip.flash_attn_fwd(q, k, v, causal=True, variant=var)
        err = max_err(outs[var], ref)
        assert err <= tol, f"{shape} q*{qmul} causal variant {var}: max |err| {err:.4e} > {tol:.4e}"
    assert torch.equal(outs[73], outs[74]), f"{shape}: 73 != 74"


def test_v12_causal_full_config_all_heads():
    """Causal at the bench config (B8 S4096 H32 D128, the persistent
    pair walk): all 256 heads, whole heads, against an fp32 torch attention
    with the causal mask; the default causal path agrees within rounding."""
    import pli_hip
    B, H, N, D = 8, 32, 4096, 128
    g = torch.Generator(device=DEV).manual_seed(5)
    q, k, v = (torch.randn(B, H, N, D, device=DEV, dtype=torch.bfloat16, generator=g) for _ in range(3))
    out = pli_hip.flash_attn_fwd(q, k, v, causal=True, variant=74)
    for b in range(B):
        ref = torch_attention(q[b:b + 1], k[b:b + 1], v[b:b + 1], dtype=torch.float32, heads_per_chunk=4,
                              causal=True)
        err = max_err(out[b:b + 1], ref)
        assert err <= 1e-2, f"causal batch {b}: max |err| {err:.4e} over its 32 heads"
    dflt = pli_hip.flash_attn_fwd(q, k, v, causal=True)
    assert_agree_to_rounding(dflt, out, v)


def test_v12_causal_stress():
    """The rescale branch on masked tiles: the stress inputs (spike / late /
    all) through causal 74, against the f64 causal reference."""
    import pli_hip
    from stress_cases import stress_inputs
    for name in ("spike", "late", "all", "seam5"):
        q, k, v = (dev(x) for x in stress_inputs(name))
        out = pli_hip.flash_attn_fwd(q, k, v, causal=True, variant=74)
        err = max_err(out, torch_attention(q, k, v, causal=True))
        assert err <= 2.0 ** -8 * v.abs().max().item(), f"{name}: {err:.4e}"


def _scaled_ref(q, k, v, scale, causal):
    g = q.shape[1] // k.shape[1]
    kf, vf = (t.double().repeat_interleave(g, dim=1) for t in (k, v))
    sc = (q.double() @ kf.transpose(-1, -2)) * scale
    if causal:
        nq, nk = q.shape[2], k.shape[2]
        i = torch.arange(nq, device=q.device)[:, None]
        j = torch.arange(nk, device=q.device)[None, :]
        sc = sc.masked_fill(j > i + (nk - nq), float("-inf"))
    return torch.softmax(sc, -1) @ vf


@pytest.mark.parametrize("scale", (1.0, 0.25))
@pytest.mark.parametrize("case", [(128, "bf16", 71, False), (128, "bf16", 74, True), (128, "bf16", 55, False),
                                  (128, "bf16", 60, True), (128, "f16", None, False), (64, "bf16", None, False),
                                  (64, "f16", None, True), (64, "bf16", 51, True)],
                         ids=lambda c: "d{}-{}-v{}-causal{}".format(*c))
def test_fallback_bodies_explicit_scale(case, scale):
    """The exact fallback bodies (v12 71 / 74, v10 55 / 60, v7 51; D = 64 and
    fp16 by the default route) apply c = scale * log2(e) by fma to fp32
    scores, so scale 1.0 (c > 1) runs on them instead of variant 21; against
    an f64 attention with the same scale.  Defer threshold 64 (bf16) / 8
    (fp16): at scale 1.0 the rescale path runs in most rows."""
    import pli_hip
    D, dt, var, causal = case
    dtype = torch.bfloat16 if dt == "bf16" else torch.float16
    gen = torch.Generator(device=DEV).manual_seed(D + (var or 0) + int(scale * 8))
    q = torch.randn(2, 8, 320, D, device=DEV, dtype=dtype, generator=gen)
    k = torch.randn(2, 2, 384, D, device=DEV, dtype=dtype, generator=gen)
    v = torch.randn(2, 2, 384, D, device=DEV, dtype=dtype, generator=gen)
    out = pli_hip.flash_attn_fwd(q, k, v, scale=scale, causal=causal, variant=var)
    err = max_err(out, _scaled_ref(q, k, v, scale, causal))
    tol = 2.0 ** -8 * v.abs().max().item()
    assert err <= tol, f"{case} scale {scale}: max |err| {err:.4e} > {tol:.4e}"
