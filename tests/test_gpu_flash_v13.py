"""attn_fwd_v13 (variants 80 persistent, 81 one block per workgroup, 82 =
80 with mu = max * c - 1, i.e. the rare rescale path at nearly every tile)
against references that share none of its code (cdna_hip_programming.md
§5.4 rule 26) -- the same checks as tests/test_gpu_flash_v12.py:

* a float64 torch attention on the device over the WHOLE output tensor
  (the reference's naive_attention, ch06/attention_memory.py:19-33, in f64)
  at every persistent-seam shape, plain and with Q scaled by 4 (peaky rows
  that take the rescale branch);
* an fp32 torch attention per head over all 256 heads of the bench config
  (B8 S4096 H32 D128);
* the rescale sweep: 82 (rescale whenever a tile's max reaches the running
  max) and the shipped 80 agree to rounding, on randn and on the
  adversarial inputs of tests/stress_cases.py.

Bounds as in the v12 file: 1e-2 absolute on randn inputs (north_star's bf16
bound), 2^-8 * max|v| on the peaky inputs (P and output rounding).
"""
from __future__ import annotations

import pytest
import torch

from test_gpu_flash_v12 import (DEV, NK64, SEAMS, assert_agree_to_rounding, dev, inputs, max_err,
                                torch_attention)

pytestmark = pytest.mark.gpu
V13 = (80, 81, 82)
# v13 needs Nk >= 128 (two key tiles: the K/V stream runs two tiles ahead)
SHAPES = SEAMS + [(1, 2, 2, 1, 128), (2, 4, 4, 300, 128), (8, 36, 4, 256, 128), (1, 3, 1, 64, 256),
                  (2, 2, 1, 200, 128)]


@pytest.mark.parametrize("qmul", (1, 4))
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "b{}h{}kv{}q{}k{}".format(*s))
def test_v13_vs_f64_full_tensor(shape, qmul):
    """Every output element of 80 / 81 / 82 against the f64 device
    reference; 80 and 81 (one vs many blocks per workgroup) bitwise equal."""
    import pli_hip
    q, k, v = inputs(shape, sum(shape) % 997)
    q = q * qmul  # exact in bf16
    ref = torch_attention(q, k, v)
    tol = 1e-2 if qmul == 1 else 2.0 ** -8 * v.abs().max().item()
    outs = {}
    for var in V13:
        outs[var] = pli_hip.flash_attn_fwd(q, k, v, variant=var)
        err = max_err(outs[var], ref)
        assert err <= tol, f"{shape} q*{qmul} variant {var}: max |err| {err:.4e} > {tol:.4e}"
    assert torch.equal(outs[80], outs[81]), f"{shape}: 80 != 81"


def test_v13_nk64_falls_back():
    """Nk = 64 is below v13's two-tile stream: the variant routes to v12."""
    import pli_hip
    for shape in NK64[:2]:
        q, k, v = inputs(shape, 7)
        assert torch.equal(pli_hip.flash_attn_fwd(q, k, v, variant=80), pli_hip.flash_attn_fwd(q, k, v, variant=71))


def test_v13_strided_bshd_views():
    """q/k/v as [B,S,H,D] buffers through [B,H,S,D] views, O into a
    transposed view: against the f64 reference and the contiguous call."""
    import pli_hip
    from oracle.numerics import seeded_normal
    B, S, H, D = 2, 320, 8, 128
    x = dev(seeded_normal((3, B, S, H, D), 41, "bf16"))
    q, k, v = (x[i].transpose(1, 2) for i in range(3))
    ref = torch_attention(q, k, v)
    for var in V13:
        o = torch.full((B, S, H, D), float("nan"), dtype=torch.bfloat16, device=DEV)
        pli_hip.flash_attn_fwd(q, k, v, out=o.transpose(1, 2), variant=var)
        err = max_err(o.transpose(1, 2), ref)
        assert err <= 1e-2, f"variant {var}: strided max |err| {err:.4e}"
        contig = pli_hip.flash_attn_fwd(q.contiguous(), k.contiguous(), v.contiguous(), variant=var)
        assert torch.equal(o.transpose(1, 2), contig), f"variant {var}: strided != contiguous"


@pytest.mark.parametrize("variant", (80, 82))
def test_v13_full_config_all_heads(variant):
    """B8 S4096 H32 D128 bf16: all 256 (batch, head) pairs against an fp32
    torch attention per head; 82 within rounding of 80."""
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
    if variant == 82:
        assert_agree_to_rounding(out, pli_hip.flash_attn_fwd(q, k, v, variant=80), v)


@pytest.mark.parametrize("name", ("spike", "first", "late", "all", "seam2", "seam5"))
def test_v13_rescale_stress(name):
    """The adversarial inputs (each forces the rescale branch at chosen
    tiles): 80 against the f64 reference, and 82 within rounding of 80."""
    import pli_hip
    from stress_cases import stress_inputs
    q, k, v = (dev(x) for x in stress_inputs(name))
    if k.shape[2] < 128:
        pytest.skip("v13 needs Nk >= 128")
    out = pli_hip.flash_attn_fwd(q, k, v, variant=80)
    err = max_err(out, torch_attention(q, k, v))
    assert err <= 2.0 ** -8 * v.abs().max().item(), f"{name}: {err:.4e}"
    assert_agree_to_rounding(pli_hip.flash_attn_fwd(q, k, v, variant=82), out, v)


# causal (bottom-right mask, Nk % 64 == 0; any diagonal offset -- rows run as
# Nq + ((-Nq) & 63) virtual rows since round 5): 83 persistent (pair walk
# where it tiles the grid; the second block of each pair streams its key
# tiles in the reversed order of tools/v13/kernel.py Gen.tile_of), 84 one
# block per workgroup heaviest first (forward order), 85 = 83 with the
# rescale path at nearly every tile
CAUSAL = [(4, 32, 8, 1024, 1024), (2, 32, 32, 2048, 2048), (2, 16, 4, 4096, 4096), (3, 40, 8, 1024, 1024),
          (2, 8, 2, 256, 512), (1, 4, 4, 128, 128), (1, 8, 8, 704, 768), (2, 4, 2, 320, 320),
          # pair walk with reversed second blocks and a diagonal offset (Nk - Nq = 1024 / 512)
          (4, 32, 8, 1024, 2048), (2, 32, 8, 2048, 2560),
          # offsets that are not a multiple of 64 (virtual rows): 212, 24 (pair walk over 1024 virtual
          # rows), 96, 28, 255 (one query row), 1
          (2, 8, 2, 300, 512), (4, 32, 8, 1000, 1024), (2, 16, 4, 4000, 4096), (1, 4, 4, 100, 128),
          (2, 8, 8, 1, 256), (1, 8, 2, 703, 704)]


@pytest.mark.parametrize("qmul", (1, 4))
@pytest.mark.parametrize("shape", CAUSAL, ids=lambda s: "b{}h{}kv{}q{}k{}".format(*s))
def test_v13_causal_vs_f64_full_tensor(shape, qmul):
    """Every output element of causal 83 / 84 / 85 against the f64 device
    reference with the bottom-right mask; 83 and 84 agree to rounding (the
    same arithmetic per tile, key tiles summed in another order where the
    pair walk reverses a block)."""
    import pli_hip
    q, k, v = inputs(shape, sum(shape) % 991)
    q = q * qmul
    ref = torch_attention(q, k, v, causal=True)
    tol = 1e-2 if qmul == 1 else 2.0 ** -8 * v.abs().max().item()
    outs = {}
    for var in (83, 84, 85):
        outs[var] = pli_hip.flash_attn_fwd(q, k, v, causal=True, variant=var)
        err = max_err(outs[var], ref)
        assert err <= tol, f"{shape} q*{qmul} causal variant {var}: max |err| {err:.4e} > {tol:.4e}"
    assert_agree_to_rounding(outs[83], outs[84], v)


def test_v13_causal_full_config_all_heads():
    """Causal at the bench config: all 256 heads against an fp32 torch
    attention with the mask; 85 within rounding of 83."""
    import pli_hip
    B, H, N, D = 8, 32, 4096, 128
    g = torch.Generator(device=DEV).manual_seed(5)
    q, k, v = (torch.randn(B, H, N, D, device=DEV, dtype=torch.bfloat16, generator=g) for _ in range(3))
    out = pli_hip.flash_attn_fwd(q, k, v, causal=True, variant=83)
    for b in range(B):
        ref = torch_attention(q[b:b + 1], k[b:b + 1], v[b:b + 1], dtype=torch.float32, heads_per_chunk=4,
                              causal=True)
        err = max_err(out[b:b + 1], ref)
        assert err <= 1e-2, f"causal batch {b}: max |err| {err:.4e} over its 32 heads"
    assert_agree_to_rounding(pli_hip.flash_attn_fwd(q, k, v, causal=True, variant=85), out, v)


def test_v13_causal_unaligned_offset_runs_v13():
    """Nk - Nq not a multiple of 64 (chunked prefill: 300 new rows over 512
    keys) runs attn_fwd_v13c on virtual rows, not v12: the default route
    equals 83 bitwise and differs from 74 in rounding only."""
    import pli_hip
    q, k, v = inputs((2, 8, 2, 300, 512), 3)
    out = pli_hip.flash_attn_fwd(q, k, v, causal=True)
    assert torch.equal(out, pli_hip.flash_attn_fwd(q, k, v, causal=True, variant=83))
    assert_agree_to_rounding(out, pli_hip.flash_attn_fwd(q, k, v, causal=True, variant=74), v)


@pytest.mark.parametrize("scale", (1.0, 0.25, 2.0 ** -0.5 / 8))
@pytest.mark.parametrize("causal", (False, True))
def test_v13_explicit_scale(scale, causal):
    """Non-default softmax scales (ch06/flash_attention.py:18-26 takes any
    scale): v13 applies c = scale * log2(e) in fp32, so c > 1 (scale 1.0)
    stays on it; against an f64 attention with the same scale."""
    import pli_hip
    q, k, v = inputs((2, 8, 2, 256, 512) if causal else (2, 8, 2, 300, 512), 13)
    var = 83 if causal else 80
    out = pli_hip.flash_attn_fwd(q, k, v, scale=scale, causal=causal, variant=var)
    g = q.shape[1] // k.shape[1]
    kf, vf = (t.double().repeat_interleave(g, dim=1) for t in (k, v))
    sc = (q.double() @ kf.transpose(-1, -2)) * scale
    if causal:
        nq, nk = q.shape[2], k.shape[2]
        i = torch.arange(nq, device=q.device)[:, None]
        j = torch.arange(nk, device=q.device)[None, :]
        sc = sc.masked_fill(j > i + (nk - nq), float("-inf"))
    ref = torch.softmax(sc, -1) @ vf
    err = max_err(out, ref)
    tol = 1e-2 if scale < 0.5 else 2.0 ** -8 * v.abs().max().item()
    assert err <= tol, f"scale {scale} causal {causal}: max |err| {err:.4e} > {tol:.4e}"


@pytest.mark.parametrize("causal", (False, True))
def test_v13_rescale_past_default_offset(causal):
    """Row maxima that grow by more than the default mu offset + 1 (63 log2
    units, PLI_V13_MUOFF in csrc/flash_attn.hip) inside one row: key 450
    aligned with query 500 (~ +100 log2 units in tile 7) and key 200 with
    query 300 (~ +75 in tile 3; both visible under the causal mask), so the
    default program takes its rescale path on its own; against the f64
    reference, and within rounding of 82 / 85 (the rescale path at nearly
    every tile)."""
    import numpy as np
    import pli_hip
    from oracle.numerics import round_to_bf16, seeded_normal
    q = seeded_normal((1, 2, 512, 128), 31, "bf16")
    k = seeded_normal((1, 2, 512, 128), 32, "bf16")
    v = seeded_normal((1, 2, 512, 128), 33, "bf16")
    k[:, :, 450] = 8.0 * np.sign(q[:, :, 500])
    k[:, :, 200] = 6.0 * np.sign(q[:, :, 300])
    q, k, v = dev(q), dev(round_to_bf16(k)), dev(v)
    c = 128 ** -0.5 * 1.4426950408889634
    rise = (q[0, :, 500].double() * k[0, :, 450].double()).sum(-1) * c
    assert rise.min().item() > 64, "the spike must exceed the default offset"
    var = 83 if causal else 80
    out = pli_hip.flash_attn_fwd(q, k, v, causal=causal, variant=var)
    err = max_err(out, torch_attention(q, k, v, causal=causal))
    assert err <= 2.0 ** -8 * v.abs().max().item(), f"causal {causal}: {err:.4e}"
    assert_agree_to_rounding(pli_hip.flash_attn_fwd(q, k, v, causal=causal, variant=var + 2), out, v)


@pytest.mark.parametrize("vexp", (-60, 50))
@pytest.mark.parametrize("variant", (80, 83, 71, 55))
def test_v13_v_range(variant, vexp):
    """|V| scaled by 2^-60 / 2^50 (exact in bf16): with P ~ 2^-62 at the row
    max (mu offset 62; the v12 / v10 bf16 threshold 64 likewise), P * V runs
    near the fp32 subnormal range or far above 1 -- the output, scaled back,
    against the f64 reference (the range the offset supports)."""
    import pli_hip
    causal = variant == 83
    q, k, v = inputs((2, 4, 2, 256, 512) if causal else (2, 4, 2, 300, 512), 41)
    vs = v * (2.0 ** vexp)
    assert torch.isfinite(vs).all() and (vs.abs() > 0).sum() == (v.abs() > 0).sum()
    out = pli_hip.flash_attn_fwd(q, k, vs, causal=causal, variant=variant)
    ref = torch_attention(q, k, v, causal=causal)
    err = max_err(out.double() * 2.0 ** -vexp, ref)
    assert err <= 1e-2, f"variant {variant} |V| * 2^{vexp}: max |err| {err:.4e}"


@pytest.mark.parametrize("dt,hd", (("bf16", 128), ("fp16", 128), ("bf16", 64), ("fp16", 64)))
@pytest.mark.parametrize("causal", (False, True))
def test_v13_gradual_max_growth(dt, hd, causal):
    """Scores that rise steadily with the key position (about 100 log2 units
    over the 1024 keys, ~6 per tile): the row max keeps growing, so the
    defer-max rescale runs many times, triggered by the accumulated row sum
    l (round 5's check; fp16: the P-bit check) rather than by one spike;
    against the f64 reference."""
    import pli_hip
    tdt = torch.bfloat16 if dt == "bf16" else torch.float16
    g = torch.Generator(device=DEV).manual_seed(61 + hd)
    B, H, N = 1, 4, 1024
    u = torch.randn(hd, device=DEV, generator=g, dtype=torch.float64)
    u = u / u.norm()
    c = hd ** -0.5 * 1.4426950408889634
    amp = 100.0 / c  # score rise (raw units) over the sequence: 100 log2 units after scaling
    q = (u * amp ** 0.5 + 0.3 * torch.randn(B, H, N, hd, device=DEV, generator=g, dtype=torch.float64))
    pos = torch.arange(N, device=DEV, dtype=torch.float64)[:, None] / N
    k = (pos * u * amp ** 0.5 + 0.3 * torch.randn(B, H, N, hd, device=DEV, generator=g, dtype=torch.float64))
    v = torch.randn(B, H, N, hd, device=DEV, generator=g, dtype=torch.float64)
    q, k, v = (t.to(tdt) for t in (q, k, v))
    assert torch.isfinite(q).all() and torch.isfinite(k).all()
    out = pli_hip.flash_attn_fwd(q, k, v, causal=causal)
    ref = torch_attention(q, k, v, causal=causal)
    err = max_err(out, ref)
    assert err <= 2.0 ** -8 * v.abs().max().item() + 1e-2, f"{dt} D{hd} causal {causal}: max |err| {err:.4e}"
