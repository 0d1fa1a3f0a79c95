"""attn_fwd_pp64 / pp64h (csrc/flash_pp64.hip, tools/v14/pp64.py): head dim
64, bf16 / fp16, non-causal, two waves per SIMD in ping-pong, 512-row blocks
-- flash variants 86 (v13's mu offsets) and 87 (the rescale path at every
tile); 88, the default, picks 86 where its blocks fill the chip.

References: the f64 device attention over the whole output
(ch06/attention_memory.py:19-33 in float64) at block-seam / GQA / ragged-Nq /
single-tile shapes, plain and Q x 4; fp32 per head over all 256 heads at B8
S4096 H32 D64 (the bench's D = 64 leg); a late key that raises its rows' max
far past the offset (the rare path with muoff 62); BSHD views; and v13's D = 64
program (variant 80), which runs the same per-row arithmetic in the same
order, so the two agree bitwise (bf16; fp16 within rounding: v13h prescales
Q, pp64h scales the scores by fma); fp16 attention-sink rows at long
context (the mu-offset policy)."""
from __future__ import annotations

import pytest
import torch

from test_gpu_flash_v12 import DEV, assert_agree_to_rounding, max_err, torch_attention
from test_gpu_flash_v13_d64 import inputs64

pytestmark = pytest.mark.gpu

SHAPES = [(4, 16, 4, 2048, 1024), (4, 32, 8, 1024, 128), (3, 40, 8, 1000, 320), (2, 4, 1, 2048, 192),
          (1, 2, 2, 1, 128), (2, 4, 4, 300, 128), (8, 36, 4, 256, 128), (1, 3, 1, 64, 256), (2, 2, 1, 200, 128),
          (1, 4, 2, 600, 4096), (2, 8, 8, 513, 256),
          # the persistent walk (more blocks than workgroups, uneven per workgroup, ragged Nq)
          (5, 36, 4, 1000, 512), (2, 48, 8, 2100, 384)]


ROUTE = {"bf16": "attn_fwd_pp64", "fp16": "attn_fwd_pp64h"}


@pytest.mark.parametrize("dt", ("bf16", "fp16"))
@pytest.mark.parametrize("qmul", (1, 4))
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "b{}h{}kv{}q{}k{}".format(*s))
def test_pp64_vs_f64_full_tensor(shape, qmul, dt):
    import pli_hip
    q, k, v = inputs64(shape, sum(shape) % 971, dt)
    q = q * qmul  # exact
    ref = torch_attention(q, k, v)
    tol = 1e-2 if qmul == 1 else 2.0 ** -8 * v.abs().max().item()
    outs = {}
    for var in (86, 87):
        outs[var] = pli_hip.flash_attn_fwd(q, k, v, variant=var)
        assert pli_hip.last_route() == ROUTE[dt], pli_hip.last_route()
        err = max_err(outs[var], ref)
        assert err <= tol, f"{shape} {dt} q*{qmul} variant {var}: max |err| {err:.4e} > {tol:.4e}"
    assert_agree_to_rounding(outs[87], outs[86], v)
    v13 = pli_hip.flash_attn_fwd(q, k, v, variant=80)
    if dt == "bf16":  # v13's D = 64 program: the same rows, the same arithmetic in the same order
        assert torch.equal(outs[86], v13), f"{shape}: pp64 != v13"
    else:
        assert_agree_to_rounding(outs[86], v13, v)


@pytest.mark.parametrize("dt", ("bf16", "fp16"))
def test_pp64_full_config_all_heads(dt):
    """B8 S4096 H32 D64 (the bench's D = 64 legs): all 256 heads against an
    fp32 torch attention, and v13's D = 64 program (bf16: bitwise)."""
    import pli_hip
    B, H, N, D = 8, 32, 4096, 64
    g = torch.Generator(device=DEV).manual_seed(23)
    td = torch.bfloat16 if dt == "bf16" else torch.float16
    q, k, v = (torch.randn(B, H, N, D, device=DEV, dtype=td, generator=g) for _ in range(3))
    out = pli_hip.flash_attn_fwd(q, k, v)  # the default route (88) at this shape
    assert pli_hip.last_route() == ROUTE[dt]
    for b in range(B):
        ref = torch_attention(q[b:b + 1], k[b:b + 1], v[b:b + 1], dtype=torch.float32, heads_per_chunk=4)
        err = max_err(out[b:b + 1], ref)
        assert err <= 1e-2, f"{dt} batch {b}: max |err| {err:.4e} over its 32 heads"
    v13 = pli_hip.flash_attn_fwd(q, k, v, variant=80)
    if dt == "bf16":
        assert torch.equal(out, v13)
    else:
        assert_agree_to_rounding(out, v13, v)


@pytest.mark.parametrize("at", (5, 700, 2047))
def test_pp64_late_spike_rescale(at):
    """one key raises many rows' max by hundreds of log2 units at key `at`
    (past muoff 62): the rare path recomputes S, moves mu and rescales O and l"""
    import pli_hip
    q, k, v = inputs64((1, 4, 4, 1024, 2048), 41, "bf16")
    k[:, :, at] = (q.float().sum(2) * 5).to(k.dtype)  # scores ~ 5 (64 +- 256)
    ref = torch_attention(q, k, v)
    out = pli_hip.flash_attn_fwd(q, k, v, variant=86)
    assert pli_hip.last_route() == "attn_fwd_pp64"
    err = max_err(out, ref)
    assert err <= 1e-2, f"spike at {at}: max |err| {err:.4e}"
    assert torch.equal(out, pli_hip.flash_attn_fwd(q, k, v, variant=80))


def test_pp64_strided_bshd_views():
    """[B,S,H,64] projections read in place equal the contiguous result bitwise."""
    import pli_hip
    g = torch.Generator(device=DEV).manual_seed(29)
    q, k, v = (torch.randn(2, 640, 8, 64, device=DEV, dtype=torch.bfloat16, generator=g) for _ in range(3))
    contig = pli_hip.flash_attn_fwd(*(t.transpose(1, 2).contiguous() for t in (q, k, v)), variant=86)
    strided = pli_hip.flash_attn_fwd(*(t.transpose(1, 2) for t in (q, k, v)), variant=86)
    assert pli_hip.last_route() == "attn_fwd_pp64"
    assert torch.equal(strided.contiguous(), contig)


def test_pp64_falls_back_where_it_does_not_apply():
    """causal and ragged Nk take v13's programs under variant 86; the default
    route (88) keeps v13 where pp64's 512-row blocks would not fill the chip"""
    import pli_hip
    q, k, v = inputs64((2, 8, 8, 512, 512), 5, "bf16")
    pli_hip.flash_attn_fwd(q, k, v)
    assert pli_hip.last_route() == "attn_fwd_v13_d64"
    q, k, v = inputs64((4, 32, 32, 1024, 256), 5, "bf16")
    pli_hip.flash_attn_fwd(q, k, v)
    assert pli_hip.last_route() == "attn_fwd_pp64"
    q, k, v = inputs64((1, 2, 2, 256, 320), 5, "fp16")
    pli_hip.flash_attn_fwd(q, k, v)
    assert pli_hip.last_route() == "attn_fwd_v13h_d64"
    q, k, v = inputs64((1, 2, 2, 200, 320), 5, "fp16")  # causal, Nq % 64 != 0
    pli_hip.flash_attn_fwd(q, k, v, causal=True, variant=86)
    assert pli_hip.last_route() == "attn_fwd_v13hc_d64"
    q, k, v = inputs64((1, 2, 2, 200, 320), 5, "bf16")  # causal, Nq % 64 != 0
    pli_hip.flash_attn_fwd(q, k, v, causal=True, variant=86)
    assert pli_hip.last_route() == "attn_fwd_v13c_d64"
    q, k, v = inputs64((1, 2, 2, 256, 300), 5, "bf16")
    pli_hip.flash_attn_fwd(q, k, v, variant=86)
    assert pli_hip.last_route() == "attn_fwd_v13r_d64"


@pytest.mark.parametrize("N", (8192, 32768))
@pytest.mark.parametrize("d", (14, 18, 22))
def test_pp64h_attention_sink_long_context(d, N):
    """fp16 attention-sink rows (one dominant key, N - 1 keys d log2 units
    under it) on pp64h with the launcher's Nk-dependent mu offset
    (v13_muoff_f16; tests/test_gpu_flash_v13_f16.py holds the v13h twin)"""
    import pli_hip
    D, Nq = 64, 512
    g = torch.Generator(device=DEV).manual_seed(1000 * d + N % 997)
    c = D ** -0.5 * 1.4426950408889634
    q = torch.zeros(1, 1, Nq, D, device=DEV, dtype=torch.float64)
    q[..., 0] = 1.0
    q[..., 1] = 0.05 * torch.randn(1, 1, Nq, device=DEV, dtype=torch.float64, generator=g)
    k = torch.zeros(1, 1, N, D, device=DEV, dtype=torch.float64)
    a = 8.0 / c
    delta = d + 2.0 * torch.rand(N, device=DEV, dtype=torch.float64, generator=g) - 1.0
    k[0, 0, :, 0] = a - delta / c
    k[0, 0, 0, 0] = a
    k[0, 0, :, 1] = torch.randn(N, device=DEV, dtype=torch.float64, generator=g)
    v = torch.randn(1, 1, N, D, device=DEV, dtype=torch.float64, generator=g)
    q, k, v = (t.to(torch.float16) for t in (q, k, v))
    ref = torch_attention(q, k, v)
    out = pli_hip.flash_attn_fwd(q, k, v, variant=86)
    assert pli_hip.last_route() == "attn_fwd_pp64h"
    err = max_err(out, ref)
    assert err <= 5e-3, f"N {N} d {d}: max |err| {err:.3e}"


CROUTE = {"bf16": "attn_fwd_pp64c", "fp16": "attn_fwd_pp64hc"}
CAUSAL = [(4, 32, 8, 1024, 1024), (2, 16, 4, 2048, 2048), (3, 40, 8, 1024, 1024), (2, 8, 2, 256, 512),
          (1, 4, 4, 128, 128), (4, 32, 8, 1024, 2048), (2, 8, 2, 576, 576), (1, 2, 1, 64, 4096)]


@pytest.mark.parametrize("dt", ("bf16", "fp16"))
@pytest.mark.parametrize("shape", CAUSAL, ids=lambda s: "b{}h{}kv{}q{}k{}".format(*s))
def test_pp64_causal_vs_f64_full_tensor(shape, dt):
    """the causal forms (bottom-right; Nq and Nk - Nq multiples of 64): the
    diagonal tiles masked by VALU, P = 0 past them; 87 (rescale every tile)
    within rounding of 86, and v13c's D = 64 program within rounding"""
    import pli_hip
    q, k, v = inputs64(shape, sum(shape) % 967, dt)
    ref = torch_attention(q, k, v, causal=True)
    outs = {}
    for var in (86, 87):
        outs[var] = pli_hip.flash_attn_fwd(q, k, v, causal=True, variant=var)
        assert pli_hip.last_route() == CROUTE[dt], pli_hip.last_route()
        err = max_err(outs[var], ref)
        assert err <= 1e-2, f"{shape} {dt} causal variant {var}: max |err| {err:.4e}"
    assert_agree_to_rounding(outs[87], outs[86], v)
    assert_agree_to_rounding(outs[86], pli_hip.flash_attn_fwd(q, k, v, causal=True, variant=83), v)


@pytest.mark.parametrize("dt", ("bf16", "fp16"))
def test_pp64_causal_full_config_all_heads(dt):
    """B8 S4096 H32 D64 causal (the bench's causal D = 64 legs): all 256 heads
    against an fp32 torch attention"""
    import pli_hip
    B, H, N, D = 8, 32, 4096, 64
    g = torch.Generator(device=DEV).manual_seed(31)
    td = torch.bfloat16 if dt == "bf16" else torch.float16
    q, k, v = (torch.randn(B, H, N, D, device=DEV, dtype=td, generator=g) for _ in range(3))
    out = pli_hip.flash_attn_fwd(q, k, v, causal=True, variant=86)
    assert pli_hip.last_route() == CROUTE[dt]
    for b in range(B):
        ref = torch_attention(q[b:b + 1], k[b:b + 1], v[b:b + 1], dtype=torch.float32, heads_per_chunk=4,
                              causal=True)
        err = max_err(out[b:b + 1], ref)
        assert err <= 1e-2, f"{dt} batch {b}: max |err| {err:.4e} over its 32 heads"
