"""attn_fwd_v13 at head dim 64 (csrc/flash_v13_d64.hip, tools/v13/kernel.py
Gen(hd=64)): bf16 and fp16, plain and causal -- the default route for D = 64
since round 5 (before: v10, variants 55 / 60).  The reference's own GPU
tests run fp16 head_dim 64 (ch06/test_ch06.py:158-189) and
ch01.MultiHeadAttention d=512 h=8 is head_dim 64 (ch01/attention.py:45-72).

References: the f64 device attention over the whole output tensor
(ch06/attention_memory.py:19-33 in float64) at seam / GQA / ragged shapes,
plain and with Q x 4 (peaky rows); fp32 per head over all 256 heads at
B8 S4096 H32; the rescale sweep (82 / 85) within rounding of 80 / 83."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from test_gpu_flash_v12 import DEV, assert_agree_to_rounding, max_err, torch_attention

pytestmark = pytest.mark.gpu

TD = {"bf16": torch.bfloat16, "fp16": torch.float16}
SHAPES = [(4, 16, 4, 2048, 1024), (4, 32, 8, 1024, 128), (3, 40, 8, 1000, 320), (2, 4, 1, 2048, 192),
          (1, 2, 2, 1, 128), (2, 4, 4, 300, 128), (8, 36, 4, 256, 128), (1, 3, 1, 64, 256), (2, 2, 1, 200, 128)]
CAUSAL = [(4, 32, 8, 1024, 1024), (2, 16, 4, 2048, 2048), (3, 40, 8, 1024, 1024), (2, 8, 2, 256, 512),
          (1, 4, 4, 128, 128), (2, 4, 2, 320, 320), (4, 32, 8, 1024, 2048)]


def inputs64(shape, seed, dt):
    from oracle.numerics import seeded_normal
    B, H, Hkv, Nq, Nk = shape
    f = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV).to(TD[dt])  # noqa: E731
    return (f(seeded_normal((B, H, Nq, 64), seed, dt)), f(seeded_normal((B, Hkv, Nk, 64), seed + 1, dt)),
            f(seeded_normal((B, Hkv, Nk, 64), seed + 2, dt)))


@pytest.mark.parametrize("dt", ("bf16", "fp16"))
@pytest.mark.parametrize("qmul", (1, 4))
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "b{}h{}kv{}q{}k{}".format(*s))
def test_v13_d64_vs_f64_full_tensor(shape, qmul, dt):
    import pli_hip
    q, k, v = inputs64(shape, sum(shape) % 971, dt)
    q = q * qmul  # exact
    ref = torch_attention(q, k, v)
    tol = 1e-2 if qmul == 1 else 2.0 ** -8 * v.abs().max().item()
    outs = {}
    for var in (80, 81, 82):
        outs[var] = pli_hip.flash_attn_fwd(q, k, v, variant=var)
        err = max_err(outs[var], ref)
        assert err <= tol, f"{shape} {dt} q*{qmul} variant {var}: max |err| {err:.4e} > {tol:.4e}"
    assert torch.equal(outs[80], outs[81]), f"{shape}: 80 != 81"
    assert_agree_to_rounding(outs[82], outs[80], v)
    # the default route is this program (D = 64 routed to v10 before round 5),
    # or since round 6 attn_fwd_pp64 where its 512-row blocks fill the chip:
    # bitwise v13 for bf16, within rounding for fp16 (pp64h scales by fma,
    # v13h prescales Q)
    d = pli_hip.flash_attn_fwd(q, k, v)
    if pli_hip.last_route() == "attn_fwd_pp64h":
        assert_agree_to_rounding(d, outs[80], v)
    else:
        assert torch.equal(d, outs[80])


@pytest.mark.parametrize("dt", ("bf16", "fp16"))
@pytest.mark.parametrize("shape", CAUSAL, ids=lambda s: "b{}h{}kv{}q{}k{}".format(*s))
def test_v13_d64_causal_vs_f64_full_tensor(shape, dt):
    import pli_hip
    q, k, v = inputs64(shape, sum(shape) % 967, dt)
    ref = torch_attention(q, k, v, causal=True)
    outs = {}
    for var in (83, 84, 85):
        outs[var] = pli_hip.flash_attn_fwd(q, k, v, causal=True, variant=var)
        err = max_err(outs[var], ref)
        assert err <= 1e-2, f"{shape} {dt} causal variant {var}: max |err| {err:.4e}"
    assert_agree_to_rounding(outs[83], outs[84], v)
    assert_agree_to_rounding(outs[85], outs[83], v)


@pytest.mark.parametrize("dt", ("bf16", "fp16"))
@pytest.mark.parametrize("causal", (False, True))
def test_v13_d64_full_config_all_heads(causal, dt):
    """B8 S4096 H32 D64: all 256 heads against an fp32 torch attention."""
    import pli_hip
    B, H, N, D = 8, 32, 4096, 64
    g = torch.Generator(device=DEV).manual_seed(23)
    q, k, v = (torch.randn(B, H, N, D, device=DEV, dtype=TD[dt], generator=g) for _ in range(3))
    out = pli_hip.flash_attn_fwd(q, k, v, causal=causal)
    for b in range(B):
        ref = torch_attention(q[b:b + 1], k[b:b + 1], v[b:b + 1], dtype=torch.float32, heads_per_chunk=4,
                              causal=causal)
        err = max_err(out[b:b + 1], ref)
        assert err <= 1e-2, f"{dt} batch {b} causal {causal}: max |err| {err:.4e} over its 32 heads"


def test_v13_d64_strided_bshd_views():
    """[B,S,H,64] projections read in place (ch01 MHA layout) equal the
    contiguous [B,H,S,64] result bitwise."""
    import pli_hip
    g = torch.Generator(device=DEV).manual_seed(29)
    q, k, v = (torch.randn(2, 384, 8, 64, device=DEV, dtype=torch.float16, generator=g) for _ in range(3))
    contig = pli_hip.flash_attn_fwd(*(t.transpose(1, 2).contiguous() for t in (q, k, v)))
    strided = pli_hip.flash_attn_fwd(*(t.transpose(1, 2) for t in (q, k, v)))
    assert torch.equal(strided.contiguous(), contig)
