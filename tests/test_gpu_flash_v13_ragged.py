"""attn_fwd_v13r / v13hr / v13rc / v13hrc (and the head-dim-64 forms): Nk not
a multiple of 64 on the generated v13 program, plain and causal
(tools/v13/kernel.py Gen(ragged=True), round 5; before, these shapes ran v12 /
v10).  The last key tile is streamed from key
Nk - 64 -- inside the head, so no K / V read leaves it -- and the keys it
shares with the tile before get P = 0 before the row sums and PV read them.

References share none of the kernel's code: the f64 device attention over the
whole output (the reference's naive_attention, ch06/attention_memory.py:
19-33), 1e-2 absolute on randn inputs and 2^-8 max|v| with Q scaled by 4
(peaky rows that take the rescale path); variant 82 (mu = max * c, the rescale
path at every tile, the tail's included) agrees with 80 to rounding on randn
inputs and meets the same f64 bound on the peaky ones; 80 (the
persistent walk) and 81 (one block per workgroup) are bitwise equal."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from test_gpu_flash_v12 import DEV, assert_agree_to_rounding, max_err, torch_attention

pytestmark = pytest.mark.gpu

# (B, H, Hkv, Nq, Nk, D): seams of the persistent walk with a shifted last
# tile in every block; Nk = 65 (the last tile overlaps the first by 63 keys),
# 127, 130, 190, 200, 333; GQA; a single query row
SHAPES = [(4, 32, 8, 1024, 130, 128), (3, 40, 8, 1000, 333, 128), (2, 4, 1, 2048, 190, 128),
          (1, 2, 2, 1, 65, 128), (2, 4, 4, 300, 127, 128), (8, 36, 4, 256, 200, 128),
          (4, 32, 8, 1024, 130, 64), (3, 40, 8, 1000, 333, 64), (2, 4, 4, 300, 127, 64), (1, 2, 2, 1, 77, 64)]


def inputs(shape, seed, dtype):
    from oracle.numerics import seeded_normal
    B, H, Hkv, Nq, Nk, D = shape
    name = "fp16" if dtype == torch.float16 else "bf16"
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV).to(dtype)  # noqa: E731
    return (t(seeded_normal((B, H, Nq, D), seed, name)), t(seeded_normal((B, Hkv, Nk, D), seed + 1, name)),
            t(seeded_normal((B, Hkv, Nk, D), seed + 2, name)))


@pytest.mark.parametrize("dtype", (torch.bfloat16, torch.float16), ids=("bf16", "fp16"))
@pytest.mark.parametrize("qmul", (1, 4))
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "b{}h{}kv{}q{}k{}d{}".format(*s))
def test_v13_ragged_vs_f64_full_tensor(shape, qmul, dtype):
    import pli_hip
    q, k, v = inputs(shape, sum(shape) % 991, dtype)
    q = q * qmul  # exact in bf16 / fp16
    ref = torch_attention(q, k, v)
    tol = 1e-2 if qmul == 1 else 2.0 ** -8 * v.abs().max().item()
    outs = {}
    for var in (80, 81, 82):
        outs[var] = pli_hip.flash_attn_fwd(q, k, v, variant=var)
        err = max_err(outs[var], ref)
        assert err <= tol, f"{shape} q*{qmul} variant {var}: max |err| {err:.4e} > {tol:.4e}"
    assert torch.equal(outs[80], outs[81]), f"{shape}: 80 != 81"
    assert torch.equal(outs[80], pli_hip.flash_attn_fwd(q, k, v)), f"{shape}: the default route is not 80"
    if qmul == 1:  # (peaky rows: both are within the f64 bound above; their P round against different mu)
        assert_agree_to_rounding(outs[80], outs[82], v)


def test_v13_ragged_overlap_spikes():
    """a key in the overlap of the last tile with the one before (counted
    once, in the earlier tile) and one in the last tile's own keys, each far
    above its row's other scores: the step's and the tail's rescale paths"""
    import pli_hip
    q, k, v = inputs((1, 2, 2, 256, 200, 128), 29, torch.bfloat16)
    k[0, 0, 150] = 8.0 * torch.sign(q[0, 0, 10])
    k[0, 1, 195] = 8.0 * torch.sign(q[0, 1, 99])
    ref = torch_attention(q, k, v)
    out = pli_hip.flash_attn_fwd(q, k, v, variant=80)
    err = max_err(out, ref)
    assert err <= 2.0 ** -8 * v.abs().max().item(), f"max |err| {err:.4e}"


# causal with Nk % 64 != 0 (attn_fwd_v13rc / v13hrc and the D64 pair): the
# shifted last tile masked by VALU on its shifted keys; prefill of N tokens
# (Nq = Nk), chunked prefill (Nq < Nk, any offset), the pair walk's reversed
# blocks, one query row, Nk = 65
CAUSAL_SHAPES = [(4, 32, 8, 1000, 1000, 128), (2, 16, 4, 4000, 4000, 128), (1, 4, 4, 200, 200, 128),
                 (2, 8, 2, 300, 430, 128), (1, 2, 2, 65, 65, 128), (2, 8, 8, 1, 77, 128),
                 (4, 32, 8, 1000, 1000, 64), (2, 8, 2, 300, 430, 64)]


@pytest.mark.parametrize("dtype", (torch.bfloat16, torch.float16), ids=("bf16", "fp16"))
@pytest.mark.parametrize("qmul", (1, 4))
@pytest.mark.parametrize("shape", CAUSAL_SHAPES, ids=lambda s: "b{}h{}kv{}q{}k{}d{}".format(*s))
def test_v13_ragged_causal_vs_f64_full_tensor(shape, qmul, dtype):
    import pli_hip
    q, k, v = inputs(shape, sum(shape) % 977, dtype)
    q = q * qmul
    ref = torch_attention(q, k, v, causal=True)
    tol = 1e-2 if qmul == 1 else 2.0 ** -8 * v.abs().max().item()
    outs = {}
    for var in (83, 84, 85):
        outs[var] = pli_hip.flash_attn_fwd(q, k, v, causal=True, variant=var)
        err = max_err(outs[var], ref)
        assert err <= tol, f"{shape} q*{qmul} causal variant {var}: max |err| {err:.4e} > {tol:.4e}"
    assert torch.equal(outs[83], pli_hip.flash_attn_fwd(q, k, v, causal=True)), f"{shape}: default route is not 83"
    if qmul == 1:
        assert_agree_to_rounding(outs[83], outs[84], v)


def test_v13_ragged_bench_scale():
    """Nq = Nk = 4000 at 8 heads x 2 batches (a prefill length that is not a
    multiple of 64): fp32 per-head reference over every head"""
    import pli_hip
    q, k, v = inputs((2, 8, 8, 4000, 4000, 128), 37, torch.bfloat16)
    out = pli_hip.flash_attn_fwd(q, k, v)
    ref = torch_attention(q, k, v, dtype=torch.float32, heads_per_chunk=4)
    err = max_err(out, ref)
    assert err <= 1e-2, f"max |err| {err:.4e}"
