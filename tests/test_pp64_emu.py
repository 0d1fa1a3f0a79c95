"""attn_fwd_pp64's generated program (tools/v14/pp64.py, the body of
csrc/flash_pp64.hip) on the CPU: the 8-wave workgroup run by the emulator of
tools/v13/emu.py against a float64 attention on bf16-rounded inputs.  Covers
one and many key tiles (the stream parking on the last tile, the 6-slot
ring), the persistent walk (the stream crossing into the next block, the
block change inside a matrix phase), the rescale path at every tile (muoff 0) and after a late spike, GQA,
BSHD strides and a ragged query count, every A/B knob placement, the
committed header's freshness and the hazard pass's idempotence."""
from __future__ import annotations

import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))

from test_v13_emu import f64_attention  # noqa: E402
from v13.isa import S, analyse, finalize  # noqa: E402
from v14 import pp64  # noqa: E402
from v14 import pp64_run as P  # noqa: E402

CASES = [  # (B, H, Hkv, Nq, Nk, layout, muoff)
    (1, 1, 1, 512, 64, "bhsd", 62.0),     # one key tile: C(0), M(0), the tail
    (1, 1, 1, 512, 448, "bhsd", 62.0),    # seven tiles: the ring wraps, the stream parks
    (1, 1, 1, 512, 384, "bhsd", 0.0),     # the rescale path at every tile
    (1, 2, 1, 300, 320, "bshd", 62.0),    # GQA, BSHD strides, ragged Nq
    (2, 1, 1, 1024, 128, "bhsd", 62.0),   # two blocks per head, two batches
]
PERSISTENT = [  # (B, H, Hkv, Nq, Nk, layout, muoff, grid): blocks L, L + G, ... per workgroup
    (1, 2, 1, 1024, 256, "bhsd", 62.0, 1),    # four blocks on one workgroup
    (1, 2, 2, 1000, 384, "bshd", 62.0, 3),    # uneven walk, ragged Nq, BSHD
    (2, 2, 1, 512, 320, "bhsd", 0.0, 2),      # the rescale path at every tile across block changes
]


@pytest.mark.parametrize("dtype", ("bf16", "f16"))
@pytest.mark.parametrize("case", PERSISTENT, ids=lambda c: "b{}h{}kv{}q{}k{}-{}-mu{}-g{}".format(*c))
def test_pp64_persistent_walk_vs_f64(case, dtype):
    B, H, Hkv, Nq, Nk, lay, muoff, G = case
    if dtype == "f16":
        muoff = 4.0 if muoff > 0 else -1.0
    rng = np.random.default_rng(sum(case[:5]))
    q = rng.standard_normal((B, H, Nq, 64))
    k = rng.standard_normal((B, Hkv, Nk, 64))
    v = rng.standard_normal((B, Hkv, Nk, 64))
    o, em = P.run(q, k, v, muoff=muoff, layout=lay, dtype=dtype, grid=G)
    err = np.abs(o - f64_attention(q, k, v, dtype=dtype)).max()
    assert err <= (1e-2 if dtype == "bf16" else 5e-3), f"max |err| {err:.3e}"



@pytest.mark.parametrize("case", CASES, ids=lambda c: "b{}h{}kv{}q{}k{}-{}-mu{}".format(*c))
def test_pp64_program_vs_f64(case):
    B, H, Hkv, Nq, Nk, lay, muoff = case
    rng = np.random.default_rng(sum(case[:5]))
    q = rng.standard_normal((B, H, Nq, 64))
    k = rng.standard_normal((B, Hkv, Nk, 64))
    v = rng.standard_normal((B, Hkv, Nk, 64))
    P._PROG.pop("p", None)
    o, em = P.run(q, k, v, muoff=muoff, layout=lay)
    err = np.abs(o - f64_attention(q, k, v)).max()
    assert err <= 1e-2, f"max |err| {err:.3e}"
    if muoff <= 0:
        assert em.counts.get("v_sub_f32", 0) > 0, "the rescale path never ran"


def test_pp64_late_spike_rescale():
    """a key at tile 5 raises its rows' max far past muoff 62"""
    rng = np.random.default_rng(5)
    q = rng.standard_normal((1, 1, 512, 64))
    k = rng.standard_normal((1, 1, 448, 64))
    v = rng.standard_normal((1, 1, 448, 64))
    k[0, 0, 330] = 5.0 * q[0, 0].sum(0)  # scores ~ 5 (64 +- 180): growth >> 62 / c on many rows
    P._PROG.pop("p", None)
    o, em = P.run(q, k, v)
    assert em.counts.get("v_sub_f32", 0) > 0, "the rescale path never ran"
    err = np.abs(o - f64_attention(q, k, v)).max()
    assert err <= 1e-2, f"max |err| {err:.3e}"


KNOBS = [dict(dma_in="M", vr_in="M", rs_in="M"), dict(dma_in="M", vr_in="M", rs_in="M", split=8),
         dict(dma_in="C", vr_in="C", split=16, rs_in="M"), dict(dma_in="C", vr_in="M", rs_in="C")]


@pytest.mark.parametrize("kw", KNOBS, ids=lambda d: "-".join(f"{k}{v}" for k, v in sorted(d.items())))
def test_pp64_knobs_vs_f64(kw):
    rng = np.random.default_rng(11)
    q = rng.standard_normal((1, 1, 512, 64))
    k = rng.standard_normal((1, 1, 384, 64))
    v = rng.standard_normal((1, 1, 384, 64))
    P._PROG["p"], _ = finalize(pp64.PP64(tag="emu", **kw).build(in_kernarg=S(0, 2), in_wg=S(2), in_wave=S(3)))
    try:
        for muoff in (62.0, 0.0):
            o, _ = P.run(q, k, v, muoff=muoff)
            err = np.abs(o - f64_attention(q, k, v)).max()
            assert err <= 1e-2, f"{kw} muoff {muoff}: max |err| {err:.3e}"
    finally:
        P._PROG.pop("p", None)


F16_CASES = [(1, 1, 1, 512, 384, 4.0), (1, 1, 1, 512, 384, -1.0), (1, 2, 1, 300, 64, 4.0)]


@pytest.mark.parametrize("case", F16_CASES, ids=lambda c: "b{}h{}kv{}q{}k{}-mu{}".format(*c))
def test_pp64h_program_vs_f64(case):
    """the fp16 body: P-bit check in the vector phase, its rescale path there
    (muoff -1: every tile), fp16-rounded inputs"""
    B, H, Hkv, Nq, Nk, muoff = case
    rng = np.random.default_rng(sum(case[:5]))
    q = rng.standard_normal((B, H, Nq, 64))
    k = rng.standard_normal((B, Hkv, Nk, 64))
    v = rng.standard_normal((B, Hkv, Nk, 64))
    o, em = P.run(q, k, v, muoff=muoff, dtype="f16")
    err = np.abs(o - f64_attention(q, k, v, dtype="f16")).max()
    assert err <= 5e-3, f"max |err| {err:.3e}"
    if muoff < 0:
        assert em.counts.get("v_sub_f32", 0) > 0, "the rescale path never ran"


CAUSAL = [  # (B, H, Hkv, Nq, Nk, layout, muoff): bottom-right mask, Nq and Nk - Nq multiples of 64
    (1, 1, 1, 512, 512, "bhsd", 62.0),     # one block: each wave's diagonal tile, tiles past it
    (1, 2, 1, 1024, 1024, "bhsd", 62.0),   # two blocks of 8 / 16 tiles (heaviest first), GQA
    (1, 1, 1, 512, 768, "bshd", 62.0),     # diagonal offset 4 tiles, BSHD
    (1, 1, 1, 1024, 1024, "bhsd", 0.0),    # the rescale path at every tile (and not on the tiles past it)
    (1, 1, 1, 576, 576, "bhsd", 62.0),     # a ragged last block (rows past Nq)
]


@pytest.mark.parametrize("dtype", ("bf16", "f16"))
@pytest.mark.parametrize("case", CAUSAL, ids=lambda c: "b{}h{}kv{}q{}k{}-{}-mu{}".format(*c))
def test_pp64_causal_vs_f64(case, dtype):
    B, H, Hkv, Nq, Nk, lay, muoff = case
    if dtype == "f16":
        muoff = 4.0 if muoff > 0 else -1.0
    rng = np.random.default_rng(Nq + Nk)
    q = rng.standard_normal((B, H, Nq, 64))
    k = rng.standard_normal((B, Hkv, Nk, 64))
    v = rng.standard_normal((B, Hkv, Nk, 64))
    o, em = P.run(q, k, v, muoff=muoff, layout=lay, dtype=dtype, causal=True)
    err = np.abs(o - f64_attention(q, k, v, causal=True, dtype=dtype)).max()
    assert err <= 1e-2, f"max |err| {err:.3e}"
    if muoff <= 0:
        assert em.counts.get("v_sub_f32", 0) > 0, "the rescale path never ran"


def test_pp64_header_is_fresh():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "v14", "pp64.py"), "--check"])
    assert r.returncode == 0, "csrc/flash_pp64_asm.h is stale: run python tools/v14/pp64.py"


@pytest.mark.parametrize("causal", (False, True))
@pytest.mark.parametrize("dtype", ("bf16", "f16"))
def test_pp64_hazard_pass_idempotent(dtype, causal):
    prog, _ = finalize(pp64.PP64(dtype=dtype, causal=causal).build())
    assert not analyse(prog), "finalize left hazards or waits unresolved"


@pytest.mark.parametrize("causal", (False, True))
@pytest.mark.parametrize("dtype", ("bf16", "f16"))
def test_pp64_register_budget(dtype, causal):
    """128 VGPRs + 128 AGPRs (two waves per SIMD) and no SGPR past s99 / s32"""
    prog, _ = finalize(pp64.PP64(dtype=dtype, causal=causal).build())
    for ins in prog:
        for o in ins.ops:
            r = getattr(o, "r", o)
            f = getattr(r, "f", None)
            if f in ("v", "a"):
                assert r.i + r.n <= 128, ins.text()
            elif f == "s":
                assert 16 <= r.i and r.i + r.n <= 100 and not (r.i <= 32 < r.i + r.n), ins.text()
