"""attn_fwd_v13's generated program on the CPU (no GPU): the instruction
stream that csrc/flash_v13_asm.h holds is executed by tools/v13/emu.py and
compared with a float64 attention (the reference's naive_attention,
ch06/attention_memory.py:19-33) on bf16-rounded inputs.  This checks the
operand maps, LDS image layouts, DMA offsets, K/V stream and ring, the
persistent walk (grid smaller than the block count), GQA, BSHD strides,
ragged Nq and the defer-max rescale path; the hazard / wait-count pass is
checked for idempotence, and the committed header for staleness."""
from __future__ import annotations

import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))

from v13 import emu as E  # noqa: E402
from v13 import run as R  # noqa: E402
from v13.isa import analyse  # noqa: E402


def f64_attention(q, k, v, causal=False, dtype="bf16"):
    enc, dec = (E.f16_rne, E.f16_to_f32) if dtype == "f16" else (E.bf16_rne, E.bf16_to_f32)
    r = lambda x: dec(enc(x.astype(np.float32))).astype(np.float64)  # noqa: E731
    qf, kf, vf = r(q), r(k), r(v)
    g = q.shape[1] // k.shape[1]
    kf, vf = np.repeat(kf, g, axis=1), np.repeat(vf, g, axis=1)
    s = np.einsum("bhqd,bhkd->bhqk", qf, kf) / np.sqrt(q.shape[-1])
    if causal:  # bottom-right: row i sees keys j <= i + Nk - Nq (ch01/attention.py:66-67)
        nq, nk = q.shape[2], k.shape[2]
        s = np.where(np.arange(nk)[None, :] > np.arange(nq)[:, None] + nk - nq, -np.inf, s)
    s -= s.max(-1, keepdims=True)
    p = np.exp(s)
    p /= p.sum(-1, keepdims=True)
    return np.einsum("bhqk,bhkd->bhqd", p, vf)


CASES = [  # (B, H, Hkv, Nq, Nk, grid, layout, muoff, causal)
    # muoff 62: the product's offset (csrc/flash_attn.hip PLI_V13_MUOFF); 7: round 4's first builds
    (1, 1, 1, 256, 128, None, "bhsd", 7.0, False),      # one block, two key tiles
    (1, 2, 2, 256, 320, 1, "bhsd", 62.0, False),        # persistent: two blocks of five tiles on one workgroup
    (2, 2, 1, 200, 128, 1, "bshd", 7.0, False),         # GQA, ragged Nq, BSHD strides, nt = 2 across seams
    (1, 1, 1, 256, 256, None, "bhsd", 0.0, False),      # the rescale path at every tile (l >= 1 from the start)
    (1, 2, 1, 256, 512, None, "bhsd", 62.0, True),      # causal, Nq < Nk (diagonal offset 4 tiles)
    (1, 1, 1, 512, 512, None, "bhsd", 0.0, True),       # causal, two blocks, rescales on masked tiles
    (1, 2, 1, 200, 512, None, "bhsd", 62.0, True),      # causal, diagonal offset 312 (virtual rows: + 56)
    (1, 8, 8, 1000, 1024, 16, "bhsd", 62.0, True),      # causal pair walk over 1024 virtual rows (offset 24)
    (1, 1, 1, 100, 256, None, "bhsd", 0.0, True),       # causal, offset 156, rescales at every tile
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "b{}h{}kv{}q{}k{}g{}-{}-mu{}-causal{}".format(*c))
def test_v13_program_vs_f64(case):
    B, H, Hkv, Nq, Nk, grid, lay, muoff, causal = case
    rng = np.random.default_rng(sum(case[:5]))
    q = rng.standard_normal((B, H, Nq, 128))
    k = rng.standard_normal((B, Hkv, Nk, 128))
    v = rng.standard_normal((B, Hkv, Nk, 128))
    o, em = R.run(q, k, v, grid=grid, layout=lay, muoff=muoff, causal=causal)
    err = np.abs(o - f64_attention(q, k, v, causal)).max()
    assert err <= 1e-2, f"max |err| {err:.3e}"
    if muoff <= 0:
        assert em.counts.get("v_sub_f32", 0) > 0, "the rescale path never ran"


def test_v13_spike_rescale():
    """a key that raises one row's max by far more than 8 (log2) at a late
    tile: the rare path recomputes S, moves mu and rescales O and l"""
    rng = np.random.default_rng(3)
    q = rng.standard_normal((1, 1, 256, 128))
    k = rng.standard_normal((1, 1, 256, 128))
    v = rng.standard_normal((1, 1, 256, 128))
    k[0, 0, 200] = 40.0 * q[0, 0].mean(0)
    o, em = R.run(q, k, v)
    assert em.counts.get("v_sub_f32", 0) > 0
    err = np.abs(o - f64_attention(q, k, v)).max()
    assert err <= 2.0 ** -8 * np.abs(v).max(), f"max |err| {err:.3e}"


def test_v13_hazard_pass_is_idempotent():
    """the committed programs need no further padding or waits"""
    for causal in (False, True):
        for dtype in ("bf16", "f16"):
            assert analyse(R.program(causal=causal, dtype=dtype)) == {}


def _shipped_bodies():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import gen_flash_v13 as G
    return [(name, dict(G.PARAMS, **extra), causal) for name, extra, causal in G.BODIES + G.BODIES64]


@pytest.mark.parametrize("shipped", _shipped_bodies(), ids=lambda b: b[0])
def test_v13_hazard_pass_idempotent_on_every_shipped_body(shipped):
    """the exact body list tools/gen_flash_v13.py emits into both
    headers (16 bodies), each regenerated and re-analysed: the hazard / wait
    pass adds nothing to the committed program"""
    from v13.isa import finalize
    from v13.kernel import Gen
    name, params, causal = shipped
    prog, _ = finalize(Gen(tag="%=", causal=causal, **params).build())
    assert analyse(prog) == {}, name


def test_v13_header_is_current():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_flash_v13.py"), "--check"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def test_v13_spike_past_product_offset():
    """at the product's mu offset (62): key 200 aligned with query 230 raises
    that row's max by ~100 log2 units in tile 3, past the 63 the offset
    allows, so the rare path runs; P <= 2^-62 elsewhere stays exact"""
    rng = np.random.default_rng(5)
    q = rng.standard_normal((1, 1, 256, 128))
    k = rng.standard_normal((1, 1, 256, 128))
    v = rng.standard_normal((1, 1, 256, 128))
    k[0, 0, 200] = 8.0 * np.sign(q[0, 0, 230])
    assert (q[0, 0, 230] @ k[0, 0, 200]) / np.sqrt(128) * np.log2(np.e) > 64
    o, em = R.run(q, k, v, muoff=62.0)
    assert em.counts.get("v_sub_f32", 0) > 0, "the rescale path never ran"
    err = np.abs(o - f64_attention(q, k, v)).max()
    assert err <= 2.0 ** -8 * np.abs(v).max(), f"max |err| {err:.3e}"


F16_CASES = [  # (B, H, Hkv, Nq, Nk, grid, layout, muoff, causal): the fp16 program (Gen(dtype="f16"))
    (1, 2, 2, 256, 320, 1, "bhsd", 4.0, False),         # the launcher's fp16 offset, persistent
    (2, 2, 1, 200, 128, 1, "bshd", 4.0, False),         # GQA, ragged Nq, BSHD
    (1, 1, 1, 256, 256, None, "bhsd", -1.0, False),     # P-bit check: the rescale path at nearly every tile
    (1, 2, 1, 256, 512, None, "bhsd", 4.0, True),       # causal, diagonal offset
]


@pytest.mark.parametrize("case", F16_CASES, ids=lambda c: "f16-b{}h{}kv{}q{}k{}g{}-{}-mu{}-causal{}".format(*c))
def test_v13_f16_program_vs_f64(case):
    """fp16 Q / K / V / O on v_mfma_f32_16x16x32_f16, P packed to fp16 (RNE)
    and checked with the bit-14 test, against f64 on fp16-rounded inputs"""
    B, H, Hkv, Nq, Nk, grid, lay, muoff, causal = case
    rng = np.random.default_rng(7 + sum(case[:5]))
    q = rng.standard_normal((B, H, Nq, 128))
    k = rng.standard_normal((B, Hkv, Nk, 128))
    v = rng.standard_normal((B, Hkv, Nk, 128))
    o, em = R.run(q, k, v, grid=grid, layout=lay, muoff=muoff, causal=causal, dtype="f16")
    assert em.counts.get("v_mfma_f32_16x16x32_f16", 0) > 0 and em.counts.get("v_mfma_f32_16x16x32_bf16", 0) == 0
    err = np.abs(o - f64_attention(q, k, v, causal, dtype="f16")).max()
    assert err <= 1e-2, f"max |err| {err:.3e}"
    if muoff < 0:
        assert em.counts.get("v_sub_f32", 0) > 0, "the rescale path never ran"


D64_CASES = [  # (B, H, Hkv, Nq, Nk, grid, layout, muoff, causal, dtype): head dim 64 (Gen(hd=64))
    (1, 2, 2, 256, 320, 1, "bhsd", 62.0, False, "bf16"),   # persistent: two blocks of five tiles
    (2, 2, 1, 200, 128, 1, "bshd", 62.0, False, "bf16"),   # GQA, ragged Nq, BSHD
    (1, 1, 1, 256, 256, None, "bhsd", 0.0, False, "bf16"),  # the rescale path at every tile
    (1, 2, 1, 256, 512, None, "bhsd", 62.0, True, "bf16"),  # causal, diagonal offset
    (1, 2, 2, 256, 320, 1, "bhsd", 4.0, False, "f16"),     # fp16, persistent
    (1, 1, 1, 256, 256, None, "bhsd", -1.0, True, "f16"),   # fp16 causal, P-bit rescale at nearly every tile
]


@pytest.mark.parametrize("case", D64_CASES, ids=lambda c: "d64-b{}h{}kv{}q{}k{}g{}-{}-mu{}-causal{}-{}".format(*c))
def test_v13_d64_program_vs_f64(case):
    """head dim 64: the first halves of the D = 128 tile images, 4 DMA pieces
    per wave, 32 + 32 MFMAs per tile (reference ch01 MHA d=512 h=8 and the
    ch06 GPU tests run head_dim 64)"""
    B, H, Hkv, Nq, Nk, grid, lay, muoff, causal, dtype = case
    rng = np.random.default_rng(11 + sum(case[:5]))
    q = rng.standard_normal((B, H, Nq, 64))
    k = rng.standard_normal((B, Hkv, Nk, 64))
    v = rng.standard_normal((B, Hkv, Nk, 64))
    o, em = R.run(q, k, v, grid=grid, layout=lay, muoff=muoff, causal=causal, dtype=dtype)
    err = np.abs(o - f64_attention(q, k, v, causal, dtype=dtype)).max()
    assert err <= 1e-2, f"max |err| {err:.3e}"
    if muoff <= 0:
        assert em.counts.get("v_sub_f32", 0) > 0, "the rescale path never ran"


RAGGED_CASES = [  # (B, H, Hkv, Nq, Nk, grid, layout, muoff, D, dtype): Nk % 64 != 0 (Gen(ragged=True))
    (1, 2, 2, 256, 200, 1, "bhsd", 62.0, 128, "bf16"),   # persistent: the stream shifts and parks on a ragged tile
    (2, 2, 1, 200, 330, 1, "bshd", 62.0, 128, "bf16"),   # GQA, ragged Nq, BSHD strides
    (1, 1, 1, 256, 190, None, "bhsd", 0.0, 128, "bf16"),  # the rescale path at every tile, the last one too
    (1, 1, 1, 130, 65, None, "bhsd", 62.0, 128, "bf16"),  # Nk = 65: the last tile overlaps the first by 63 keys
    (1, 2, 2, 256, 200, 1, "bhsd", 4.0, 128, "f16"),     # fp16, persistent
    (1, 1, 1, 256, 190, None, "bhsd", -1.0, 128, "f16"),  # fp16 P-bit check: rescales at nearly every tile
    (1, 2, 2, 256, 330, 1, "bhsd", 62.0, 64, "bf16"),    # head dim 64, persistent
    (1, 1, 1, 256, 190, None, "bhsd", -1.0, 64, "f16"),   # head dim 64, fp16, rescales
]


@pytest.mark.parametrize("case", RAGGED_CASES,
                         ids=lambda c: "ragged-b{}h{}kv{}q{}k{}g{}-{}-mu{}-d{}-{}".format(*c))
def test_v13_ragged_program_vs_f64(case):
    """Nk not a multiple of 64 (non-causal): the last key tile streams from key
    Nk - 64 and the keys it shares with the tile before get P = 0; the heap
    is bounds-checked, so a read past the last head's rows would fail"""
    B, H, Hkv, Nq, Nk, grid, lay, muoff, D, dtype = case
    rng = np.random.default_rng(13 + sum(case[:5]))
    q = rng.standard_normal((B, H, Nq, D))
    k = rng.standard_normal((B, Hkv, Nk, D))
    v = rng.standard_normal((B, Hkv, Nk, D))
    o, em = R.run(q, k, v, grid=grid, layout=lay, muoff=muoff, dtype=dtype)
    err = np.abs(o - f64_attention(q, k, v, dtype=dtype)).max()
    assert err <= 1e-2, f"max |err| {err:.3e}"
    if muoff <= 0:
        assert em.counts.get("v_sub_f32", 0) > 0, "the rescale path never ran"


def test_v13_ragged_spikes():
    """a key in the overlap (counted once, in the tile before) and a key in
    the last tile's own part, each raising its row's max past the product's
    offset: the rare paths of the step and of the tail, with the overlap
    masked after the redo"""
    rng = np.random.default_rng(17)
    q = rng.standard_normal((1, 1, 256, 128))
    k = rng.standard_normal((1, 1, 200, 128))
    v = rng.standard_normal((1, 1, 200, 128))
    k[0, 0, 150] = 8.0 * np.sign(q[0, 0, 10])   # overlap: keys 136..191 are the last tile's first 56
    k[0, 0, 195] = 8.0 * np.sign(q[0, 0, 99])   # the last tile's own keys 192..199
    o, em = R.run(q, k, v, muoff=62.0)
    assert em.counts.get("v_sub_f32", 0) > 0, "the rescale path never ran"
    err = np.abs(o - f64_attention(q, k, v)).max()
    assert err <= 2.0 ** -8 * np.abs(v).max(), f"max |err| {err:.3e}"


def test_v13_ragged_hazard_pass_is_idempotent():
    for dtype in ("bf16", "f16"):
        for hd in (128, 64):
            for causal in (False, True):
                assert analyse(R.program(causal=causal, dtype=dtype, ragged=True, hd=hd)) == {}


RAGGED_CAUSAL_CASES = [  # (B, H, Hkv, Nq, Nk, grid, muoff, D, dtype): causal, Nk % 64 != 0
    (1, 2, 1, 200, 200, None, 62.0, 128, "bf16"),     # causal prefill of 200 tokens (one block)
    (1, 8, 8, 1000, 1000, 16, 62.0, 128, "bf16"),     # the pair walk: reversed blocks meet the shifted tile at position 3
    (1, 8, 8, 1000, 1000, 16, 0.0, 128, "bf16"),      # ... with the rescale path at every tile
    (2, 8, 2, 700, 770, 16, 62.0, 128, "bf16"),       # GQA, offset 70 (virtual rows + 6), remap walk
    (1, 2, 1, 65, 65, None, 62.0, 128, "bf16"),       # NT = 2: the last tile overlaps the first by 63 keys
    (1, 2, 2, 77, 300, None, 4.0, 128, "f16"),        # fp16, short query block
    (1, 8, 8, 990, 990, 16, 4.0, 64, "f16"),          # head dim 64, fp16, pair walk
]


@pytest.mark.parametrize("case", RAGGED_CAUSAL_CASES,
                         ids=lambda c: "ragged-causal-b{}h{}kv{}q{}k{}g{}-mu{}-d{}-{}".format(*c))
def test_v13_ragged_causal_program_vs_f64(case):
    """causal with Nk % 64 != 0: key tile NT - 1 streams from key Nk - 64 and
    its step masks the shifted keys by VALU (already-counted keys and keys
    past each row's diagonal), in both stream orders of the pair walk"""
    B, H, Hkv, Nq, Nk, grid, muoff, D, dtype = case
    rng = np.random.default_rng(19 + sum(case[:5]))
    q = rng.standard_normal((B, H, Nq, D))
    k = rng.standard_normal((B, Hkv, Nk, D))
    v = rng.standard_normal((B, Hkv, Nk, D))
    o, em = R.run(q, k, v, grid=grid, muoff=muoff, causal=True, dtype=dtype)
    err = np.abs(o - f64_attention(q, k, v, True, dtype=dtype)).max()
    assert err <= 1e-2, f"max |err| {err:.3e}"
    if muoff <= 0:
        assert em.counts.get("v_sub_f32", 0) > 0, "the rescale path never ran"


OLINE_CASES = [  # (B, H, Hkv, Nq, Nk, grid, muoff, D, dtype, causal): Gen(oline=True), the whole-line O stores
    (2, 2, 1, 200, 128, 1, 62.0, 128, "bf16", False),   # ragged Nq (row masks on both 8-row halves), seams
    (1, 8, 8, 1000, 1000, 16, 62.0, 128, "bf16", True),  # causal pair walk, virtual rows, ragged Nk
    (1, 2, 1, 77, 300, None, 4.0, 64, "f16", False),     # head dim 64: one 128-B line per row
]


@pytest.mark.parametrize("case", OLINE_CASES, ids=lambda c: "oline-b{}h{}kv{}q{}k{}g{}-mu{}-d{}-{}-causal{}".format(*c))
def test_v13_whole_line_stores_vs_f64(case):
    """the A/B epilogue that stores O as 8 rows x 128 B per instruction (DPP
    row_ror:8 exchange of the 64-B halves between lanes j and j + 8)"""
    B, H, Hkv, Nq, Nk, grid, muoff, D, dtype, causal = case
    rng = np.random.default_rng(23 + sum(case[:5]))
    q = rng.standard_normal((B, H, Nq, D))
    k = rng.standard_normal((B, Hkv, Nk, D))
    v = rng.standard_normal((B, Hkv, Nk, D))
    o, em = R.run(q, k, v, grid=grid, muoff=muoff, causal=causal, dtype=dtype, oline=True)
    assert em.counts.get("v_mov_b32_dpp", 0) > 0
    err = np.abs(o - f64_attention(q, k, v, causal, dtype=dtype)).max()
    assert err <= 1e-2, f"max |err| {err:.3e}"


def test_v13_seam_wait_knob():
    """Gen(seam_wait=True) (A/B knob): the block's first barrier waits for key
    tile 0 only -- vmcnt(NPW + 4 NDS) there, vmcnt(NPW) after the first
    block's setup -- and its program is hazard-clean; run on the emulator"""
    for hd, npw, nds in ((128, 8, 4), (64, 4, 2)):
        prog = R.program(causal=False, dtype="bf16", hd=hd, seam_wait=True)
        waits = [i.ops[0] for i in prog if i.op == "s_waitcnt"]
        assert f"vmcnt({npw + 4 * nds})" in waits and f"vmcnt({npw})" in waits
        assert analyse(prog) == {}
    rng = np.random.default_rng(5)
    q, k, v = (rng.standard_normal(s) for s in ((1, 2, 256, 128), (1, 2, 320, 128), (1, 2, 320, 128)))
    o, _ = R.run(q, k, v, grid=1, muoff=62.0, seam_wait=True)
    assert np.abs(o - f64_attention(q, k, v)).max() <= 1e-2


BEYOND_CASES = [  # (B, H, Hkv, Nq, Nk, grid, muoff, D, dtype): causal, Gen(beyond=True)
    (1, 1, 1, 512, 512, None, 0.0, 128, "bf16"),    # rescales at every tile, beside the skipped tiles
    (1, 8, 8, 1000, 1024, 16, 62.0, 128, "bf16"),   # pair walk, virtual rows
    (1, 8, 8, 990, 990, 16, 4.0, 64, "f16"),        # ragged, fp16 P-bit check, head dim 64
]


@pytest.mark.parametrize("case", BEYOND_CASES, ids=lambda c: "beyond-b{}h{}kv{}q{}k{}g{}-mu{}-d{}-{}".format(*c))
def test_v13_beyond_light_steps_vs_f64(case):
    """the A/B form whose tiles past a wave's diagonal skip QK and the
    softmax (P = 0, the deferred slices' S words = -inf) instead of running
    them on -inf C operands"""
    B, H, Hkv, Nq, Nk, grid, muoff, D, dtype = case
    rng = np.random.default_rng(29 + sum(case[:5]))
    q = rng.standard_normal((B, H, Nq, D))
    k = rng.standard_normal((B, Hkv, Nk, D))
    v = rng.standard_normal((B, Hkv, Nk, D))
    o, em = R.run(q, k, v, grid=grid, muoff=muoff, causal=True, dtype=dtype, beyond=True)
    err = np.abs(o - f64_attention(q, k, v, True, dtype=dtype)).max()
    assert err <= 1e-2, f"max |err| {err:.3e}"
    assert analyse(R.program(causal=True, dtype=dtype, hd=D, ragged=Nk % 64 != 0, beyond=True)) == {}


BALANCED_CASES = [  # (B, H, Hkv, Nq, Nk, grid, muoff, D, dtype): Gen(causal=True, balanced=True)
    (1, 2, 1, 256, 512, None, 62.0, 128, "bf16"),    # diagonal offset 4 tiles: plain tiles, then the group
    (1, 1, 1, 512, 512, None, 0.0, 128, "bf16"),     # two blocks, the rescale path at every tile (dead rows too)
    (1, 2, 1, 200, 512, None, 62.0, 128, "bf16"),    # virtual rows (+ 56), offset 312
    (1, 8, 8, 512, 512, 8, 62.0, 128, "bf16"),       # the pair walk: reversed blocks start on the group
    (1, 1, 1, 320, 320, None, 62.0, 128, "bf16"),    # 320 rows: the last block's group clipped at sTD + 1
    (1, 2, 1, 256, 512, None, 4.0, 128, "f16"),      # fp16 (P-bit check; row sums inside PV)
    (1, 1, 1, 256, 256, None, -1.0, 64, "f16"),      # D 64 fp16, rescales at nearly every tile
    (1, 2, 1, 256, 512, None, 62.0, 64, "bf16"),     # D 64
]


@pytest.mark.parametrize("case", BALANCED_CASES,
                         ids=lambda c: "balanced-b{}h{}kv{}q{}k{}g{}-mu{}-d{}-{}".format(*c))
def test_v13_balanced_causal_vs_f64(case):
    """causal with the interleaved q-block rows (Gen(balanced=True)): every
    wave has one 16-row q-block on each diagonal tile; group steps drop the
    dead q-blocks' chains, softmax and PV, and mask the diagonal q-block by
    VALU against LIMW"""
    B, H, Hkv, Nq, Nk, grid, muoff, D, dtype = case
    rng = np.random.default_rng(23 + sum(case[:5]) + D)
    q = rng.standard_normal((B, H, Nq, D))
    k = rng.standard_normal((B, Hkv, Nk, D))
    v = rng.standard_normal((B, Hkv, Nk, D))
    o, em = R.run(q, k, v, grid=grid, muoff=muoff, causal=True, dtype=dtype, balanced=True)
    err = np.abs(o - f64_attention(q, k, v, True, dtype=dtype)).max()
    assert err <= 1e-2, f"max |err| {err:.3e}"
    if muoff <= 0:
        assert em.counts.get("v_sub_f32", 0) > 0, "the rescale path never ran"


@pytest.mark.parametrize("D", (128, 64))
def test_v13_qscale_f16_first_tile_far_below_zero(D):
    """The fp16 QSCALE program (the product's non-causal fp16 bodies): every
    score of the first tile ~ -120 log2 units and lower after it
    (tests/stress_cases.py "first", shrunk).  The prologue must leave S
    shifted (c s - mu) in place for the next step's deferred slices, which
    exp S in place; reading it unshifted gives P = 2^(c s) = 0 for the rows'
    largest keys (caught on the GPU in round 6: non-finite output)."""
    rng = np.random.default_rng(31)
    q = rng.standard_normal((1, 1, 256, D))
    k = rng.standard_normal((1, 1, 256, D))
    v = rng.standard_normal((1, 1, 256, D))
    sgn = np.sign(q[:, :, :1])
    q = np.abs(q) * sgn
    k[:, :, :64] = -16.0 * sgn * np.abs(k[:, :, :64]) * np.sqrt(128 / D)
    k[:, :, 64:] = -20.0 * sgn * np.abs(k[:, :, 64:]) * np.sqrt(128 / D)
    o, em = R.run(q, k, v, muoff=4.0, dtype="f16", qscale=True)
    assert np.isfinite(o).all()
    err = np.abs(o - f64_attention(q, k, v, dtype="f16")).max()
    assert err <= 2.0 ** -8 * np.abs(v).max(), f"max |err| {err:.3e}"


@pytest.mark.parametrize("kind", ("randn", "q4", "first"))
def test_v13_qsplit_d64_matches_exact_scale(kind):
    """QSPLIT (Gen(qscale=True, qsplit=True), bf16 head dim 64): Q c as two
    bf16 parts, hi + lo, each QK chain running both -- QSCALE's fma saving
    without bf16(q c)'s 2^-9 score error.  Its error against f64 must be the
    exact-scale program's, on plain, q x 4 (peaky) and far-negative rows,
    where plain QSCALE is 2.5-8x worse"""
    rng = np.random.default_rng(41)
    q = rng.standard_normal((1, 1, 256, 64))
    k = rng.standard_normal((1, 1, 512, 64))
    v = rng.standard_normal((1, 1, 512, 64))
    if kind == "q4":
        q = q * 4.0
    elif kind == "first":
        sgn = np.sign(q[:, :, :1])
        q = np.abs(q) * sgn
        k[:, :, :64] = -16.0 * sgn * np.abs(k[:, :, :64]) * np.sqrt(2.0)
        k[:, :, 64:] = -20.0 * sgn * np.abs(k[:, :, 64:]) * np.sqrt(2.0)
    ref = f64_attention(q, k, v)
    o_exact, _ = R.run(q, k, v, muoff=62.0)
    o_split, _ = R.run(q, k, v, muoff=62.0, qscale=True, qsplit=True)
    e_exact, e_split = np.abs(o_exact - ref).max(), np.abs(o_split - ref).max()
    assert e_split <= 1.05 * e_exact + 1e-4, f"{kind}: qsplit {e_split:.3e} vs exact {e_exact:.3e}"


TAILEPI_CASES = [  # (B, H, Hkv, Nq, Nk, grid, muoff, causal, D)
    (1, 2, 2, 256, 320, 1, 62.0, False, 128),   # persistent: the next block's Q loads beside the stores
    (2, 2, 1, 200, 128, 1, 62.0, False, 128),   # ragged Nq: rows past Nq masked in the units
    (1, 1, 1, 256, 256, None, 0.0, False, 128),  # the rescale path at every tile, the last one too
    (1, 2, 1, 200, 512, None, 62.0, True, 128),  # causal virtual rows (the units' row shift)
    (1, 8, 8, 512, 512, 8, 62.0, True, 128),    # the pair walk (light tails keep the plain epilogue)
    (1, 2, 2, 256, 200, 1, 62.0, False, 64),    # head dim 64, ragged Nk
]


@pytest.mark.parametrize("case", TAILEPI_CASES,
                         ids=lambda c: "tailepi-b{}h{}kv{}q{}k{}g{}-mu{}-causal{}-d{}".format(*c))
def test_v13_tail_epilogue_vs_f64(case):
    """Gen(tailepi=2): the epilogue's normalise / pack / store of O as fills
    of the tail's PV(T), unit by unit once PV(T) has finished their d-blocks"""
    B, H, Hkv, Nq, Nk, grid, muoff, causal, D = case
    rng = np.random.default_rng(43 + sum(case[:5]) + D)
    q = rng.standard_normal((B, H, Nq, D))
    k = rng.standard_normal((B, Hkv, Nk, D))
    v = rng.standard_normal((B, Hkv, Nk, D))
    o, em = R.run(q, k, v, grid=grid, muoff=muoff, causal=causal, tailepi=2)
    err = np.abs(o - f64_attention(q, k, v, causal)).max()
    assert err <= 1e-2, f"max |err| {err:.3e}"
