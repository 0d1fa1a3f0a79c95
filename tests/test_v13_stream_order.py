"""The causal K/V stream of attn_fwd_v13c, structurally (CPU, no GPU): the
generated program runs in tools/v13/emu.py with only its scalar and control
flow executed, every LDS-DMA logging its source base, and the key tiles each
workgroup streams are compared with an independent model of the walk:

* the pair walk (tools/v13/kernel.py block_params walk 1, the causal
  default where it tiles the grid): workgroup l's blocks are query heights
  QB-1-a (forward, tiles 0 .. T-1) then a (reversed: T-4 .. T-1, then
  T-5 down to 0 -- Gen.tile_of), T = min(nt, 4 qblk + 4 + (Nk - Nq) / 64);
* the remap walk (walk 2, one block per workgroup, heaviest first): forward.

The reference's causal mask is ch01/attention.py:66-67 (bottom-right for
Nq < Nk, ch02/cached_generation.py:85-91); the numbers themselves are
checked by tests/test_v13_emu.py and tests/test_gpu_flash_v13.py."""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))

from v13 import run as R  # noqa: E402


def stream(B, H, Hkv, Nq, Nk, grid):
    z = np.zeros
    _, em = R.run(z((B, H, Nq, 128)), z((B, Hkv, Nk, 128)), z((B, Hkv, Nk, 128)), grid=grid, causal=True,
                  structural=True)
    row_b, head_b = 128 * 2, Nk * 128 * 2
    seq = {}
    for (wg, wv), base, off, _m0 in em.dma_log:
        rel = base - em.kbase
        if wv == 0 and off == 0 and 0 <= rel < B * Hkv * head_b:  # wave 0's first K piece of each tile
            seq.setdefault(wg, []).append((rel // head_b, (rel % head_b) // row_b))  # (kv head, first key row)
    return seq


def expected(B, H, Hkv, Nq, Nk, G):
    Nqv = Nq + ((Nk - Nq) & 63)  # virtual rows (launch_attn_v13): the diagonal on tile boundaries
    QB, nt, offt = -(-Nqv // 256), -(-Nk // 64), (Nk - Nqv) // 64
    row = lambda t: Nk - 64 if t == nt - 1 else 64 * t  # noqa: E731  (ragged Nk: the last tile shifted back)
    nb = B * H * QB
    walk, lg8, lghq, per, hx = R.pair_walk(nb, QB, G)
    out = {}
    for L in range(G):
        seq = []
        for l in range(L, nb, G):
            if walk == 1:
                x, l8 = l & 7, l >> 3
                j, wg = l8 >> lg8, l8 & ((1 << lg8) - 1)
                wgq, a = wg >> lghq, wg & ((1 << lghq) - 1)
                bh = x * hx + wgq + per * (j >> 1)
                qblk, rev = (a, True) if j & 1 else (QB - 1 - a, False)
            else:  # remap walk, heaviest first
                n8, r8 = nb >> 3, nb & 7
                x, i = l & 7, l >> 3
                lb = x * n8 + min(x, r8) + i
                bh, r = divmod(lb, QB)
                qblk, rev = QB - 1 - r, False
            T = min(nt, 4 * qblk + 4 + offt)
            rev = rev and T >= 4
            order = list(range(T - 4, T)) + list(range(T - 5, -1, -1)) if rev else list(range(T))
            b, h = divmod(bh, H)
            seq += [(b * Hkv + h // (H // Hkv), row(t)) for t in order]
        out[L] = seq
    return walk, out


@pytest.mark.parametrize("shape", [(1, 8, 8, 1024, 1024, 16), (1, 8, 4, 1024, 1280, 16), (2, 8, 2, 512, 512, 16),
                                   (1, 8, 8, 1024, 1024, None), (1, 8, 8, 1000, 1024, 16), (1, 8, 4, 990, 1280, 16),
                                   (1, 8, 4, 700, 1280, None),
                                   # ragged Nk: the shifted last tile in both orders, the park on tile 0
                                   (1, 8, 8, 1000, 1000, 16), (1, 8, 4, 900, 1250, 16), (2, 8, 2, 700, 770, None)],
                         ids=lambda s: "b{}h{}kv{}q{}k{}g{}".format(*s))
def test_causal_stream_order(shape):
    B, H, Hkv, Nq, Nk, grid = shape
    QB = -(-(Nq + ((Nk - Nq) & 63)) // 256)
    G = grid or B * H * QB
    walk, want = expected(B, H, Hkv, Nq, Nk, G)
    assert walk == (1 if grid else 2)
    got = stream(B, H, Hkv, Nq, Nk, grid)
    for L, seq in want.items():
        # past its last block the stream parks on one tile (at most two extra loads)
        assert got[L][:len(seq)] == seq, f"workgroup {L}: {got[L][:len(seq)]} != {seq}"
        assert len(got[L]) - len(seq) <= 2


def ragged_stream(B, H, Hkv, Nq, Nk, grid):
    """non-causal, Nk % 64 != 0: (kv head, first key row) of every tile each
    workgroup streams (wave 0's first K piece)"""
    z = np.zeros
    _, em = R.run(z((B, H, Nq, 128)), z((B, Hkv, Nk, 128)), z((B, Hkv, Nk, 128)), grid=grid, structural=True)
    row_b, head_b = 128 * 2, Nk * 128 * 2
    seq = {}
    for (wg, wv), base, off, _m0 in em.dma_log:
        rel = base - em.kbase
        if wv == 0 and off == 0 and 0 <= rel < B * Hkv * head_b:
            assert (rel % head_b) % row_b == 0
            seq.setdefault(wg, []).append((rel // head_b, (rel % head_b) // row_b))
    return seq


@pytest.mark.parametrize("shape", [(1, 8, 8, 512, 200, 16), (2, 4, 2, 300, 130, 8), (1, 16, 4, 256, 65, None)],
                         ids=lambda s: "b{}h{}kv{}q{}k{}g{}".format(*s))
def test_ragged_stream_stays_in_head(shape):
    """Gen(ragged=True): every block streams key rows 0, 64, ..., 64 (nt - 2)
    and then Nk - 64 (the last tile overlapping the one before), so no K / V
    read leaves its head; the persistent walk's seams and park included"""
    B, H, Hkv, Nq, Nk, grid = shape
    QB, nt = -(-Nq // 256), -(-Nk // 64)
    nb = B * H * QB
    G = grid or nb
    rows = [64 * t for t in range(nt - 1)] + [Nk - 64]
    got = ragged_stream(B, H, Hkv, Nq, Nk, grid)
    for L in range(G):
        seq = []
        for l in range(L, nb, G):
            n8, r8 = (0, 8) if nb < 8 else (nb >> 3, nb & 7)
            x, i = l & 7, l >> 3
            lb = x * n8 + min(x, r8) + i
            bh = lb // QB
            b, h = divmod(bh, H)
            seq += [(b * Hkv + h // (H // Hkv), r) for r in rows]
        assert got[L][:len(seq)] == seq, f"workgroup {L}: {got[L][:len(seq)]} != {seq}"
        # past its last block the stream parks on its last (shifted) tile
        assert all(t == seq[-1] for t in got[L][len(seq):]) and len(got[L]) - len(seq) <= 2
