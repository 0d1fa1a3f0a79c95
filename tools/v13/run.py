"""Host-side argument block of attn_fwd_v13 (the Python mirror of
launch_attn_v13 in csrc/flash_v13.hip) and an emulator driver."""
from __future__ import annotations

import math
import struct

import numpy as np

from . import emu as E
from .isa import S, finalize
from .kernel import AI, ARG_LAYOUT, Gen


def magic(d: int):
    """(m, l) with floor(x / d) == ((x * m) >> 31) >> l for 0 <= x < 2^31"""
    assert d >= 1
    l = 0
    while (1 << l) < d:
        l += 1
    m = -(-(1 << (31 + l)) // d)
    assert m < (1 << 32)
    return m, l


def pair_walk(nb, qblocks, G):
    """(walk, lgG8, lghq, per, hx): the causal pair walk where it tiles the
    grid exactly (launch_attn_v13's rule), else the remap walk"""
    bh = nb // qblocks
    w = G // 8
    hq = qblocks // 2
    pw2 = lambda x: x > 0 and (x & (x - 1)) == 0  # noqa: E731
    if (G < nb and qblocks % 2 == 0 and hq > 0 and w % hq == 0 and bh % 8 == 0 and (bh // 8) % (w // hq) == 0
            and nb % G == 0 and (nb // G) % 2 == 0 and pw2(w) and pw2(hq)):
        return 1, w.bit_length() - 1, hq.bit_length() - 1, w // hq, bh // 8
    return 2, 0, 0, 0, 0


def args_for(qa, ka, va, oa, B, H, Hkv, Nq, Nk, strides_el, scale, G, muoff=7.0, causal=False):
    """the argument block (ARG_LAYOUT); strides_el: 12 element strides
    (qb, qh, qn, kb, kh, kn, vb, vh, vn, ob, oh, on) of bf16 tensors"""
    st = [2 * s for s in strides_el]
    # causal: rows are virtual, shifted by s = (-Nq) & 63 so the diagonal sits
    # on 64-key tile boundaries (launch_attn_v13)
    Nqv = Nq + ((Nk - Nq) & 63) if causal else Nq
    qblocks = -(-Nqv // 256)
    nblocks = B * H * qblocks
    group = H // Hkv
    d = dict.fromkeys(ARG_LAYOUT, 0)
    for name, ptr in (("q", qa), ("k", ka), ("v", va), ("o", oa)):
        d[name], d[name + "_hi"] = ptr & 0xFFFFFFFF, ptr >> 32
    for name, val in (("qb", st[0]), ("qh", st[1]), ("kb", st[3]), ("kh", st[4]), ("vb", st[6]),
                      ("vh", st[7]), ("ob", st[9]), ("oh", st[10])):
        d[name], d[name + "_hi"] = val & 0xFFFFFFFF, val >> 32
    d["qn"], d["kn"], d["vn"], d["on"] = st[2], st[5], st[8], st[11]
    d["nq"], d["nt"], d["qblocks"], d["nblocks"] = Nq, -(-Nk // 64), qblocks, nblocks
    d["magq"], shq = magic(qblocks)
    d["magh"], shh = magic(H)
    d["magg"], shg = magic(group)
    assert H < (1 << 16)
    d["shifts"] = shq | (shh << 5) | (shg << 10) | (H << 16)
    if causal:
        walk, lg8, lghq, per, hx = pair_walk(nblocks, qblocks, G)
        d["cw"] = walk | (lg8 << 8) | (lghq << 16) | (per << 24)
        d["hx"] = hx
        d["offt"] = (Nk - Nqv) // 64
        if Nk % 64:  # ragged causal: P0 in the top byte of hx
            assert d["hx"] < (1 << 24)
            d["hx"] |= (64 - Nk % 64) << 24
    elif Nk % 64:
        d["cw"] = 64 - Nk % 64  # ragged: keys of the last (shifted) tile already counted
    d["c"] = struct.unpack("<I", struct.pack("<f", scale * 1.4426950408889634))[0]
    d["muoff"] = struct.unpack("<I", struct.pack("<f", muoff))[0]
    d["G"] = G
    d["tbk"], d["tbv"] = 64 * st[5], 64 * st[8]
    return np.array([d[n] for n in ARG_LAYOUT], dtype=np.uint32)


_PROG = {}


def program(**kw):
    key = tuple(sorted(kw.items()))
    if key not in _PROG:
        g = Gen(tag="emu", **kw)
        prog = g.build(in_kernarg=S(0, 2), in_wg=S(2), in_wave=S(3))
        prog, _ = finalize(prog)
        _PROG[key] = prog
    return _PROG[key]


def run(q, k, v, scale=None, grid=None, muoff=7.0, layout="bhsd", causal=False, structural=False, dtype="bf16", **kw):
    """q [B,H,Nq,D], k / v [B,Hkv,Nk,D] (D = 128 or 64) float arrays (rounded to bf16, or
    fp16 with dtype="f16") -> O [B,H,Nq,128] float32 from the emulated kernel.
    layout 'bshd' stores the tensors as [B,S,H,D] (strided heads)."""
    enc, dec = (E.f16_rne, E.f16_to_f32) if dtype == "f16" else (E.bf16_rne, E.bf16_to_f32)
    B, H, Nq, D = q.shape
    Hkv, Nk = k.shape[1], k.shape[2]
    ragged = Nk % 64 != 0
    assert D in (64, 128) and (Nk >= 128 if not ragged else Nk > 64)
    assert not causal or Nk - Nq >= 0
    if ragged:
        kw = dict(kw, ragged=True)
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    heap = E.Heap()

    def put(x, lay):
        b16 = enc(np.asarray(x, dtype=np.float32)).astype(np.uint16)
        if lay == "bshd":
            b16 = np.ascontiguousarray(b16.transpose(0, 2, 1, 3))
            Bx, Sx, Hx, Dx = b16.shape
            strides = (Sx * Hx * Dx, Dx, Hx * Dx)
        else:
            Bx, Hx, Sx, Dx = b16.shape
            strides = (Hx * Sx * Dx, Sx * Dx, Dx)
        return heap.alloc(b16.nbytes + 256, b16.tobytes()), strides

    qa, sq = put(q, layout)
    ka, sk = put(k, layout)
    va, sv = put(v, layout)
    oa = heap.alloc(B * H * Nq * D * 2 + 256)
    so = (Nq * H * D, D, H * D) if layout == "bshd" else (H * Nq * D, Nq * D, D)
    qblocks = -(-(Nq + ((Nk - Nq) & 63 if causal else 0)) // 256)
    nb = B * H * qblocks
    G = nb if grid is None else grid
    if causal and pair_walk(nb, qblocks, G)[0] != 1:
        G = nb  # the remap walk runs one block per workgroup
    args = args_for(qa, ka, va, oa, B, H, Hkv, Nq, Nk, list(sq) + list(sk) + list(sv) + list(so), scale, G, muoff,
                    causal)
    kaddr = heap.alloc(args.nbytes, args.tobytes())
    prog = program(causal=causal, dtype=dtype, **(dict(kw, hd=64) if D == 64 else kw))
    em = E.Emu(prog, heap, structural=structural)
    em.kbase = ka
    for wg in range(G):
        waves = []
        for wv in range(4):
            w = E.Wave()
            w.s[0], w.s[1], w.s[2], w.s[3] = kaddr & 0xFFFFFFFF, kaddr >> 32, wg, wv
            w.wid = (wg, wv)
            waves.append(w)
        em.lds[:] = 0
        em.run_wg(waves)
    if structural:
        return None, em
    raw = heap.view(oa)[:B * H * Nq * D * 2].view(np.uint16)
    if layout == "bshd":
        o = dec(raw.reshape(B, Nq, H, D).astype(np.uint32)).transpose(0, 2, 1, 3)
    else:
        o = dec(raw.reshape(B, H, Nq, D).astype(np.uint32))
    return np.ascontiguousarray(o), em
