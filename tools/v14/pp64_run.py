"""Emulator driver for attn_fwd_pp64 (tools/v14/pp64.py): the argument block
of launch_attn_v13 with 512-row blocks (csrc/flash_v13.hip, pp64 route) and
one workgroup of 8 waves per block."""
from __future__ import annotations

import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from v13 import emu as E  # noqa: E402
from v13 import run as R  # noqa: E402
from v13.isa import S, finalize  # noqa: E402
from v14.pp64 import PP64  # noqa: E402

_PROG = {}


def program(dtype="bf16", causal=False):
    key = ("p" if dtype == "bf16" else dtype) + ("c" if causal else "")
    if key not in _PROG:
        prog = PP64(tag="emu", dtype=dtype, causal=causal).build(in_kernarg=S(0, 2), in_wg=S(2), in_wave=S(3))
        _PROG[key], _ = finalize(prog)
    return _PROG[key]


def run(q, k, v, scale=None, muoff=62.0, layout="bhsd", dtype="bf16", grid=None, causal=False):
    """q [B,H,Nq,64], k / v [B,Hkv,Nk,64] -> O [B,H,Nq,64] (inputs rounded to
    bf16, or fp16 with dtype="f16")"""
    enc, dec = (E.f16_rne, E.f16_to_f32) if dtype == "f16" else (E.bf16_rne, E.bf16_to_f32)
    B, H, Nq, D = q.shape
    Hkv, Nk = k.shape[1], k.shape[2]
    assert D == 64 and Nk % 64 == 0 and Nk >= 64
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
    qblocks = -(-Nq // 512)
    nb = B * H * qblocks
    G = nb if grid is None else grid  # grid < nb: the persistent walk (L, L + G, ...)
    args = R.args_for(qa, ka, va, oa, B, H, Hkv, Nq, Nk, list(sq) + list(sk) + list(sv) + list(so), scale, G,
                      muoff, False)
    from v13.kernel import AI
    args[AI["qblocks"]], args[AI["nblocks"]] = qblocks, nb
    args[AI["magq"]], shq = R.magic(qblocks)
    args[AI["shifts"]] = (int(args[AI["shifts"]]) & ~31) | shq
    if causal:  # bottom-right, Nq and Nk - Nq multiples of 64: the remap walk, heaviest first
        assert Nq % 64 == 0 and (Nk - Nq) % 64 == 0 and Nk >= Nq and grid is None
        args[AI["cw"]], args[AI["offt"]] = 2, (Nk - Nq) // 64
    kaddr = heap.alloc(args.nbytes, args.tobytes())
    em = E.Emu(program(dtype, causal), heap)
    for wg in range(G):
        waves = []
        for wv in range(8):
            w = E.Wave()
            w.s[0], w.s[1], w.s[2], w.s[3] = kaddr & 0xFFFFFFFF, kaddr >> 32, wg, wv
            w.wid = (wg, wv)
            waves.append(w)
        em.lds[:] = 0
        em.run_wg(waves)
    raw = heap.view(oa)[:B * H * Nq * D * 2].view(np.uint16)
    if layout == "bshd":
        o = dec(raw.reshape(B, Nq, H, D).astype(np.uint32)).transpose(0, 2, 1, 3)
    else:
        o = dec(raw.reshape(B, H, Nq, D).astype(np.uint32))
    return np.ascontiguousarray(o), em
