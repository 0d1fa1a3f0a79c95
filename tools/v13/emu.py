"""CPU emulator for the generated attn_fwd_v13 program (test infrastructure).

Executes the same `Ins` list that tools/gen_flash_v13.py prints for hipcc,
one workgroup at a time: 4 waves x 64 lanes run in turn between s_barriers,
LDS-DMA and loads complete at issue (s_waitcnt is a no-op here; the hazard /
wait-count pass in tools/v13/isa.py is checked separately), every global and
LDS access is bounds-checked.  What it proves: the operand maps, LDS image
layouts, DMA offsets, stream / ring bookkeeping, persistent walk, softmax and
defer-max logic and the epilogue produce the right output.  What it does not:
timing, wait counts, races between waves inside one barrier interval.

Semantics of the less common instructions, as this file implements them:
  v_mfma_f32_16x16x32_bf16 / _f16  A lane l: row l&15, k = 8(l>>4)+j (j-th bf16 of
      the 4 registers, low half first); B lane l: col l&15, same k; C/D lane
      l: col l&15, rows 4(l>>4)+r (register r)
  ds_read_b64_tr_b16  per 16-lane group, lane 4q+p addresses row q, columns
      4p..4p+3 of a 4 x 16 block; lane i gets column i, row q in element q
  global_load_lds_dwordx4  global = sbase + voffset + offset, LDS = M0 +
      offset + 16 * lane
  v_permlane16_swap_b32 a, b  rows (16 lanes) 1, 3 of a <-> rows 0, 2 of b
  v_permlane32_swap_b32 a, b  lanes 32-63 of a <-> lanes 0-31 of b
  v_exp_f32 ... clamp  VOP3 clamp of the result to [0, 1]
  v_mov_b32_dpp d, s row_ror:N ... bank_mask:M  lane i of each 16-lane row
      reads s from lane (i - N) mod 16 of that row; only lanes whose bank
      (i & 15) >> 2 is set in M (and in exec) are written
"""
from __future__ import annotations

import struct

import numpy as np

from .isa import Neg, Reg

LANES = 64
# ds_read_b64_tr_b16: source lane and byte offset of lane l's four words
_TR_SRC = np.array([[16 * (l // 16) + 4 * q + ((l % 16) >> 2) for q in range(4)] for l in range(64)])
_TR_OFF = np.array([2 * ((l % 16) & 3) for l in range(64)])
# MFMA output: lane l holds D[4 (l // 16) + r, l % 16], r = 0..3
_MF_ROW = 4 * (np.arange(64) // 16)[None, :] + np.arange(4)[:, None]
_MF_COL = np.broadcast_to(np.arange(64) % 16, (4, 64))


_KIND = {}  # opcode -> isa.Ins.kind()


def _bf16_halves(u):
    """(n, 4) uint32 words -> (n, 8) float64: half j = word j // 2, bits 16 (j % 2)"""
    h = np.empty((u.shape[0], 8), dtype=np.uint32)
    h[:, 0::2] = u << 16
    h[:, 1::2] = u & 0xFFFF0000
    return h.view(np.float32).astype(np.float64)
M32 = 0xFFFFFFFF


def f2u(x):
    return np.asarray(x, dtype=np.float32).view(np.uint32)


def u2f(x):
    return np.asarray(x, dtype=np.uint32).view(np.float32)


def bf16_rne(f32):
    """f32 array -> bf16 bit patterns (uint32 holding 16 bits), RNE"""
    u = f2u(f32).astype(np.uint64)
    r = ((u >> 16) & 1) + 0x7FFF
    out = ((u + r) >> 16) & 0xFFFF
    nan = np.isnan(np.asarray(f32, dtype=np.float32))
    out = np.where(nan, 0x7FC0, out)
    return out.astype(np.uint32)


def bf16_to_f32(b):
    return u2f((np.asarray(b, dtype=np.uint32) & 0xFFFF) << 16)


def f16_rne(f32):
    """f32 array -> fp16 bit patterns (uint32 holding 16 bits), RNE"""
    with np.errstate(over="ignore"):
        h = np.asarray(f32, dtype=np.float32).astype(np.float16)
    return h.view(np.uint16).astype(np.uint32)


def f16_to_f32(b):
    return (np.asarray(b, dtype=np.uint32) & 0xFFFF).astype(np.uint16).view(np.float16).astype(np.float32)


class Heap:
    """flat device memory with bounds-checked accesses"""

    BASE = 0x100000000

    def __init__(self):
        self.bufs = []  # (start, np.uint8 array)
        self.next = self.BASE

    def alloc(self, nbytes, data=None):
        start = self.next
        arr = np.zeros(nbytes, dtype=np.uint8)
        if data is not None:
            b = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else \
                np.ascontiguousarray(data).view(np.uint8).ravel()
            arr[:b.size] = b
        self.bufs.append((start, arr))
        self.next = (start + nbytes + 0xFFFF) & ~0xFFFF
        self.next += 0x10000
        return start

    def find(self, addr, n):
        for start, arr in self.bufs:
            if start <= addr and addr + n <= start + arr.size:
                return arr, addr - start
        raise IndexError(f"global access out of bounds: {addr:#x} + {n}")

    def read(self, addr, n):
        arr, off = self.find(addr, n)
        return arr[off:off + n]

    def write(self, addr, data):
        arr, off = self.find(addr, len(data))
        arr[off:off + len(data)] = data

    def lanes(self, addrs, n):
        """the buffer and (lanes, n) byte indices of a vector access whose lanes
        all fall inside one allocation, else None (the caller then goes lane
        by lane, which raises on the out-of-bounds lane)"""
        lo, hi = int(addrs.min()), int(addrs.max())
        for start, arr in self.bufs:
            if start <= lo and hi + n <= start + arr.size:
                return arr, (addrs - start)[:, None] + np.arange(n)[None, :]
        return None

    def view(self, start):
        for s, arr in self.bufs:
            if s == start:
                return arr
        raise KeyError(start)


class Wave:
    def __init__(self):
        self.v = np.zeros((256, LANES), dtype=np.uint32)
        self.a = np.zeros((256, LANES), dtype=np.uint32)
        self.s = np.zeros(128, dtype=np.uint64)  # held as < 2^32
        self.vcc = np.zeros(LANES, dtype=bool)
        self.exec = np.ones(LANES, dtype=bool)
        self.scc = 0
        self.m0 = 0
        self.pc = 0
        self.done = False
        self.count = 0
        self.wid = None  # (workgroup, wave), set by the runner


class Emu:
    def __init__(self, prog, heap, lds_bytes=163840, trace=False, structural=False):
        # structural: scalar and control flow only -- MFMA, VALU, DS and the
        # vector memory traffic are skipped, each LDS-DMA records its wave
        # and scalar source base in dma_log (the stream-order tests)
        self.structural = structural
        self.dma_log = []
        self.prog = [i for i in prog]
        self.labels = {ins.ops[0]: k for k, ins in enumerate(self.prog) if ins.op == "label"}
        self.heap = heap
        self.lds = np.zeros(lds_bytes, dtype=np.uint8)
        self.trace = trace
        self.counts = {}

    # ---- operand access ---------------------------------------------------
    def vec(self, w, o):
        """operand as a per-lane uint32 vector (one register)"""
        if isinstance(o, Neg):
            return f2u(-u2f(self.vec(w, o.r)))
        if isinstance(o, Reg):
            assert o.n == 1, o
            if o.f == "v":
                return w.v[o.i].copy()
            if o.f == "a":
                return w.a[o.i].copy()
            if o.f == "s":
                return np.full(LANES, int(w.s[o.i]) & M32, dtype=np.uint32)
            if o.f == "m0":
                return np.full(LANES, w.m0, dtype=np.uint32)
            raise ValueError(o)
        if isinstance(o, float):
            return np.full(LANES, struct.unpack("<I", struct.pack("<f", o))[0], dtype=np.uint32)
        if isinstance(o, int):
            return np.full(LANES, o & M32, dtype=np.uint32)
        raise ValueError(o)

    def sc(self, w, o):
        """scalar operand"""
        if isinstance(o, Reg):
            if o.f == "s":
                if o.n == 1:
                    return int(w.s[o.i]) & M32
                return (int(w.s[o.i]) & M32) | ((int(w.s[o.i + 1]) & M32) << 32)
            if o.f == "exec":
                return int(np.packbits(w.exec[::-1]).view(">u8")[0]) if False else \
                    sum(1 << k for k in range(LANES) if w.exec[k])
            if o.f == "vcc":
                return sum(1 << k for k in range(LANES) if w.vcc[k])
            if o.f == "m0":
                return w.m0
            raise ValueError(o)
        if isinstance(o, int):
            return o & M32
        raise ValueError(o)

    def sset(self, w, o, val):
        if o.f == "s":
            if o.n == 1:
                w.s[o.i] = val & M32
            else:
                assert o.n == 2
                w.s[o.i] = val & M32
                w.s[o.i + 1] = (val >> 32) & M32
        elif o.f == "m0":
            w.m0 = val & M32
        elif o.f == "exec":
            w.exec = np.array([(val >> k) & 1 for k in range(LANES)], dtype=bool)
        elif o.f == "vcc":
            w.vcc = np.array([(val >> k) & 1 for k in range(LANES)], dtype=bool)
        else:
            raise ValueError(o)

    def vset(self, w, o, val, mask=None):
        m = w.exec if mask is None else mask
        assert o.n == 1
        arr = w.v if o.f == "v" else w.a
        arr[o.i] = np.where(m, np.asarray(val, dtype=np.uint32), arr[o.i])

    def regs(self, w, o):
        arr = w.v if o.f == "v" else w.a
        return arr[o.i:o.i + o.n]

    @staticmethod
    def off(ins):
        for part in ins.mods.split():
            if part.startswith("offset:"):
                return int(part[7:])
        return 0

    # ---- execution ----------------------------------------------------------
    def run_wg(self, waves, max_steps=50_000_000):
        """run a workgroup's waves to completion (barrier-synchronised)"""
        steps = 0
        while not all(w.done for w in waves):
            progressed = False
            for w in waves:
                if w.done:
                    continue
                while not w.done:
                    ins = self.prog[w.pc]
                    if ins.op == "s_barrier":
                        w.pc += 1
                        w.at_barrier = True
                        break
                    self.step(w, ins)
                    steps += 1
                    progressed = True
                    if steps > max_steps:
                        raise RuntimeError("emulator step limit")
                    if w.pc >= len(self.prog):
                        w.done = True
            # barrier release: every live wave waits at it
            live = [w for w in waves if not w.done]
            if live and not all(getattr(w, "at_barrier", False) for w in live):
                if not progressed:
                    raise RuntimeError("barrier deadlock")
            for w in waves:
                w.at_barrier = False
        return steps

    def step(self, w, ins):
        op, o = ins.op, ins.ops
        self.counts[op] = self.counts.get(op, 0) + 1
        w.pc += 1
        if op in ("label", "s_nop", "s_waitcnt"):
            return
        k = _KIND.get(op)
        if k is None:
            k = _KIND[op] = ins.kind()  # (a function of the opcode alone)
        if self.structural and not op.startswith("s_"):
            if op == "global_load_lds_dwordx4":
                self.dma_log.append((w.wid, self.sc(w, o[1]), self.off(ins), w.m0))
            return
        if k == "mfma":
            return self.mfma(w, ins)
        if op.startswith("v_"):
            return self.valu(w, ins)
        if op.startswith("s_"):
            return self.salu(w, ins)
        if op.startswith("ds_"):
            return self.ds(w, ins)
        if op.startswith("global_"):
            return self.vmem(w, ins)
        raise NotImplementedError(op)

    # ---- MFMA -------------------------------------------------------------
    def mfma(self, w, ins):
        d, a, b, c = ins.ops
        f16 = ins.op.endswith("_f16")
        # halves j = 0..7 of lane l: word j // 2, bits 16 (j % 2); A[i, k] with
        # i = l % 16, k = 8 (l // 16) + j (B transposed the same way)
        ua = np.ascontiguousarray(np.asarray(self.regs(w, a), dtype=np.uint32).T)  # (64 lanes, 4 words)
        ub = np.ascontiguousarray(np.asarray(self.regs(w, b), dtype=np.uint32).T)
        if f16:
            fa = ua.view(np.float16).astype(np.float64)  # (64, 8): half j of lane l
            fb = ub.view(np.float16).astype(np.float64)
        else:
            fa = _bf16_halves(ua)
            fb = _bf16_halves(ub)
        # lane l = 16 g + i: A row i, columns 8 g .. 8 g + 7
        A = fa.reshape(4, 16, 8).transpose(1, 0, 2).reshape(16, 32)
        B = fb.reshape(4, 16, 8).transpose(0, 2, 1).reshape(32, 16)
        D = A @ B
        if isinstance(c, int):
            assert c == 0
            C = np.zeros((4, LANES))
        else:
            C = u2f(self.regs(w, c)).astype(np.float64)
        out = C + D[_MF_ROW, _MF_COL]
        self.regs(w, d)[:] = f2u(out.astype(np.float32))

    # ---- VALU -------------------------------------------------------------
    def valu(self, w, ins):
        op, o = ins.op, ins.ops
        g = lambda x: self.vec(w, x)  # noqa: E731
        gf = lambda x: u2f(self.vec(w, x))  # noqa: E731
        # (the softmax stream's ops first: the chain is walked per instruction)
        if op == "v_fma_f32":
            r = (gf(o[1]).astype(np.float64) * gf(o[2]) + gf(o[3])).astype(np.float32)
            return self.vset(w, o[0], f2u(r))
        if op == "v_pk_fma_f32":  # two fp32 fmas on register pairs; op_sel / op_sel_hi pick each source dword
            md = {}
            for part in ins.mods.split():
                if ":" in part:
                    key, val = part.split(":", 1)
                    md[key] = [int(x) for x in val.strip("[]").split(",")]
            sel = (md.get("op_sel", [0, 0, 0]), md.get("op_sel_hi", [1, 1, 1]))
            neg = (md.get("neg_lo", [0, 0, 0]), md.get("neg_hi", [0, 0, 0]))

            def dw(x, k):
                return u2f(self.vec(w, Reg(x.f, x.i + k, 1)))
            res = []
            for h in range(2):
                a, b, c_ = ((-1.0 if neg[h][j] else 1.0) * dw(o[1 + j], sel[h][j]).astype(np.float64) for j in range(3))
                res.append((a * b + c_).astype(np.float32))
            for h in range(2):
                self.vset(w, Reg("v", o[0].i + h, 1), f2u(res[h]))
            return
        if op == "v_exp_f32":
            with np.errstate(over="ignore"):
                r = np.exp2(gf(o[1]))
            if "clamp" in ins.mods.split():  # VOP3 clamp: [0, 1] (NaN -> 0)
                r = np.where(np.isnan(r), np.float32(0), np.clip(r, np.float32(0), np.float32(1)))
            return self.vset(w, o[0], f2u(r.astype(np.float32)))
        if op == "v_cvt_pk_bf16_f32":
            lo, hi = bf16_rne(gf(o[1])), bf16_rne(gf(o[2]))
            return self.vset(w, o[0], lo | (hi << 16))
        if op == "v_mov_b32":
            return self.vset(w, o[0], g(o[1]))
        if op == "v_writelane_b32":  # vdst[lane] = scalar (EXEC ignored)
            w.v[o[0].i][int(o[2])] = self.sc(w, o[1]) & M32
            return
        if op == "v_readlane_b32":  # sdst = vsrc[lane]
            return self.sset(w, o[0], int(w.v[o[1].i][int(o[2])]))
        if op == "v_accvgpr_write_b32":
            return self.vset(w, o[0], g(o[1]))
        if op == "v_accvgpr_read_b32":
            return self.vset(w, o[0], g(o[1]))
        if op == "v_add_u32":
            return self.vset(w, o[0], (g(o[1]).astype(np.uint64) + g(o[2])) & M32)
        if op == "v_sub_u32":
            return self.vset(w, o[0], (g(o[1]).astype(np.int64) - g(o[2])) & M32)
        if op == "v_add3_u32":
            return self.vset(w, o[0], (g(o[1]).astype(np.uint64) + g(o[2]) + g(o[3])) & M32)
        if op == "v_and_b32":
            return self.vset(w, o[0], g(o[1]) & g(o[2]))
        if op == "v_or_b32":
            return self.vset(w, o[0], g(o[1]) | g(o[2]))
        if op == "v_or3_b32":
            return self.vset(w, o[0], g(o[1]) | g(o[2]) | g(o[3]))
        if op == "v_lshlrev_b32":
            return self.vset(w, o[0], (g(o[2]).astype(np.uint64) << (g(o[1]) & 31)) & M32)
        if op == "v_lshrrev_b32":
            return self.vset(w, o[0], g(o[2]) >> (g(o[1]) & 31))
        if op == "v_mul_lo_u32":
            return self.vset(w, o[0], (g(o[1]).astype(np.uint64) * g(o[2])) & M32)
        if op == "v_min_u32":
            return self.vset(w, o[0], np.minimum(g(o[1]), g(o[2])))
        if op == "v_max_u32":
            return self.vset(w, o[0], np.maximum(g(o[1]), g(o[2])))
        if op == "v_subrev_u32":
            return self.vset(w, o[0], (g(o[2]).astype(np.int64) - g(o[1])) & M32)
        if op == "v_mbcnt_lo_u32_b32":
            lane = np.arange(LANES)
            return self.vset(w, o[0], (np.minimum(lane, 32) + g(o[2])).astype(np.uint32))
        if op == "v_mbcnt_hi_u32_b32":
            lane = np.arange(LANES)
            return self.vset(w, o[0], (np.maximum(lane - 32, 0) + g(o[2])).astype(np.uint32))
        if op == "v_mul_f32":
            return self.vset(w, o[0], f2u(gf(o[1]) * gf(o[2])))
        if op == "v_add_f32":
            return self.vset(w, o[0], f2u(gf(o[1]) + gf(o[2])))
        if op == "v_sub_f32":
            return self.vset(w, o[0], f2u(gf(o[1]) - gf(o[2])))
        if op == "v_max_f32":
            return self.vset(w, o[0], f2u(np.maximum(gf(o[1]), gf(o[2]))))
        if op == "v_max3_f32":
            return self.vset(w, o[0], f2u(np.maximum(np.maximum(gf(o[1]), gf(o[2])), gf(o[3]))))
        if op == "v_rcp_f32":
            with np.errstate(divide="ignore"):
                return self.vset(w, o[0], f2u(np.float32(1.0) / gf(o[1])))
        if op == "v_cvt_f32_f16":  # the low half
            return self.vset(w, o[0], f2u(f16_to_f32(g(o[1]) & 0xFFFF).astype(np.float32)))
        if op == "v_cvt_pk_f16_f32":
            lo, hi = f16_rne(gf(o[1])), f16_rne(gf(o[2]))
            return self.vset(w, o[0], lo | (hi << 16))
        if op in ("v_cmp_lt_f32_e32", "v_cmp_le_f32_e32"):
            a, b = gf(o[1]), gf(o[2])
            w.vcc = np.where(w.exec, a < b if op == "v_cmp_lt_f32_e32" else a <= b, False)
            return
        if op in ("v_cmp_ne_u32_e32", "v_cmp_gt_u32_e32", "v_cmp_gt_i32_e32", "v_cmp_lt_i32_e32",
                  "v_cmp_le_u32_e32"):
            a, b = g(o[1]), g(o[2])
            if op.endswith("i32_e32"):
                a, b = a.view(np.int32), b.view(np.int32)
            r = {"v_cmp_ne_u32_e32": a != b, "v_cmp_gt_u32_e32": a > b, "v_cmp_gt_i32_e32": a > b,
                 "v_cmp_lt_i32_e32": a < b, "v_cmp_le_u32_e32": a <= b}[op]
            w.vcc = np.where(w.exec, r, False)
            return
        if op == "v_cndmask_b32_e32":
            return self.vset(w, o[0], np.where(w.vcc, g(o[2]), g(o[1])))
        if op == "v_permlane16_swap_b32":
            A_, B_ = o[0], o[1]
            va, vb = g(A_), g(B_)
            na, nb = va.copy(), vb.copy()
            for row in (1, 3):
                sa = slice(16 * row, 16 * row + 16)
                sb = slice(16 * (row - 1), 16 * row)
                na[sa], nb[sb] = vb[sb], va[sa]
            full = np.ones(LANES, dtype=bool)
            self.vset(w, A_, na, full)
            self.vset(w, B_, nb, full)
            return
        if op == "v_mov_b32_dpp":
            kv = dict(m.split(":") for m in ins.mods.split())
            assert set(kv) <= {"row_ror", "row_mask", "bank_mask", "bound_ctrl"}, ins.mods
            n = int(kv["row_ror"], 0)
            assert int(kv.get("row_mask", "0xf"), 0) == 0xF
            bank = int(kv.get("bank_mask", "0xf"), 0)
            lane = np.arange(LANES)
            src = g(o[1])[(lane & ~15) | ((lane - n) & 15)]
            mask = w.exec & (((bank >> ((lane & 15) >> 2)) & 1) == 1)
            return self.vset(w, o[0], src, mask)
        if op == "v_permlane32_swap_b32":
            A_, B_ = o[0], o[1]
            va, vb = g(A_), g(B_)
            na, nb = va.copy(), vb.copy()
            na[32:], nb[:32] = vb[:32], va[32:]
            full = np.ones(LANES, dtype=bool)
            self.vset(w, A_, na, full)
            self.vset(w, B_, nb, full)
            return
        raise NotImplementedError(op)

    # ---- SALU ---------------------------------------------------------------
    def salu(self, w, ins):
        op, o = ins.op, ins.ops
        g = lambda x: self.sc(w, x)  # noqa: E731
        if op in ("s_mov_b32", "s_mov_b64"):
            return self.sset(w, o[0], g(o[1]))
        if op == "s_add_u32":
            r = g(o[1]) + g(o[2])
            w.scc = int(r > M32)
            return self.sset(w, o[0], r & M32)
        if op == "s_addc_u32":
            r = g(o[1]) + g(o[2]) + w.scc
            w.scc = int(r > M32)
            return self.sset(w, o[0], r & M32)
        if op == "s_sub_u32":
            r = g(o[1]) - g(o[2])
            w.scc = int(r < 0)
            return self.sset(w, o[0], r & M32)
        if op == "s_subb_u32":
            r = g(o[1]) - g(o[2]) - w.scc
            w.scc = int(r < 0)
            return self.sset(w, o[0], r & M32)
        if op == "s_bitcmp1_b32":
            w.scc = (g(o[0]) >> (g(o[1]) & 31)) & 1
            return
        if op == "s_mul_i32":
            a, b = g(o[1]), g(o[2])
            a = a - (1 << 32) if a >= 1 << 31 else a
            b = b - (1 << 32) if b >= 1 << 31 else b
            return self.sset(w, o[0], (a * b) & M32)
        if op == "s_mul_hi_u32":
            return self.sset(w, o[0], ((g(o[1]) * g(o[2])) >> 32) & M32)
        if op == "s_lshl_b32":
            r = (g(o[1]) << (g(o[2]) & 31)) & M32
            w.scc = int(r != 0)
            return self.sset(w, o[0], r)
        if op == "s_lshr_b32":
            r = g(o[1]) >> (g(o[2]) & 31)
            w.scc = int(r != 0)
            return self.sset(w, o[0], r)
        if op == "s_ashr_i32":
            a = g(o[1])
            a = a - (1 << 32) if a >= 1 << 31 else a
            r = (a >> (g(o[2]) & 31)) & M32
            w.scc = int(r != 0)
            return self.sset(w, o[0], r)
        if op == "s_and_b32":
            r = g(o[1]) & g(o[2])
            w.scc = int(r != 0)
            return self.sset(w, o[0], r)
        if op == "s_or_b32":
            r = g(o[1]) | g(o[2])
            w.scc = int(r != 0)
            return self.sset(w, o[0], r)
        if op == "s_min_u32":
            a, b = g(o[1]), g(o[2])
            w.scc = int(a < b)
            return self.sset(w, o[0], min(a, b))
        if op == "s_cmp_eq_u32":
            w.scc = int(g(o[0]) == g(o[1]))
            return
        if op == "s_cmp_lt_u32":
            w.scc = int(g(o[0]) < g(o[1]))
            return
        if op == "s_cmp_ge_u32":
            w.scc = int(g(o[0]) >= g(o[1]))
            return
        if op == "s_cmp_gt_u32":
            w.scc = int(g(o[0]) > g(o[1]))
            return
        if op == "s_cmp_le_u32":
            w.scc = int(g(o[0]) <= g(o[1]))
            return
        if op == "s_cmp_gt_i32":
            a, b = g(o[0]), g(o[1])
            a = a - (1 << 32) if a >= 1 << 31 else a
            b = b - (1 << 32) if b >= 1 << 31 else b
            w.scc = int(a > b)
            return
        if op in ("s_cselect_b32", "s_cselect_b64"):
            return self.sset(w, o[0], g(o[1]) if w.scc else g(o[2]))
        if op == "s_and_saveexec_b64":
            old = g(Reg("exec"))
            self.sset(w, o[0], old)
            new = old & g(o[1])
            w.scc = int(new != 0)
            self.sset(w, Reg("exec"), new)
            return
        if op == "s_branch":
            w.pc = self.labels[o[0]]
            return
        if op in ("s_cbranch_scc0", "s_cbranch_scc1", "s_cbranch_vccnz", "s_cbranch_vccz"):
            take = {"s_cbranch_scc0": not w.scc, "s_cbranch_scc1": bool(w.scc),
                    "s_cbranch_vccnz": bool((w.vcc & w.exec).any()),
                    "s_cbranch_vccz": not bool((w.vcc & w.exec).any())}[op]
            if take:
                w.pc = self.labels[o[0]]
            return
        if op == "s_endpgm":
            w.pc = len(self.prog)
            return
        if op.startswith("s_load_dword"):
            n = {"s_load_dword": 1, "s_load_dwordx2": 2, "s_load_dwordx4": 4, "s_load_dwordx8": 8,
                 "s_load_dwordx16": 16}[op]
            base = g(o[1])
            data = self.heap.read(base + int(o[2]), 4 * n).view(np.uint32)
            for k in range(n):
                w.s[o[0].i + k] = int(data[k])
            return
        raise NotImplementedError(op)

    # ---- LDS ------------------------------------------------------------------
    def lds_read(self, addr, n):
        assert 0 <= addr and addr + n <= self.lds.size, f"LDS read out of bounds {addr}+{n}"
        return self.lds[addr:addr + n]

    def ds(self, w, ins):
        op, o = ins.op, ins.ops
        off = self.off(ins)
        addr = self.vec(w, o[1]).astype(np.int64) + off
        if op == "ds_read_b128":
            dst = self.regs(w, o[0])
            act = np.nonzero(w.exec)[0]
            a = addr[act]
            assert act.size == 0 or (a.min() >= 0 and a.max() + 16 <= self.lds.size), "LDS read out of bounds"
            data = self.lds[a[:, None] + np.arange(16)[None, :]]  # (lanes, 16 bytes), gathered
            dst[:, act] = np.ascontiguousarray(data).view(np.uint32).T
            return
        if op == "ds_read_b64_tr_b16":
            assert w.exec.all()
            dst = self.regs(w, o[0])
            # lane l = 16 grp + i takes the 16-bit word at byte 2 (i & 3) of lane
            # 16 grp + 4 q + (i >> 2)'s address, for q = 0..3 (vectorised)
            a = addr[_TR_SRC] + _TR_OFF[:, None]  # (64, 4) byte addresses
            assert a.min() >= 0 and a.max() + 2 <= self.lds.size, "LDS read out of bounds"
            if (a & 1).any():
                vals = self.lds[a].astype(np.uint32) | (self.lds[a + 1].astype(np.uint32) << 8)
            else:
                vals = self.lds.view(np.uint16)[a >> 1].astype(np.uint32)
            dst[0, :] = vals[:, 0] | (vals[:, 1] << 16)
            dst[1, :] = vals[:, 2] | (vals[:, 3] << 16)
            return
        raise NotImplementedError(op)

    # ---- global -----------------------------------------------------------------
    def vmem(self, w, ins):
        op, o = ins.op, ins.ops
        off = self.off(ins)
        if op == "global_load_lds_dwordx4":
            assert w.exec.all()
            voff = self.vec(w, o[0])
            base = self.sc(w, o[1])
            la = w.m0 + off
            assert 0 <= la and la + 16 * LANES <= self.lds.size, f"LDS-DMA out of bounds {la}"
            g = self.heap.lanes(base + voff.astype(np.int64) + off, 16)
            if g is not None:
                self.lds[la:la + 16 * LANES] = g[0][g[1]].ravel()
                return
            for l in range(LANES):
                self.lds[la + 16 * l:la + 16 * l + 16] = self.heap.read(base + int(voff[l]) + off, 16)
            return
        if op == "global_load_dwordx4":
            dst = self.regs(w, o[0])
            voff = self.vec(w, o[1])
            base = self.sc(w, o[2])
            act = np.nonzero(w.exec)[0]
            if act.size == 0:
                return
            g = self.heap.lanes(base + voff[act].astype(np.int64) + off, 16)
            if g is not None:
                dst[:, act] = np.ascontiguousarray(g[0][g[1]]).view(np.uint32).T
                return
            for l in act:
                dst[:, l] = self.heap.read(base + int(voff[l]) + off, 16).view(np.uint32)
            return
        if op == "global_store_dwordx4":
            voff = self.vec(w, o[0])
            src = self.regs(w, o[1])
            base = self.sc(w, o[2])
            act = np.nonzero(w.exec)[0]
            if act.size == 0:
                return
            g = self.heap.lanes(base + voff[act].astype(np.int64) + off, 16)
            if g is not None:
                g[0][g[1]] = np.ascontiguousarray(np.asarray(src, dtype=np.uint32)[:, act].T).view(np.uint8)
                return
            for l in act:
                self.heap.write(base + int(voff[l]) + off, src[:, l].copy().view(np.uint8))
            return
        raise NotImplementedError(op)
