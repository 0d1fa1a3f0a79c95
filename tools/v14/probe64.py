"""Timing probe for head dim 64 at two waves per SIMD, 64 query rows per
wave (round-6 verdict item 2b; timing only, results meaningless;
tools/v14/run_probe64.py drives it on the GPU box).

attn_fwd_v13's D = 64 form runs one wave per SIMD and is bound by its
softmax stream (64 fma + 64 exp + 32 cvt per 64 x 64 wave-tile against 72
MFMAs; MFMA busy ~0.52).  The question before writing a new program: with 8
waves of 64 rows each -- waves w and w + 4 sharing a SIMD, 256 registers each
(128 V + 128 A), one in its matrix phase (PV(t-1) with its row sums, QK(t):
72 v_mfma_f32_16x16x32_bf16 with 16 fragment reads) while its partner runs
its vector phase (the softmax of its 64 x 64 tile, the row-sum check, its 2
LDS-DMA pieces), barrier-separated -- how many cycles does one period (both
phases, i.e. two wave-tiles per SIMD) take, and at what clock?  Unlike the
D = 128 ping-pong probe (tools/v14/probe.py, 32 rows per wave), 64 rows per
wave keep one fragment read per 4 MFMAs, as in v13.

Register plan (the probe is also the budget check): a0-63 O (4 d-blocks x 4
q-blocks), a64-95 Q, a96-127 an 8-slot fragment ring; v0-63 S (softmax in
place), v64-95 P, v96-111 l, v112-115 ones, v116-119 mu, v120-127 addresses
and temporaries.

Variants (Probe64(...)): stagger (False: both waves of a SIMD in the same
phase -- the plain 8-wave control), soft (no softmax stream), reads (no
fragment reads), dma (no LDS-DMA), noexp (v_exp -> v_mov).
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from v13.isa import A, EXEC, Ins, M0, Neg, S, V, VCC, finalize, label  # noqa: E402

MFMA = "v_mfma_f32_16x16x32_bf16"


def I(op, *ops, mods=""):
    return Ins(op, *ops, mods=mods)


def O_(db, qb):
    return A(4 * (4 * db + qb), 4)       # a0..a63


def Q_(qb, ds):
    return A(64 + 4 * (2 * qb + ds), 4)  # a64..a95


NF = 8


def F(slot):
    return A(96 + 4 * slot, 4)           # a96..a127


def S_(kb, qb):
    return V(4 * (4 * qb + kb), 4)       # v0..v63


def P_(qb, kp):
    return V(64 + 4 * (2 * qb + kp), 4)  # v64..v95


def L_(qb):
    return V(96 + 4 * qb, 4)             # v96..v111


ONES = V(112, 4)


def MU(qb):
    return V(116 + qb)


VKL, VVL, VKA, VVA, DMAK, DMAV, T0, T1 = (V(120 + k) for k in range(8))

sKA = S(16, 2)
sWG, sWAVE = S(18), S(19)
sBUF, sOUT = S(20, 2), S(22, 2)
sNIT, sC, sMU = S(24), S(25), S(26)
sGRP, sWOFF, sHEAD, sIT = S(28), S(29), S(30), S(31)
sDK = S(48, 2)
sTI = S(34)
sSM1, sS0, sS1, sS2, sS3 = S(35), S(36), S(37), S(38), S(39)
sT0, sT1, sT2, sT3 = S(40), S(41), S(42), S(43)
sTM0 = S(44, 2)
sTM1 = S(46, 2)
sWC, sWM = S(50), S(51)
sBA, sBB = S(52, 2), S(54, 2)
SLOT = 32768
NSLOT = 5
VIMG = 16384


class Probe64:
    def __init__(self, stagger=True, soft=True, reads=True, dma=True, noexp=False, stamps=True, order="pair",
                 dma_in="M", split=0, tag="%="):
        self.stagger, self.soft, self.reads, self.dma, self.noexp, self.stamps = stagger, soft, reads, dma, noexp, stamps
        self.order, self.dma_in, self.split = order, dma_in, split
        self.tag = tag
        self.prog = []

    def L(self, n):
        return f"p64_{n}_{self.tag}"

    def e(self, c):
        self.prog.extend(c)

    def dma_piece(self, j, slot_reg):
        """this wave's K (j = 0) or V (j = 1) piece (1 KiB) of the tile at sDK"""
        c = [I("s_add_u32", M0, slot_reg, sWOFF)]
        if j == 1:
            c += [I("s_add_u32", M0, M0, VIMG)]
        c += [I("global_load_lds_dwordx4", DMAK if j == 0 else DMAV, sDK)]
        return c

    def dma_advance(self):
        return [I("s_add_u32", sTI, sTI, 1), I("s_and_b32", sTI, sTI, 63),
                I("s_lshl_b32", sT0, sTI, 15), I("s_lshl_b32", sT1, sHEAD, 21), I("s_add_u32", sT0, sT0, sT1),
                I("s_add_u32", sDK[0], sBUF[0], sT0), I("s_addc_u32", sDK[1], sBUF[1], 0)]

    def frag_read(self, n):
        """fragment n of the matrix phase (0-7: V(t-1) (db, kp); 8-15: K(t) (kb, ds)) into ring slot n % 8"""
        f = F(n % NF)
        if n < 8:
            db, kp = n // 2, n % 2
            return [I("ds_read_b64_tr_b16", f.sub(2 * h, 2), VVA,
                      mods=f"offset:{256 * (db & 1) + 512 * ((db >> 1) & 1) + 2048 * h + 4096 * kp}")
                    for h in range(2)]
        m = n - 8
        kb, ds = m // 2, m % 2
        return [I("ds_read_b128", f, VKA, mods=f"offset:{512 * ds + 2048 * kb}")]

    def mfmas(self):
        """(instruction, fragment index): PV(t-1) with the row sums, then QK(t)"""
        out = []
        for db in range(4):
            for kp in range(2):
                n = 2 * db + kp
                for qb in range(4):
                    out.append((I(MFMA, O_(db, qb), F(n % NF), P_(qb, kp), O_(db, qb)), n))
                out.append((I(MFMA, L_(db), ONES, P_(db, kp), L_(db)), None))  # row sums of q-block db
        for kb in range(4):
            for ds in range(2):
                n = 8 + 2 * kb + ds
                for qb in range(4):
                    out.append((I(MFMA, S_(kb, qb), F(n % NF), Q_(qb, ds), S_(kb, qb) if ds else 0), n))
        return out

    def c_phase(self):
        c = []
        ms = self.mfmas()
        last = {}
        for k, (_, n) in enumerate(ms):
            if n is not None:
                last[n] = k
        after = {}
        for n in range(NF, 16):
            after.setdefault(last[n - NF], []).append(n)
        dma_at = {20: 0, 52: 1} if self.dma and self.dma_in == "C" else {}
        cs = self.c_softmax() if self.soft and self.split else []
        start = 50       # QK(t) of key block 0 is issued by MFMA 47
        per = -(-len(cs) // (len(ms) - start)) if cs else 0
        for k, (ins, n) in enumerate(ms):
            c.append(ins)
            if cs and k >= start:
                c += cs[:per]
                cs = cs[per:]
            if self.reads:
                for m in after.get(k, []):
                    c += self.frag_read(m)
            if k in dma_at:
                c += self.dma_piece(dma_at[k], sS3)
        c += cs
        if dma_at:
            c += self.dma_advance()
        return c

    def softmax(self):
        """32 slices (q-block, key block, half) in four groups of 8: fma x2, exp x2
        in place on S, then cvt into P (with split: the slices the matrix phase does not take)"""
        sl = self.slices()[self.split:]
        gs = len(sl) // 4
        groups = []
        for g in range(4):
            vs, ex, cv = [], [], []
            for (qb, kb, hh) in sl[gs * g:gs * g + gs]:
                s = S_(kb, qb)
                y0, y1 = s[2 * hh], s[2 * hh + 1]
                vs += [I("v_fma_f32", y0, y0, sC, Neg(MU(qb))), I("v_fma_f32", y1, y1, sC, Neg(MU(qb)))]
                xo = "v_mov_b32" if self.noexp else "v_exp_f32"
                ex += [I(xo, y0, y0, mods="" if self.noexp else "clamp"), I(xo, y1, y1, mods="" if self.noexp else "clamp")]
                cv.append(I("v_cvt_pk_bf16_f32", P_(qb, kb >> 1)[2 * (kb & 1) + hh], y0, y1))
            if self.order == "wide":       # all fmas of the group, then its exps, then its cvts
                groups.append(vs + ex + cv)
                continue
            if self.order == "skew":       # a slice's exps four fmas after its fmas, cvts two slices later
                out = []
                for n in range(10):
                    if n < 8:
                        out += vs[2 * n:2 * n + 2]
                    if 2 <= n < 10:
                        out += ex[2 * (n - 2):2 * (n - 1)]
                    if 4 <= n:
                        out.append(cv[n - 4])
                out += cv[6:8]
                groups.append(out)
                continue
            # interleave: each slice's exps two fmas after its fmas
            groups.append(self.pair_order(vs, ex, cv))
        return groups

    @staticmethod
    def pair_order(vs, ex, cv):
        n_sl = len(cv)
        out = []
        for n in range(n_sl):
            out += vs[2 * n:2 * n + 2]
            if n >= 1:
                out += ex[2 * (n - 1):2 * n]
            if n >= 2:
                out.append(cv[n - 2])
        out += ex[2 * n_sl - 2:] + cv[max(0, n_sl - 2):]
        return out

    def slices(self):
        if self.split:   # key-block major, so the matrix phase's share is ready early in QK
            return [(qb, kb, hh) for kb in range(4) for qb in range(4) for hh in range(2)]
        return [(qb, kb, hh) for qb in range(4) for kb in range(4) for hh in range(2)]

    def c_softmax(self):
        """the first `split` slices, for the matrix phase (same instructions as the vector phase's)"""
        vs, ex, cv = [], [], []
        for (qb, kb, hh) in self.slices()[:self.split]:
            s_ = S_(kb, qb)
            y0, y1 = s_[2 * hh], s_[2 * hh + 1]
            vs += [I("v_fma_f32", y0, y0, sC, Neg(MU(qb))), I("v_fma_f32", y1, y1, sC, Neg(MU(qb)))]
            ex += [I("v_exp_f32", y0, y0, mods="clamp"), I("v_exp_f32", y1, y1, mods="clamp")]
            cv.append(I("v_cvt_pk_bf16_f32", P_(qb, kb >> 1)[2 * (kb & 1) + hh], y0, y1))
        return self.pair_order(vs, ex, cv)

    def m_phase(self, grp):
        c = [I("s_mov_b32", sSM1, sS0), I("s_mov_b32", sS0, sS1), I("s_mov_b32", sS1, sS2), I("s_mov_b32", sS2, sS3),
             I("s_add_u32", sS3, sS3, SLOT), I("s_cmp_ge_u32", sS3, SLOT * NSLOT), I("s_cselect_b32", sS3, 0, sS3)]
        side = [self.dma_piece(j, sS2) for j in range(2)] if self.dma and self.dma_in == "M" else []
        pre = [self.frag_read(n) for n in range(NF)] if self.reads else []
        groups = self.softmax() if self.soft else [[], [], [], []]
        c += [I("v_add_u32", VVA, sSM1, VVL), I("v_add_u32", VKA, sS0, VKL)]
        for g in range(4):
            vs = groups[g]
            if side and g < 2:
                c += side[g]
            rd = pre[4 * (g - 2):4 * (g - 2) + 4] if g >= 2 and pre else []
            step = max(1, len(vs) // (len(rd) + 1)) if rd else 0
            k = 0
            for i, ins in enumerate(vs):
                c.append(ins)
                if rd and k < len(rd) and (i + 1) % step == 0:
                    c += rd[k]
                    k += 1
            while rd and k < len(rd):
                c += rd[k]
                k += 1
        if side:
            c += self.dma_advance()
        # the row-sum check (never taken here)
        c += [I("v_max3_f32", T0, L_(0)[0], L_(1)[0], L_(2)[0]), I("v_max_f32", T0, T0, L_(3)[0]),
              I("v_cmp_le_f32_e32", VCC, 1.0, T0), I("s_cbranch_vccnz", self.L(f"rare{grp}")),
              label(self.L(f"ret{grp}"))]
        return c

    def bar(self, acc):
        if not self.stamps:
            return [I("s_barrier")]
        return [I("s_memtime", sBA), I("s_barrier"), I("s_memtime", sBB), I("s_waitcnt", "lgkmcnt(0)"),
                I("s_sub_u32", sT3, sBB[0], sBA[0]), I("s_add_u32", acc, acc, sT3)]

    def build(self, in_kernarg="%0", in_wg="%1", in_wave="%2"):
        e = self.e
        e([I("s_mov_b64", sKA, in_kernarg), I("s_mov_b32", sWG, in_wg), I("s_mov_b32", sWAVE, in_wave),
           I("s_load_dwordx8", S(20, 8), sKA, 0), I("s_waitcnt", "lgkmcnt(0)")])
        e([I("s_lshr_b32", sGRP, sWAVE, 2), I("s_lshl_b32", sWOFF, sWAVE, 10)])
        e([I("s_and_b32", sT0, sWG, 7), I("s_lshl_b32", sT0, sT0, 1), I("s_lshr_b32", sT1, sWG, 7),
           I("s_and_b32", sT1, sT1, 1), I("s_add_u32", sHEAD, sT0, sT1), I("s_mov_b32", sTI, 0),
           I("s_lshl_b32", sT1, sHEAD, 21), I("s_add_u32", sDK[0], sBUF[0], sT1), I("s_addc_u32", sDK[1], sBUF[1], 0)])
        lane, vi, vg, t = V(0), V(1), V(2), [V(3 + k) for k in range(4)]  # (S's registers, before the loop)
        e([I("v_mbcnt_lo_u32_b32", lane, -1, 0), I("v_mbcnt_hi_u32_b32", lane, -1, lane),
           I("v_and_b32", vi, 15, lane), I("v_lshrrev_b32", vg, 4, lane)])
        e([I("v_and_b32", t[0], 1, vg), I("v_lshlrev_b32", t[0], 4, t[0]),
           I("v_and_b32", t[1], 7, vi), I("v_lshlrev_b32", t[1], 5, t[1]), I("v_add_u32", t[0], t[0], t[1]),
           I("v_lshrrev_b32", t[1], 1, vg), I("v_lshlrev_b32", t[1], 8, t[1]), I("v_add_u32", t[0], t[0], t[1]),
           I("v_lshrrev_b32", t[1], 3, vi), I("v_lshlrev_b32", t[1], 10, t[1]), I("v_add_u32", VKL, t[0], t[1])])
        e([I("v_lshlrev_b32", t[0], 3, vi), I("v_and_b32", t[1], 1, vg), I("v_lshlrev_b32", t[1], 7, t[1]),
           I("v_add_u32", t[0], t[0], t[1]), I("v_lshrrev_b32", t[1], 1, vg), I("v_lshlrev_b32", t[1], 10, t[1]),
           I("v_add_u32", t[0], t[0], t[1]), I("v_add_u32", VVL, VIMG, t[0])])
        e([I("v_lshlrev_b32", t[0], 4, lane), I("v_add_u32", DMAK, sWOFF, t[0]), I("v_add_u32", DMAV, VIMG, DMAK)])
        e([I("v_lshlrev_b32", t[2], 6, lane)])
        for qb in range(4):
            for ds in range(2):
                e([I("global_load_dwordx4", Q_(qb, ds), t[2], sBUF, mods=f"offset:{64 * (2 * qb + ds)}")])
        e([I("v_accvgpr_write_b32", A(k), 0) for k in range(64)])
        e([I("v_mov_b32", L_(qb)[r], 0) for qb in range(4) for r in range(4)])
        e([I("v_mov_b32", ONES[k], 0x3F803F80) for k in range(4)])
        e([I("v_mov_b32", MU(qb), sMU) for qb in range(4)])
        e([I("v_mov_b32", P_(qb, kp)[r], 0x3C003C00) for qb in range(4) for kp in range(2) for r in range(4)])
        e([I("s_mov_b32", sSM1, 4 * SLOT), I("s_mov_b32", sS0, 0), I("s_mov_b32", sS1, SLOT),
           I("s_mov_b32", sS2, 2 * SLOT), I("s_mov_b32", sS3, 3 * SLOT)])
        for slot in range(3):
            e([I("s_mov_b32", sT2, slot * SLOT)])
            for j in range(2):
                e(self.dma_piece(j, sT2))
            e(self.dma_advance())
        e([I("s_waitcnt", "vmcnt(0)"), I("s_barrier")])
        e([I("v_add_u32", VVA, sSM1, VVL), I("v_add_u32", VKA, sS0, VKL)])
        if self.reads:
            for n in range(NF):
                e(self.frag_read(n))
        e([I("s_memtime", sTM0), I("s_waitcnt", "lgkmcnt(0)")])
        if self.stagger:
            skip = self.L("nostag")
            e([I("s_cmp_eq_u32", sGRP, 0), I("s_cbranch_scc1", skip), I("s_barrier"), label(skip)])
        e([I("s_mov_b32", sWC, 0), I("s_mov_b32", sWM, 0)])
        e([I("s_mov_b32", sIT, 0), I("s_cmp_eq_u32", sGRP, 1), I("s_cbranch_scc1", self.L("loopB"))])
        for grp, wait in ((0, 4), (1, 2)):
            lp = self.L("loopA" if grp == 0 else "loopB")
            e([label(lp)])
            e(self.c_phase())
            e(self.bar(sWC))
            e(self.m_phase(grp))
            e([I("s_waitcnt", f"vmcnt({wait if self.stagger else 2})")])
            e(self.bar(sWM))
            e([I("s_add_u32", sIT, sIT, 1), I("s_cmp_lt_u32", sIT, sNIT), I("s_cbranch_scc1", lp)])
            if grp == 0:
                if self.stagger:
                    e([I("s_barrier")])
                e([I("s_branch", self.L("done"))])
        e([label(self.L("done"))])
        e([I("s_memtime", sTM1), I("s_waitcnt", "vmcnt(0) lgkmcnt(0)")])
        e([I("s_sub_u32", sT0, sTM1[0], sTM0[0]), I("v_mov_b32", T1, sT0),
           I("s_lshl_b32", sT1, sWG, 3), I("s_add_u32", sT1, sT1, sWAVE), I("s_lshl_b32", sT1, sT1, 2),
           I("v_mov_b32", T0, sT1),
           I("v_accvgpr_read_b32", V(4), O_(0, 0)[0]), I("v_add_u32", V(4), V(4), L_(0)[0]),
           I("v_add_u32", V(4), V(4), S_(0, 0)[0]),
           I("s_mov_b64", EXEC, 1), I("global_store_dword", T0, T1, sOUT),
           I("v_add_u32", V(5), 8192, T0), I("global_store_dword", V(5), V(4), sOUT),
           I("v_mov_b32", V(6), sWC), I("v_add_u32", V(7), 16384, T0), I("global_store_dword", V(7), V(6), sOUT),
           I("v_mov_b32", V(8), sWM), I("v_add_u32", V(9), 24576, T0), I("global_store_dword", V(9), V(8), sOUT),
           I("s_mov_b64", EXEC, -1), I("s_waitcnt", "vmcnt(0)"), I("s_branch", self.L("exit"))])
        e([label(self.L("rare0")), I("s_branch", self.L("ret0"))])
        e([label(self.L("rare1")), I("s_branch", self.L("ret1"))])
        e([label(self.L("exit"))])
        return self.prog


VARIANTS = {
    "pp64": dict(),
    "pp64_nostamp": dict(stamps=False),
    "lockstep64": dict(stagger=False),
    "pp64_nosoft": dict(soft=False),
    "pp64_noexp": dict(noexp=True),
    "pp64_nodma": dict(dma=False),
    "mfma_only64": dict(dma=False, soft=False, reads=False),
    "pp64_wide": dict(stamps=False, order="wide"),
    "pp64_skew": dict(stamps=False, order="skew"),
    "pp64_dmaC": dict(stamps=False, dma_in="C"),
    "pp64_wide_dmaC": dict(stamps=False, order="wide", dma_in="C"),
    "pp64_split4": dict(split=4),
    "pp64_split8": dict(split=8),
    "pp64_split12": dict(split=12),
    "pp64_split16": dict(split=16),
    "pp64_split8_dmaC": dict(split=8, dma_in="C"),
}


def render():
    lines = ["// GENERATED by tools/v14/probe64.py -- timing probe, results meaningless", "#pragma once", ""]
    for name, kw in VARIANTS.items():
        prog, st = finalize(Probe64(**kw).build())
        lines.append(f"// {name}: {len(prog)} instructions, nops {st['nop_ws']}, waits {st['waits']}")
        lines.append(f"#define PP64_BODY_{name} \\")
        for ins in prog:
            t = ins.text()
            lines.append(f'    "{t}\\n" \\' if ins.op == "label" else f'    "\\t{t}\\n" \\')
        lines.append('    ""')
        lines.append("")
    clob = [f'"v{i}"' for i in range(128)] + [f'"a{i}"' for i in range(128)] + \
           [f'"s{i}"' for i in range(16, 56) if i != 32] + ['"vcc"', '"scc"', '"m0"', '"memory"']
    lines.append("#define PP64_CLOBBERS \\")
    for k in range(0, len(clob), 16):
        sep = ", \\" if k + 16 < len(clob) else ""
        lines.append("    " + ", ".join(clob[k:k + 16]) + sep)
    lines.append("")
    lines.append("#define PP64_VARIANTS(X) " + " ".join(f"X({n})" for n in VARIANTS))
    lines.append("")
    return "\n".join(lines)


if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "probe64_asm.h")
    with open(out, "w") as f:
        f.write(render())
    print(out)
