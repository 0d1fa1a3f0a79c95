"""Timing probe for a two-waves-per-SIMD ("ping-pong") flash-attention step
(timing only, results meaningless; tools/v14/run_probe.py drives it on the
GPU box).

The question it answers before the real kernel is written: with 8 waves of
32 query rows each, waves w and w + 4 sharing a SIMD, one wave of each pair in
a matrix phase (PV(t-1) + QK(t): 68 v_mfma_f32_16x16x32_bf16 with the K / V
fragment reads from LDS) while its partner is in a vector phase (the softmax
stream of its 32 x 64 tile: 32 v_fma_f32, 32 v_exp_f32, 16 v_cvt_pk_bf16_f32,
8 v_or3_b32, the defer-max check, 4 LDS-DMA pieces of a tile three ahead),
separated by s_barrier -- how many cycles does one period (both phases =
64 rows x 64 keys per SIMD) take?  attn_fwd_v13 (one wave per SIMD, the same
work per SIMD in one stream) takes 2872; the MFMA floor is 2176.

Variants (Probe(...) keywords): stagger (False: both waves of a SIMD run the
same phase at the same time -- the plain 8-wave control), dma ("M" vector
phase, "C" matrix phase, "none"), prio ("none", "flip": s_setprio 1 for the
matrix phase, "B": waves 4-7 at priority 1 throughout), soft (False: no
softmax stream), reads (False: no fragment reads).
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from v13.isa import A, EXEC, Ins, M0, Neg, S, V, VCC, finalize, label  # noqa: E402

MFMA = "v_mfma_f32_16x16x32_bf16"


def I(op, *ops, mods=""):
    return Ins(op, *ops, mods=mods)


# ---- registers (the planned attn_fwd_v14 layout) ---------------------------
def O_(db, qb):
    return A(4 * (2 * db + qb), 4)       # a0..a63


def Q_(qb, ds):
    return A(64 + 4 * (4 * qb + ds), 4)  # a64..a95


NF = 8


def F(slot):
    return A(96 + 4 * slot, 4)           # a96..a127: fragment ring


def S_(kb, qb):
    return V(4 * (2 * kb + qb), 4)       # v0..v31


def P_(qb, kp):
    return V(32 + 4 * (2 * qb + kp), 4)  # v32..v47


def L_(qb):
    return V(48 + 4 * qb, 4)


ONES = V(56, 4)


def MU(qb):
    return V(60 + qb)


ACC = V(62)
VKL, VVL, VKA, VVA = V(63), V(64), V(65), V(66)


def DMAK(j):
    return V(67 + j)


def DMAV(j):
    return V(69 + j)


def Y(k):
    return V(72 + k)


LANE, VI, VG = V(80), V(81), V(82)


def T(k):
    return V(84 + k)


# SGPRs
sKA = S(16, 2)
sWG, sWAVE = S(18), S(19)
sBUF, sOUT = S(20, 2), S(22, 2)
sNIT, sC, sMU = S(24), S(25), S(26)
sGRP, sWOFF, sHEAD, sIT = S(28), S(29), S(30), S(31)
sDK = S(48, 2)  # (s32 is hipcc's stack pointer: never used)
sTI = S(34)
sSM1, sS0, sS1, sS2, sS3 = S(35), S(36), S(37), S(38), S(39)  # slots of t-1, t, t+1, t+2, t+3
sT0, sT1, sT2, sT3 = S(40), S(41), S(42), S(43)
sTM0 = S(44, 2)
sTM1 = S(46, 2)
sWC, sWM = S(50), S(51)          # stamps build: barrier-wait cycles after the matrix / vector phase
sBA, sBB = S(52, 2), S(54, 2)
SLOT = 32768
NSLOT = 5
VIMG = 16384
REGION = 1 << 21


class Probe:
    def __init__(self, stagger=True, dma="M", prio="none", soft=True, reads=True, noexp=False, stamps=True, tag="%="):
        self.stagger, self.dma, self.prio, self.soft, self.reads, self.tag = stagger, dma, prio, soft, reads, tag
        self.noexp, self.stamps = noexp, stamps
        self.prog = []

    def L(self, n):
        return f"pp_{n}_{self.tag}"

    def e(self, c):
        self.prog.extend(c)

    # ---- pieces -------------------------------------------------------------
    def dma_piece(self, j, slot_reg):
        """this wave's K (j = 0, 1) or V (j = 2, 3) piece of the tile at sDK into slot_reg"""
        c = []
        if j in (0, 2):
            c += [I("s_add_u32", M0, slot_reg, sWOFF)]
            if j == 2:
                c += [I("s_add_u32", M0, M0, VIMG)]
        off = DMAK(j) if j < 2 else DMAV(j - 2)
        c += [I("global_load_lds_dwordx4", off, sDK, mods=f"offset:{1024 * (j % 2)}")]
        return c

    def dma_advance(self):
        # next tile of the head's 64-tile region (wraps)
        return [I("s_add_u32", sTI, sTI, 1), I("s_and_b32", sTI, sTI, 63),
                I("s_lshl_b32", sT0, sTI, 15), I("s_lshl_b32", sT1, sHEAD, 21), I("s_add_u32", sT0, sT0, sT1),
                I("s_add_u32", sDK[0], sBUF[0], sT0), I("s_addc_u32", sDK[1], sBUF[1], 0)]

    def frag_read(self, n):
        """fragment n of the matrix phase (0-15: V(t-1) (db, kp); 16-31: K(t) (kb, ds)) into ring slot n % 8"""
        f = F(n % NF)
        if n < 16:
            dbp, kp, lo = n // 4, (n // 2) % 2, n % 2
            db = 2 * dbp + lo
            return [I("ds_read_b64_tr_b16", f.sub(2 * h, 2), VVA,
                      mods=f"offset:{256 * (db & 1) + 512 * ((db >> 1) & 1) + 2048 * h + 4096 * kp + 8192 * (db >> 2)}")
                    for h in range(2)]
        m = n - 16
        kbp, ds, lo = m // 8, (m // 2) % 4, m % 2
        kb = 2 * kbp + lo
        return [I("ds_read_b128", f, VKA, mods=f"offset:{512 * (ds & 1) + 2048 * kb + 8192 * (ds >> 1)}")]

    def mfmas(self):
        """(instruction, fragment index) of the matrix phase: PV(t-1) with the row sums, then QK(t)"""
        out = []
        for dbp in range(4):
            for kp in range(2):
                for lo in range(2):
                    db = 2 * dbp + lo
                    n = 4 * dbp + 2 * kp + lo
                    for qb in range(2):
                        out.append((I(MFMA, O_(db, qb), F(n % NF), P_(qb, kp), O_(db, qb)), n))
            qb, kp = dbp & 1, dbp >> 1
            out.append((I(MFMA, L_(qb), ONES, P_(qb, kp), L_(qb)), None))
        for kbp in range(2):
            for ds in range(4):
                for lo in range(2):
                    kb = 2 * kbp + lo
                    n = 16 + 8 * kbp + 2 * ds + lo
                    for qb in range(2):
                        out.append((I(MFMA, S_(kb, qb), F(n % NF), Q_(qb, ds), S_(kb, qb) if ds else 0), n))
        return out

    def c_phase(self):
        c = []
        if self.prio == "flip":
            c.append(I("s_setprio", 1))
        ms = self.mfmas()
        last = {}
        for k, (_, n) in enumerate(ms):
            if n is not None:
                last[n] = k
        after = {}
        for n in range(NF, 32):
            after.setdefault(last[n - NF], []).append(n)
        dma_at = {8: 0, 24: 1, 40: 2, 56: 3} if self.dma == "C" else {}
        for k, (ins, n) in enumerate(ms):
            c.append(ins)
            if self.reads:
                for m in after.get(k, []):
                    c += self.frag_read(m)
            if k in dma_at:
                c += self.dma_piece(dma_at[k], sS3)
        if self.dma == "C":
            c += self.dma_advance()
        if self.prio == "flip":
            c.append(I("s_setprio", 0))
        return c

    def softmax_groups(self):
        """four groups of four slices: [fma x8, exp x8, cvt x4, or3 x2]"""
        sl = [(qb, kb, hh) for qb in range(2) for kb in range(4) for hh in range(2)]
        groups = []
        for g in range(4):
            grp = sl[4 * g:4 * g + 4]
            fm, ex, cv, orr = [], [], [], []
            ws = []
            for n, (qb, kb, hh) in enumerate(grp):
                y0, y1 = Y(2 * n), Y(2 * n + 1)
                s = S_(kb, qb)
                fm += [I("v_fma_f32", y0, s[2 * hh], sC, Neg(MU(qb))), I("v_fma_f32", y1, s[2 * hh + 1], sC, Neg(MU(qb)))]
                xo = "v_mov_b32" if self.noexp else "v_exp_f32"
                ex += [I(xo, y0, y0), I(xo, y1, y1)]
                w = P_(qb, kb >> 1)[2 * (kb & 1) + hh]
                cv.append(I("v_cvt_pk_bf16_f32", w, y0, y1))
                ws.append(w)
            orr = [I("v_or3_b32", ACC, ACC, ws[0], ws[1]), I("v_or3_b32", ACC, ACC, ws[2], ws[3])]
            # interleave fma / exp so a slice's exp follows its fma by a few issues
            vs = []
            for n in range(4):
                vs += fm[2 * n:2 * n + 2]
                if n >= 1:
                    vs += ex[2 * (n - 1):2 * n]
            vs += ex[6:8] + cv + orr
            groups.append(vs)
        return groups

    def m_phase(self, grp):
        c = []
        # slot rotation (tile t -> t + 1) and the next matrix phase's addresses
        c += [I("s_mov_b32", sSM1, sS0), I("s_mov_b32", sS0, sS1), I("s_mov_b32", sS1, sS2), I("s_mov_b32", sS2, sS3),
              I("s_add_u32", sS3, sS3, SLOT), I("s_cmp_ge_u32", sS3, SLOT * NSLOT), I("s_cselect_b32", sS3, 0, sS3)]
        side = []
        if self.dma == "M":
            for j in range(4):
                side.append(self.dma_piece(j, sS2))
        pre = []
        if self.reads:
            pre = [self.frag_read(n) for n in range(NF)]
        groups = self.softmax_groups() if self.soft else [[], [], [], []]
        c += [I("v_mov_b32", ACC, 0)]
        c += [I("v_add_u32", VVA, sSM1, VVL), I("v_add_u32", VKA, sS0, VKL)]
        for g in range(4):
            vs = groups[g]
            # one DMA piece at the head of each group, the fragment pre-reads in the last two groups
            if side:
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
        if self.dma == "M":
            c += self.dma_advance()
        # defer-max check (never taken here)
        c += [I("v_and_b32", T(0), 0x40004000, ACC), I("v_cmp_ne_u32_e32", VCC, 0, T(0)),
              I("s_cbranch_vccnz", self.L(f"rare{grp}")), label(self.L(f"ret{grp}"))]
        return c

    def bar(self, acc):
        """s_barrier; with stamps, the cycles spent waiting at it added to acc"""
        if not self.stamps:
            return [I("s_barrier")]
        return [I("s_memtime", sBA), I("s_barrier"), I("s_memtime", sBB), I("s_waitcnt", "lgkmcnt(0)"),
                I("s_sub_u32", sT3, sBB[0], sBA[0]), I("s_add_u32", acc, acc, sT3)]

    # ---- whole kernel -------------------------------------------------------
    def build(self, in_kernarg="%0", in_wg="%1", in_wave="%2"):
        e = self.e
        e([I("s_mov_b64", sKA, in_kernarg), I("s_mov_b32", sWG, in_wg), I("s_mov_b32", sWAVE, in_wave),
           I("s_load_dwordx8", S(20, 8), sKA, 0), I("s_waitcnt", "lgkmcnt(0)")])
        e([I("s_lshr_b32", sGRP, sWAVE, 2), I("s_lshl_b32", sWOFF, sWAVE, 11)])
        # head = 2 (wg & 7) + ((wg >> 3) >> 4) & 1: the 16 workgroups of a head share an XCD
        e([I("s_and_b32", sT0, sWG, 7), I("s_lshl_b32", sT0, sT0, 1), I("s_lshr_b32", sT1, sWG, 7),
           I("s_and_b32", sT1, sT1, 1), I("s_add_u32", sHEAD, sT0, sT1), I("s_mov_b32", sTI, 0),
           I("s_lshl_b32", sT1, sHEAD, 21), I("s_add_u32", sDK[0], sBUF[0], sT1), I("s_addc_u32", sDK[1], sBUF[1], 0)])
        e([I("v_mbcnt_lo_u32_b32", LANE, -1, 0), I("v_mbcnt_hi_u32_b32", LANE, -1, LANE),
           I("v_and_b32", VI, 15, LANE), I("v_lshrrev_b32", VG, 4, LANE)])
        t = [T(k) for k in range(4)]
        # K read base 16 (g&1) + 32 (i&7) + 256 (g>>1) + 1024 (i>>3); V read base 8 i + 128 (g&1) + 1024 (g>>1) + 16384
        e([I("v_and_b32", t[0], 1, VG), I("v_lshlrev_b32", t[0], 4, t[0]),
           I("v_and_b32", t[1], 7, VI), I("v_lshlrev_b32", t[1], 5, t[1]), I("v_add_u32", t[0], t[0], t[1]),
           I("v_lshrrev_b32", t[1], 1, VG), I("v_lshlrev_b32", t[1], 8, t[1]), I("v_add_u32", t[0], t[0], t[1]),
           I("v_lshrrev_b32", t[1], 3, VI), I("v_lshlrev_b32", t[1], 10, t[1]), I("v_add_u32", VKL, t[0], t[1])])
        e([I("v_lshlrev_b32", t[0], 3, VI), I("v_and_b32", t[1], 1, VG), I("v_lshlrev_b32", t[1], 7, t[1]),
           I("v_add_u32", t[0], t[0], t[1]), I("v_lshrrev_b32", t[1], 1, VG), I("v_lshlrev_b32", t[1], 10, t[1]),
           I("v_add_u32", t[0], t[0], t[1]), I("v_add_u32", VVL, VIMG, t[0])])
        # DMA lane offsets: 16 lane + 2048 wave (+ 16384 for V)
        e([I("v_lshlrev_b32", t[0], 4, LANE), I("v_add_u32", DMAK(0), sWOFF, t[0]), I("v_mov_b32", DMAK(1), DMAK(0)),
           I("v_add_u32", DMAV(0), VIMG, DMAK(0)), I("v_mov_b32", DMAV(1), DMAV(0))])
        # Q from the buffer (random bf16), O and l zero, ones, mu
        e([I("v_lshlrev_b32", t[2], 6, LANE)])
        for qb in range(2):
            for ds in range(4):
                e([I("global_load_dwordx4", Q_(qb, ds), t[2], sBUF, mods=f"offset:{64 * (4 * qb + ds)}")])
        e([I("v_accvgpr_write_b32", A(k), 0) for k in range(64)])
        e([I("v_mov_b32", L_(qb)[r], 0) for qb in range(2) for r in range(4)])
        e([I("v_mov_b32", ONES[k], 0x3F803F80) for k in range(4)])
        e([I("v_mov_b32", MU(0), sMU), I("v_mov_b32", MU(1), sMU)])
        e([I("v_mov_b32", P_(qb, kp)[r], 0x3C003C00) for qb in range(2) for kp in range(2) for r in range(4)])
        # ring: tiles 0, 1, 2 in slots 0, 1, 2 now; t = 0: slot(t-1) = 4
        e([I("s_mov_b32", sSM1, 4 * SLOT), I("s_mov_b32", sS0, 0), I("s_mov_b32", sS1, SLOT),
           I("s_mov_b32", sS2, 2 * SLOT), I("s_mov_b32", sS3, 3 * SLOT)])
        for slot in range(3):
            e([I("s_mov_b32", sT2, slot * SLOT)])
            for j in range(4):
                e(self.dma_piece(j, sT2))
            e(self.dma_advance())
        e([I("s_waitcnt", "vmcnt(0)"), I("s_barrier")])
        e([I("v_add_u32", VVA, sSM1, VVL), I("v_add_u32", VKA, sS0, VKL)])
        if self.reads:
            for n in range(NF):
                e(self.frag_read(n))
        if self.prio == "B":
            skip = self.L("noprio")
            e([I("s_cmp_eq_u32", sGRP, 0), I("s_cbranch_scc1", skip), I("s_setprio", 1), label(skip)])
        e([I("s_memtime", sTM0), I("s_waitcnt", "lgkmcnt(0)")])
        if self.stagger:
            skip = self.L("nostag")
            e([I("s_cmp_eq_u32", sGRP, 0), I("s_cbranch_scc1", skip), I("s_barrier"), label(skip)])
        # one loop per wave group: tile t+3 is DMA'd in M(t); group A (half-periods 2t / 2t+1) waits for
        # the pieces of M(t-2) at the end of M(t), group B (2t+1 / 2t+2) for those of M(t-1) -- either
        # way tile t+1 is in LDS before the first matrix phase that reads it
        e([I("s_mov_b32", sWC, 0), I("s_mov_b32", sWM, 0)])
        e([I("s_mov_b32", sIT, 0), I("s_cmp_eq_u32", sGRP, 1), I("s_cbranch_scc1", self.L("loopB"))])
        for grp, wait in ((0, 8), (1, 4)):
            lp = self.L("loopA" if grp == 0 else "loopB")
            e([label(lp)])
            e(self.c_phase())
            e(self.bar(sWC))
            e(self.m_phase(grp))
            e([I("s_waitcnt", f"vmcnt({wait if self.stagger else 4})")])
            e(self.bar(sWM))
            e([I("s_add_u32", sIT, sIT, 1), I("s_cmp_lt_u32", sIT, sNIT), I("s_cbranch_scc1", lp)])
            if grp == 0:
                if self.stagger:
                    e([I("s_barrier")])
                e([I("s_branch", self.L("done"))])
        e([label(self.L("done"))])
        e([I("s_memtime", sTM1), I("s_waitcnt", "vmcnt(0) lgkmcnt(0)")])
        # out[4 wg + wave] = cycles (low word), lane 0 only; a checksum word keeps the results live
        e([I("s_sub_u32", sT0, sTM1[0], sTM0[0]), I("v_mov_b32", T(1), sT0),
           I("s_lshl_b32", sT1, sWG, 3), I("s_add_u32", sT1, sT1, sWAVE), I("s_lshl_b32", sT1, sT1, 2),
           I("v_mov_b32", T(2), sT1),
           I("v_accvgpr_read_b32", T(3), O_(0, 0)[0]), I("v_add_u32", T(3), T(3), L_(0)[0]),
           I("v_add_u32", T(3), T(3), S_(0, 0)[0]),
           I("s_mov_b64", EXEC, 1), I("global_store_dword", T(2), T(1), sOUT),
           I("v_add_u32", T(4), 8192, T(2)), I("global_store_dword", T(4), T(3), sOUT),
           I("v_mov_b32", T(5), sWC), I("v_add_u32", T(6), 16384, T(2)), I("global_store_dword", T(6), T(5), sOUT),
           I("v_mov_b32", T(7), sWM), I("v_add_u32", T(8), 24576, T(2)), I("global_store_dword", T(8), T(7), sOUT),
           I("s_mov_b64", EXEC, -1), I("s_waitcnt", "vmcnt(0)"), I("s_branch", self.L("exit"))])
        e([label(self.L("rare0")), I("s_branch", self.L("ret0"))])
        e([label(self.L("rare1")), I("s_branch", self.L("ret1"))])
        e([label(self.L("exit"))])
        return self.prog


VARIANTS = {
    "pp": dict(),
    "pp_nostamp": dict(stamps=False),
    "pp_prioflip": dict(prio="flip"),
    "pp_dmaC": dict(dma="C"),
    "pp_nodma": dict(dma="none"),
    "pp_nosoft": dict(soft=False),
    "pp_noexp": dict(noexp=True),
    "pp_noreads": dict(reads=False),
    "lockstep": dict(stagger=False),
    "mfma_reads": dict(dma="none", soft=False),
    "mfma_only": dict(dma="none", soft=False, reads=False),
}


def render():
    lines = ["// GENERATED by tools/v14/probe.py -- timing probe, results meaningless", "#pragma once", ""]
    for name, kw in VARIANTS.items():
        prog, st = finalize(Probe(**kw).build())
        lines.append(f"// {name}: {len(prog)} instructions, nops {st['nop_ws']}, waits {st['waits']}")
        lines.append(f"#define PP_BODY_{name} \\")
        for ins in prog:
            t = ins.text()
            lines.append(f'    "{t}\\n" \\' if ins.op == "label" else f'    "\\t{t}\\n" \\')
        lines.append('    ""')
        lines.append("")
    clob = [f'"v{i}"' for i in range(128)] + [f'"a{i}"' for i in range(128)] + \
           [f'"s{i}"' for i in range(16, 56) if i != 32] + ['"vcc"', '"scc"', '"m0"', '"memory"']
    lines.append("#define PP_CLOBBERS \\")
    for k in range(0, len(clob), 16):
        sep = ", \\" if k + 16 < len(clob) else ""
        lines.append("    " + ", ".join(clob[k:k + 16]) + sep)
    lines.append("")
    lines.append("#define PP_VARIANTS(X) " + " ".join(f"X({n})" for n in VARIANTS))
    lines.append("")
    return "\n".join(lines)


if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "probe_asm.h")
    with open(out, "w") as f:
        f.write(render())
    print(out)
