"""attn_fwd_pp64 / pp64h: flash-attention forward at head dim 64 with two
waves per SIMD in ping-pong (round-6 verdict item 2b; the timing probe that
motivated it is tools/v14/probe64.py, profiles/r06/probe64/; the A/B of the
phase placements below is profiles/r06/pp64/).

Workgroup of 8 waves, 64 query rows each (a 512-row block of one head).  Waves
w and w + 4 share a SIMD.  Group A (waves 0-3) and group B (waves 4-7) run the
same per-tile program, B half a period behind A, every half-period ending at
a workgroup barrier, so while one wave of a SIMD is in its matrix phase the
other is in its vector phase:

  C(t) (matrix): l += 1^T P(t-1) (8 MFMAs) and the defer-max check of tile
         t-1 (bf16), PV(t-1) (32 MFMAs, the V^T fragments of t-1 already in
         the fragment ring) and QK(t) (32 MFMAs) with K(t)'s 8 fragment reads
         in PV's gaps, V^T(t)'s 8 fragment reads as QK frees the ring slots,
         and tile t+4's two LDS-DMA pieces (per wave);
  M(t) (vector): the softmax of S(t) in place (fma, exp, cvt into P); fp16:
         the P-bit check; the wait.

Moving the DMA, the V^T reads and the row sums out of the vector phase (the
probe's layout) into the matrix phase took bf16 from level with v13 to +14 %:
the vector phase was the long one.

The numerics are attn_fwd_v13's head-dim-64 ones (tools/v13/kernel.py):
mu = (row max of tile 0) c + muoff, P = 16-bit(exp2(s c - mu)); bf16: v_exp's
clamp and the l >= 1 check (LCHECK), bitwise v13's result; fp16: the P-bit
check (some P >= 2) in the vector phase, the fma kept (v13h prescales Q instead:
QSCALE's -mu C operands need 16 VGPRs this layout does not have).  The rare
path recomputes S from K, moves mu, rescales O and l, redoes P.  The same LDS
images, swizzle and fragment offsets as v13's D = 64 program in compact 16 KiB
ring slots (K image, then V image at +8 KiB), 6 slots.

Registers (256 per wave: 128 V + 128 A):
  a0-63 O^T (4 d-blocks x 4 q-blocks), a64-95 Q, a96-127 fragment ring (8);
  v0-63 S (softmax in place), v64-95 P, v96-111 l, v112-115 ones,
  v116-119 mu, v120-127 addresses, DMA lane offsets and two temporaries.

One block per workgroup (grid = B H ceil(Nq / 512)), the block walk of v13's
block_params (each XCD a contiguous range of blocks, so a head's blocks share
an L2).  Non-causal, Nk % 64 == 0; the launcher routes every other case, and
shapes whose 512-row blocks would not fill the chip, to attn_fwd_v13.

Vector-memory order per wave (the waits below count on it): the block's 8 Q
loads, tiles 0-3's DMA pieces (2 each), then 2 pieces per C phase (tile t+4,
or the last tile again once the stream has reached it -- into a dead slot);
the O stores last.  A ends M(t) with vmcnt(6) (its pieces up to tile t+1
landed), B with vmcnt(4) (up to t+2): B's M(t) is a half-period later and
tile t+2 is read by A right after the next barrier.  A DMA into slot
(t+4) % 6 overwrites tile t-2, last read (B's rescale path) a half-period
before A's C(t) starts.
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from v13 import kernel as K  # noqa: E402
from v13.isa import A, EXEC, Ins, M0, Neg, S, V, VCC, finalize, label  # noqa: E402

MF = "v_mfma_f32_16x16x32_bf16"
SLOT = 16384
NSLOT = 6
VIMG = 8192
BF16_ONES = 0x3F803F80
NEGONES = 0xBF80BF80


def I(op, *ops, mods=""):
    return Ins(op, *ops, mods=mods)


def mfma(d, a, b, c):
    return I(MF, d, a, b, c)


# ---- registers -------------------------------------------------------------
def S_(kb, qb):
    return V(4 * (4 * qb + kb), 4)


def P_(qb, kp):
    return V(64 + 4 * (2 * qb + kp), 4)


def L_(qb):
    return V(96 + 4 * qb, 4)


ONES = V(112, 4)


def MU(qb):
    return V(116 + qb)


VKL, VVL, VKA, VVA, DMAK, DMAV, T0, T1 = (V(120 + k) for k in range(8))


def O_(db, qb):
    return A(4 * (4 * db + qb), 4)


def Q_(qb, ds):
    return A(64 + 4 * (2 * qb + ds), 4)


def F(n):
    return A(96 + 4 * (n % 8), 4)


# SGPRs: kernel.py's for what block_params reads and writes, the rest ours
sKA, sWKOFF, sL, sC, sNT, sTBK, sTBV = K.sKA, K.sWKOFF, K.sL, K.sC, K.sNT, K.sTBK, K.sTBV
sNQH, sNOH, sNQ0, sT8, sRET = K.sNQH, K.sNOH, K.sNQ0, K.sT8, K.sRET
sT2, sT3, sT6, sT7 = K.sT2, K.sT3, K.sT6, K.sT7
ARG, AI = K.ARG, K.AI
sDK, sDV, sDI, sT = S(36, 2), S(38, 2), S(40), S(41)
sSC, sSP, sSD, sWPC, sMUO = S(42), S(43), S(44), S(45), S(46)
sM0 = S(47)  # m0 at entry (hipcc reserves m0: restored at exit, not clobbered)
# the persistent walk: the current block's O head and first row (block_params
# writes the NEXT block's into sNQH / sNOH / sNQ0), whether block L + G exists,
# and its K / V heads for the DMA stream
sCOH, sCQ0 = S(24, 2), S(26)
sNXK, sNXV = S(50, 2), S(34, 2)
# causal: the key-tile offset (Nk - Nq) / 64 (kernel.py's register, which
# block_params reads) and the wave's diagonal tile
sOFFT, sDIAG = K.sOFFT, S(48)


def slices():
    return [(qb, kb, hh) for qb in range(4) for kb in range(4) for hh in range(2)]


def block_params_512(sx, causal=False, uid=0):
    """kernel.py's block_params with 512-row blocks: q0 = 512 qblk + 64 wave;
    causal (the remap walk, heaviest block first): the block's key tiles
    min(nt, 8 qblk + 8 + offt)"""
    K.GEOM["hd"] = 64  # WSH 11: sWKOFF = wave << 11 gives 64 wave
    K.RAGGED[0] = K.BALANCED[0] = K.SHORTFIRST[0] = False
    c = K.block_params(sx, causal=causal, uid=f"pp{uid}", rev=0)

    def patch(op, a, b, old, new):
        hits = [i for i, ins in enumerate(c) if ins.op == op and str(ins.ops[0]) == str(a)
                and str(ins.ops[1]) == str(b) and ins.ops[2] == old]
        assert len(hits) == 1, (op, hits)
        c[hits[0]] = I(op, a, b, new)
    patch("s_lshl_b32", K.sT2, K.sT2, 8, 9)
    if causal:
        patch("s_lshl_b32", sT8, K.sT2, 2, 3)
        patch("s_add_u32", sT8, sT8, 4, 8)
    return c


class PP64:
    """dma_in: the tile's LDS-DMA pieces in the vector phase ("M", the
    product) or the matrix phase ("C"); split: softmax slices of key block 0
    (0-8) done in the matrix phase after QK's first key block instead of the
    vector phase; vr_in: the 8 V^T fragment reads of tile t for PV(t) at the
    end of M(t) ("M") or in C(t) as QK(t) frees the ring slots ("C")
    (A/B knobs, tools/v14/build_pp64_ab.sh); rs_in: l += 1^T P(t) at the
    end of M(t) ("M") or at the head of C(t+1), right before the check ("C")"""

    def __init__(self, tag="%=", dtype="bf16", dma_in="C", split=0, vr_in="C", rs_in="C", causal=False, hchk="M",
                 dma_at=20):
        assert dtype in ("bf16", "f16") and dma_in in ("M", "C") and vr_in in ("M", "C") and rs_in in ("M", "C")
        assert 0 <= split <= 16 and not (split and rs_in == "M" and vr_in == "C" and False)
        # fp16: P packed to fp16 and checked by the bit-14 test in the vector
        # phase (v13's fp16 rule: the l >= 1 test needs muoff >> log2 Nk, which
        # fp16 P cannot give); the product placements only
        self.f16 = dtype == "f16"
        assert not self.f16 or (dma_in, vr_in, rs_in) == ("C", "C", "C")
        self.mf = "v_mfma_f32_16x16x32_f16" if self.f16 else MF
        self.cvt = "v_cvt_pk_f16_f32" if self.f16 else "v_cvt_pk_bf16_f32"
        self.ones = 0x3C003C00 if self.f16 else BF16_ONES
        self.negones = 0xBC00BC00 if self.f16 else NEGONES
        self.dma_in, self.split, self.vr_in, self.rs_in = dma_in, split, vr_in, rs_in
        # causal (bottom-right, Nq and Nk - Nq multiples of 64): per wave, key
        # tiles before its diagonal tile run as above, the diagonal tile is
        # masked by VALU before the softmax, tiles past it get P = 0; one
        # block per workgroup, heaviest first
        self.causal = causal
        assert not (causal and split)
        # fp16's P-bit check at the end of M(t) ("M") or at the head of
        # C(t+1), before that tile's row sums ("C": the OR of P(t)'s words
        # moves out of the vector phase; the rescale path then runs in the
        # matrix phase like bf16's, with no row sums to take back)
        assert hchk in ("M", "C") and not (hchk == "C" and split)
        self.hchk = hchk if self.f16 else "M"
        self.dma_at = dma_at  # (matrix-phase MFMA after which the DMA pieces issue; A/B knob)
        # whether block L + G exists (the persistent walk); causal needs s27
        # for block_params' key-tile offset.  (Not s33: the bf16 body with
        # sHASN in s33 ran 10 % slower, 1092 vs 1212-1244 TF/s, same process,
        # profiles/r06/pp64/ab10_regress_*.jsonl -- s33 is the ABI's frame pointer)
        global sHASN
        sHASN = S(49) if causal else S(27)
        self.tag = tag
        self.prog = []
        self.sites = []

    def L(self, n):
        return f"pp64{'h' if self.f16 else ''}{'c' if self.causal else ''}_{n}_{self.tag}"

    def e(self, c):
        self.prog.extend(c)

    # ---- pieces -------------------------------------------------------------
    def dma_tile(self, slot):
        """this wave's K piece and V piece of the stream's tile into slot (an
        SGPR or an immediate); then the stream moves on unless it is parked
        on the last tile"""
        return [I("s_add_u32", M0, slot, sWPC), I("global_load_lds_dwordx4", DMAK, sDK),
                I("s_add_u32", M0, M0, VIMG), I("global_load_lds_dwordx4", DMAV, sDV),
                I("s_add_u32", sDI, sDI, 1), I("s_cmp_lt_u32", sDI, sNT),
                I("s_cselect_b32", sT6, sTBK, 0), I("s_cselect_b32", sT7, sTBV, 0),
                I("s_add_u32", sDK[0], sDK[0], sT6), I("s_addc_u32", sDK[1], sDK[1], 0),
                I("s_add_u32", sDV[0], sDV[0], sT7), I("s_addc_u32", sDV[1], sDV[1], 0),
                # past the block's last tile: the next block's tile 0 if there is one
                I("s_cmp_eq_u32", sDI, sNT), I("s_cselect_b32", sT6, sHASN, 0), I("s_cmp_eq_u32", sT6, 1),
                I("s_cselect_b64", sDK, sNXK, sDK), I("s_cselect_b64", sDV, sNXV, sDV),
                I("s_cselect_b32", sDI, 0, sDI)]

    @staticmethod
    def next_slot(r):
        return [I("s_add_u32", r, r, SLOT), I("s_cmp_ge_u32", r, SLOT * NSLOT), I("s_cselect_b32", r, 0, r)]

    @staticmethod
    def k_read(n, base):
        """K fragment (kb, ds) = n - 8 .. of the tile at base into ring slot n"""
        m = n % 8
        kb, ds = m // 2, m % 2
        return [I("ds_read_b128", F(n), base, mods=f"offset:{512 * ds + 2048 * kb}")]

    @staticmethod
    def v_read(n, base):
        """V^T fragment (db, kp) = divmod(n, 2) of the tile at base into ring slot n"""
        db, kp = n // 2, n % 2
        return [I("ds_read_b64_tr_b16", F(n).sub(2 * h, 2), base,
                  mods=f"offset:{256 * (db & 1) + 512 * ((db >> 1) & 1) + 2048 * h + 4096 * kp}")
                for h in range(2)]

    def qk(self):
        return [I(self.mf, S_(kb, qb), F(8 + 2 * kb + ds), Q_(qb, ds), S_(kb, qb) if ds else 0)
                for kb in range(4) for ds in range(2) for qb in range(4)]

    def pv(self):
        return [I(self.mf, O_(db, qb), F(2 * db + kp), P_(qb, kp), O_(db, qb))
                for db in range(4) for kp in range(2) for qb in range(4)]

    def rowsums(self, ones):
        return [I(self.mf, L_(qb), ones, P_(qb, kp), L_(qb)) for qb in range(4) for kp in range(2)]

    def slice_ins(self, qb, kb, hh):
        s = S_(kb, qb)
        y0, y1 = s[2 * hh], s[2 * hh + 1]
        xm = "" if self.f16 else "clamp"  # (fp16: P >= 2 is the check's signal)
        # (the pair on one v_pk_fma_f32 -- hipcc's broadcast form, op_sel_hi
        # [1,0,h] -- was built and measured: 15 % slower both dtypes and the
        # bf16 output wrong, max diff 6-16, while the emulator, which models
        # no hazard for it, agreed with f64; profiles/r06/pp64/ab13_pkfma_*)
        fm = [I("v_fma_f32", y0, y0, sC, Neg(MU(qb))), I("v_fma_f32", y1, y1, sC, Neg(MU(qb)))]
        return (fm,
                [I("v_exp_f32", y0, y0, mods=xm), I("v_exp_f32", y1, y1, mods=xm)],
                [I(self.cvt, P_(qb, kb >> 1)[2 * (kb & 1) + hh], y0, y1)])

    def exps_all(self):
        c = []
        for (qb, kb, hh) in slices():
            f, x, v = self.slice_ins(qb, kb, hh)
            c += f + x + v
        return c

    def check(self, rare):
        k = len(self.sites)
        ret = self.L(f"ret{k}")
        self.sites.append((k, ret))
        return [I("v_max3_f32", T0, L_(0)[0], L_(1)[0], L_(2)[0]), I("v_max_f32", T0, T0, L_(3)[0]),
                I("v_cmp_le_f32_e32", VCC, 1.0, T0),  # some row's l >= 1
                I("s_mov_b32", sRET, k), I("s_cbranch_vccnz", rare), label(ret)]

    # ---- phases -------------------------------------------------------------
    def phase_c(self, kind):
        """kind 'first' (QK(0) only), 'mid' (check, PV(t-1), QK(t)), 'tail'
        (check, PV(T)), 'trans' (the persistent walk's block change: check,
        the next block's Q loads, PV(T), the epilogue, O and l zeroed, the
        block registers moved on, QK of the next block's tile 0)"""
        c = [I("s_mov_b32", sSP, sSC)] + self.next_slot(sSC) + [I("v_add_u32", VKA, sSC, VKL)]
        if kind != "first":
            if self.f16 and self.hchk == "C":
                c += self.pbit_check([P_(qb, kp)[w] for qb in range(4) for kp in range(2) for w in range(4)])
            if self.rs_in == "C":
                c += self.rowsums(ONES)
            if not self.f16:
                c += self.check(self.L("rare"))
        dma = self.dma_tile(sSD) + self.next_slot(sSD) if self.dma_in == "C" and kind != "tail" else []
        if kind == "trans":
            # after the check (its rescale path reads this block's Q); the
            # pieces right behind the Q loads, so the wait QK(0) needs for Q
            # leaves them and the epilogue's stores in flight
            c += self.q_loads() + dma
            dma = []
        vr = self.vr_in == "C" and kind != "tail"
        if vr:
            c += [I("v_add_u32", VVA, sSC, VVL)]
        if kind == "first":
            for n in range(8, 16):
                c += self.k_read(n, VKA)
            qk = self.qk()
            for i, ins in enumerate(qk):
                c.append(ins)
                if i == 8:
                    c += dma
                if vr and i % 4 == 3:  # ring slot i // 4 consumed: V^T fragment i // 4 of this tile
                    c += self.v_read(i // 4, VVA)
            return c
        ms = self.pv()
        after = {}
        if kind == "trans":
            after[31] = ["epi"]
        if kind in ("mid", "trans"):
            ms += self.qk()
            for n in range(8, 16):
                after.setdefault(4 * (n - 8) + 3, []).append(n)
                if vr:
                    after.setdefault(32 + 4 * (n - 8) + 3, []).append(n - 8 + 100)
            if dma:
                after.setdefault(self.dma_at, []).append("dma")
        sp = []
        if kind == "mid" and self.split:
            if self.f16:  # the P-bit OR starts with the slices this phase takes
                c += [I("v_mov_b32", T1, 0)]
            prev = None
            for x in self.c_slices():
                f, e_, v = self.slice_ins(*x)
                sp.append(f + e_ + v)
                if self.f16 and prev is not None:
                    sp[-1] = sp[-1] + [I("v_or3_b32", T1, T1, prev[0].ops[0], v[0].ops[0])]
                    prev = None
                else:
                    prev = v
            if self.f16 and prev is not None:
                sp[-1] = sp[-1] + [I("v_or_b32", T1, T1, prev[0].ops[0])]
        for i, ins in enumerate(ms):
            c.append(ins)
            for n in after.get(i, []):
                if n == "epi":
                    c += self.block_change()
                    continue
                c += dma if n == "dma" else self.v_read(n - 100, VVA) if n >= 100 else self.k_read(n, VKA)
            if sp and i >= 44 and (i - 44) % 2 == 0:
                c += sp.pop(0)
        for x in sp:
            c += x
        return c

    def q_loads(self):
        """the Q rows min(q0 + 16 qb + i, Nq - 1) of the block in sNQH / sNQ0,
        8 g elements into the row (S's registers as temporaries)"""
        LANE, VI, VG, TA, TB = V(0), V(1), V(2), V(3), V(4)
        c = [I("v_mbcnt_lo_u32_b32", LANE, -1, 0), I("v_mbcnt_hi_u32_b32", LANE, -1, LANE),
             I("v_and_b32", VI, 15, LANE), I("v_lshrrev_b32", VG, 4, LANE), I("v_lshlrev_b32", TB, 4, VG),
             I("s_sub_u32", sT6, ARG(AI["nq"]), 1)]
        for qb in range(4):
            c += [I("v_add_u32", TA, sNQ0, VI), I("v_add_u32", TA, 16 * qb, TA), I("v_min_u32", TA, sT6, TA),
                  I("v_mul_lo_u32", TA, TA, ARG(AI["qn"])), I("v_add_u32", V(8 + qb), TA, TB)]
        for qb in range(4):
            for ds in range(2):
                c += [I("global_load_dwordx4", Q_(qb, ds), V(8 + qb), sNQH, mods=f"offset:{64 * ds}")]
        return c

    def next_params(self):
        """sHASN = L + G < nblocks; if so block L + G's Q / O heads and first
        row into sNQH / sNOH / sNQ0 and its K / V heads into sNXK / sNXV"""
        skip = self.L(f"nonext{len(self.prog)}_{self.nuid()}")
        return ([I("s_add_u32", sT7, sL, ARG(AI["G"])), I("s_cmp_lt_u32", sT7, ARG(AI["nblocks"])),
                 I("s_cselect_b32", sHASN, 1, 0), I("s_cbranch_scc0", skip)] + block_params_512(sT7, False, self.nuid()) +
                [I("s_mov_b64", sNXK, S(K.sT0.i, 2)), I("s_mov_b64", sNXV, S(sT2.i, 2)), label(skip)])

    def nuid(self):
        self.uid = getattr(self, "uid", 0) + 1
        return self.uid

    def block_change(self):
        """inside the block-change matrix phase, after PV(T): this block's
        epilogue, O and l zeroed, the next block current, its successor's
        parameters"""
        c = self.epilogue()
        c += [I("v_accvgpr_write_b32", A(k), 0) for k in range(64)]
        c += [I("v_mov_b32", L_(qb)[r], 0) for qb in range(4) for r in range(4)]
        c += [I("s_add_u32", sL, sL, ARG(AI["G"])), I("s_mov_b64", sCOH, sNOH), I("s_mov_b32", sCQ0, sNQ0)]
        return c + self.next_params()

    def pbit_check(self, words):
        """fp16: the rescale path when some P >= 2 (bit 14 of a half) among words"""
        c = [I("v_or3_b32", T1, words[0], words[1], words[2])]
        for k in range(3, len(words) - 1, 2):
            c.append(I("v_or3_b32", T1, T1, words[k], words[k + 1]))
        if len(words) % 2 == 0:
            c.append(I("v_or_b32", T1, T1, words[-1]))
        k = len(self.sites)
        ret = self.L(f"ret{k}")
        self.sites.append((k, ret))
        return c + [I("v_and_b32", T0, 0x40004000, T1), I("v_cmp_ne_u32_e32", VCC, 0, T0),
                    I("s_mov_b32", sRET, k), I("s_cbranch_vccnz", self.L("rare")), label(ret)]

    def diag_mask(self):
        """the wave's diagonal key tile: 64 t = q0 + Nk - Nq, so key 16 kb +
        4 g + r of the tile is past row 16 qb + i iff kb > qb, or kb == qb and
        4 g + r > i: those scores -> -inf (P's registers as temporaries)"""
        LANE, VI, G4, TR, NINF = V(64), V(65), V(66), V(67), V(68)
        c = [I("v_mov_b32", S_(kb, qb)[r], 0xFF800000) for qb in range(4) for kb in range(qb + 1, 4) for r in range(4)]
        c += [I("v_mbcnt_lo_u32_b32", LANE, -1, 0), I("v_mbcnt_hi_u32_b32", LANE, -1, LANE),
              I("v_and_b32", VI, 15, LANE), I("v_lshrrev_b32", G4, 4, LANE), I("v_lshlrev_b32", G4, 2, G4),
              I("v_mov_b32", NINF, 0xFF800000)]
        for r in range(4):
            c += [I("v_add_u32", TR, r, G4), I("v_cmp_lt_i32_e32", VCC, VI, TR)]
            c += [I("v_cndmask_b32_e32", S_(qb, qb)[r], S_(qb, qb)[r], NINF, VCC) for qb in range(4)]
        return c

    def c_slices(self):
        """the slices the matrix phase takes (key block 0, q-block major)"""
        return [(qb, kb, hh) for kb in range(2) for qb in range(4) for hh in range(2)][:self.split]

    def phase_m(self, first, wait):
        """tile t's softmax (and the knobs' row sums, V^T reads, DMA); causal:
        the wave's diagonal tile masked first, the tiles past it P = 0"""
        if not self.causal:
            return self.m_body(first) + [I("s_waitcnt", f"vmcnt({wait})"), I("s_barrier")]
        u = self.nuid()
        dg, by, done = self.L(f"mdiag{u}"), self.L(f"mbeyond{u}"), self.L(f"mdone{u}")
        c = [I("s_cmp_eq_u32", sT, sDIAG), I("s_cbranch_scc1", dg)]
        if not first:  # (tile 0 is never past a diagonal)
            c += [I("s_cmp_gt_u32", sT, sDIAG), I("s_cbranch_scc1", by)]
        c += self.m_body(first) + [I("s_branch", done), label(dg)] + self.diag_mask() + self.m_body(first)
        if not first:
            c += [I("s_branch", done), label(by)]
            c += [I("v_mov_b32", P_(qb, kp)[r], 0) for qb in range(4) for kp in range(2) for r in range(4)]
        return c + [label(done), I("s_waitcnt", f"vmcnt({wait})"), I("s_barrier")]

    def m_body(self, first):
        c = self.dma_tile(sSD) + self.next_slot(sSD) if self.dma_in == "M" else []
        if first:
            # exact row max of tile 0 -> mu = max c + muoff (P's registers as temporaries)
            for qb in range(4):
                m = V(64 + qb)
                c += K.row_max(qb, m, V(68), V(69))
                c += [I("v_mul_f32", m, sC, m), I("v_add_f32", MU(qb), sMUO, m)]
        sl = slices() if first else [x for x in slices() if x not in self.c_slices()]
        fm, ex, cv = zip(*(self.slice_ins(*x) for x in sl))
        rs = self.rowsums(ONES) if self.rs_in == "M" else [[] for _ in range(8)]
        if not first and self.rs_in == "M":  # row sums of the P blocks the matrix phase completed
            cs = self.c_slices()
            c += [rs[2 * qb + kp] for qb in range(4) for kp in range(2)
                  if all((qb, kb, hh) in cs for kb in (2 * kp, 2 * kp + 1) for hh in range(2))]
        reads = [self.v_read(n, VVA) for n in range(8)] if self.vr_in == "M" else []
        if reads:
            c += [I("v_add_u32", VVA, sSC, VVL)]
        n = len(sl)
        mchk = self.f16 and self.hchk == "M"
        if mchk and (first or not self.split):
            c += [I("v_mov_b32", T1, 0)]
        for j in range(n + 2):
            if j < n:
                c += fm[j]
            if 1 <= j <= n:
                c += ex[j - 1]
            if 2 <= j:
                c += cv[j - 2]
                qb, kb, hh = sl[j - 2]
                if mchk and j % 2 == 1:  # the P-bit check: OR of the tile's P words
                    c.append(I("v_or3_b32", T1, T1, cv[j - 3][0].ops[0], cv[j - 2][0].ops[0]))
                if kb & 1 and hh and self.rs_in == "M":  # P(qb, kb >> 1) complete
                    c.append(rs[2 * qb + (kb >> 1)])
            # the V^T reads over the second half
            h0 = n - 16
            if reads and j >= h0 and (j - h0) % 2 == 0 and (j - h0) // 2 < 8:
                c += reads[(j - h0) // 2]
        if mchk:
            k = len(self.sites)
            ret = self.L(f"ret{k}")
            self.sites.append((k, ret))
            c += [I("v_and_b32", T0, 0x40004000, T1), I("v_cmp_ne_u32_e32", VCC, 0, T0),  # some P >= 2
                  I("s_mov_b32", sRET, k), I("s_cbranch_vccnz", self.L("rare")), label(ret)]
        return c

    def epilogue(self):
        """O / l, packed to bf16, stored (rows >= Nq masked); S's and P's
        registers are the temporaries"""
        c = [I("s_nop", 7), I("s_nop", 7)]
        R = [V(k) for k in range(4)]
        TT = [V(4 + k) for k in range(4)]

        def W(k):
            return V(8 + k)

        OOFF = [V(16 + k) for k in range(4)]
        ROW, LANE, VI, VG, TA, TB = V(20), V(24), V(25), V(26), V(21), V(22)
        for qb in range(4):
            c.append(I("v_rcp_f32", R[qb], L_(qb)[0]))
        c += [I("v_mbcnt_lo_u32_b32", LANE, -1, 0), I("v_mbcnt_hi_u32_b32", LANE, -1, LANE),
              I("v_and_b32", VI, 15, LANE), I("v_lshrrev_b32", VG, 4, LANE)]
        for qb in range(4):
            c += [I("v_add_u32", ROW, sCQ0, VI), I("v_add_u32", ROW, 16 * qb, ROW),
                  I("v_mul_lo_u32", TA, ROW, ARG(AI["on"])),
                  I("v_and_b32", TB, 1, VG), I("v_lshlrev_b32", TB, 5, TB), I("v_add_u32", TA, TA, TB),
                  I("v_lshrrev_b32", TB, 1, VG), I("v_lshlrev_b32", TB, 4, TB), I("v_add_u32", OOFF[qb], TA, TB)]
            for dbp in range(2):
                w = 4 * dbp
                for half, db in enumerate((2 * dbp, 2 * dbp + 1)):
                    c += [I("v_accvgpr_read_b32", TT[r], O_(db, qb)[r]) for r in range(4)]
                    c += [I("v_mul_f32", TT[r], TT[r], R[qb]) for r in range(4)]
                    c += [I(self.cvt, W(w + 2 * half), TT[0], TT[1]),
                          I(self.cvt, W(w + 2 * half + 1), TT[2], TT[3])]
                c += [I("v_permlane16_swap_b32", W(w), W(w + 2)), I("v_permlane16_swap_b32", W(w + 1), W(w + 3))]
            c += [I("v_cmp_gt_u32_e32", VCC, ARG(AI["nq"]), ROW), I("s_and_saveexec_b64", S(sT2.i, 2), VCC)]
            for dbp in range(2):
                c.append(I("global_store_dwordx4", OOFF[qb], V(W(4 * dbp).i, 4), sCOH, mods=f"offset:{64 * dbp}"))
            c += [I("s_mov_b64", EXEC, S(sT2.i, 2))]
        return c

    def rare(self):
        """the tile in slot sSP (t-1, checked at the head of C(t)) raised a row
        max: l -= 1^T P(old); S = K Q^T again; mu_new = max(mu, max c +
        muoff); O, l *= exp2(mu - mu_new); P again and l += 1^T P; the V^T
        fragments of the tile back into the ring.  Returns to the site whose
        id is in sRET."""
        c = [label(self.L("rare")), I("s_nop", 7), I("s_nop", 7)]
        # bf16: the tile in slot sSP, checked at the head of C(t+1) after its
        # row sums went into l; fp16: the tile in slot sSC, checked at the end
        # of its own vector phase (its row sums not taken yet)
        mmode = self.f16 and self.hchk == "M"  # (checked in its own vector phase)
        slot, adr = (sSC, VVA) if mmode else (sSP, T1)
        if self.causal and not mmode:
            # a tile past the wave's diagonal has P = 0: l >= 1 from earlier
            # tiles (muoff 0 keeps it there) is no reason to touch it
            c += [I("s_sub_u32", sT6, sT, 1), I("s_cmp_gt_u32", sT6, sDIAG), I("s_cbranch_scc1", self.L("rare_ret"))]
        if not self.f16:
            neg = S_(0, 0)  # S is recomputed below: its first block holds the -1s meanwhile
            c += [I("v_mov_b32", neg[r], self.negones) for r in range(4)]
            c += self.rowsums(neg)
        c += [I("v_add_u32", adr, slot, VKL)]
        for n in range(8, 16):
            c += self.k_read(n, adr)
        c += self.qk()
        if self.causal:  # the checked tile: sT (fp16, vector phase) or sT - 1 (bf16, next matrix phase)
            skip = self.L("rare_nomask")
            c += [I("s_sub_u32", sT6, sT, 0 if mmode else 1), I("s_cmp_eq_u32", sT6, sDIAG),
                  I("s_cbranch_scc0", skip)] + self.diag_mask() + [label(skip)]
        m, t1, t2, al, ot = (V(64 + k) for k in range(5))  # P is rebuilt below
        for qb in range(4):
            c += K.row_max(qb, m, t1, t2)
            c += [I("v_mul_f32", m, sC, m), I("v_add_f32", m, sMUO, m), I("v_max_f32", m, m, MU(qb)),
                  I("v_sub_f32", al, MU(qb), m), I("v_exp_f32", al, al), I("v_mov_b32", MU(qb), m)]
            for db in range(4):
                for r in range(4):
                    c += [I("v_accvgpr_read_b32", ot, O_(db, qb)[r]), I("v_mul_f32", ot, ot, al),
                          I("v_accvgpr_write_b32", O_(db, qb)[r], ot)]
            c += [I("v_mul_f32", L_(qb)[r], L_(qb)[r], al) for r in range(4)]
        c += self.exps_all()
        if not self.f16:
            c += self.rowsums(ONES)
        c += [I("v_add_u32", adr, slot, VVL)]
        for n in range(8):
            c += self.v_read(n, adr)
        c += [I("s_nop", 4), label(self.L("rare_ret"))]
        for k, ret in self.sites:
            c += [I("s_cmp_eq_u32", sRET, k), I("s_cbranch_scc1", ret)]
        c += [I("s_branch", self.L("exit"))]  # unreachable
        return c

    # ---- whole kernel -------------------------------------------------------
    def init(self, in_kernarg, in_wg, in_wave):
        e = self.e
        e([I("s_mov_b32", sM0, M0), I("s_mov_b64", sKA, in_kernarg), I("s_mov_b32", sL, in_wg),
           I("s_lshl_b32", sWKOFF, in_wave, 11),
           I("s_lshl_b32", sWPC, in_wave, 10)])
        # dwords 37..44 (kn, vn, c, muoff, tbk, tbv, ..) into s88..s95, then the
        # block arguments over s56..s92 (load_args)
        e([I("s_load_dwordx8", S(88, 8), sKA, 4 * AI["kn"]), I("s_waitcnt", "lgkmcnt(0)")])
        kn, vn = S(88), S(89)
        e([I("s_mov_b32", sC, S(90)), I("s_mov_b32", sMUO, S(91)), I("s_mov_b32", sTBK, S(92)),
           I("s_mov_b32", sTBV, S(93))])
        LANE, VI, VG = V(0), V(1), V(2)
        t = [V(3 + k) for k in range(6)]
        e([I("v_mbcnt_lo_u32_b32", LANE, -1, 0), I("v_mbcnt_hi_u32_b32", LANE, -1, LANE),
           I("v_and_b32", VI, 15, LANE), I("v_lshrrev_b32", VG, 4, LANE)])
        # K read base: 16 (g&1) + 32 (i&7) + 256 (g>>1) + 1024 (i>>3)
        e([I("v_and_b32", t[0], 1, VG), I("v_lshlrev_b32", t[0], 4, t[0]),
           I("v_and_b32", t[1], 7, VI), I("v_lshlrev_b32", t[1], 5, t[1]), I("v_add_u32", t[0], t[0], t[1]),
           I("v_lshrrev_b32", t[1], 1, VG), I("v_lshlrev_b32", t[1], 8, t[1]), I("v_add_u32", t[0], t[0], t[1]),
           I("v_lshrrev_b32", t[1], 3, VI), I("v_lshlrev_b32", t[1], 10, t[1]), I("v_add_u32", VKL, t[0], t[1])])
        # V read base: 8 i + 128 (g&1) + 1024 (g>>1) + VIMG
        e([I("v_lshlrev_b32", t[0], 3, VI), I("v_and_b32", t[1], 1, VG), I("v_lshlrev_b32", t[1], 7, t[1]),
           I("v_add_u32", t[0], t[0], t[1]), I("v_lshrrev_b32", t[1], 1, VG), I("v_lshlrev_b32", t[1], 10, t[1]),
           I("v_add_u32", t[0], t[0], t[1]), I("v_add_u32", VVL, VIMG, t[0])])
        # DMA lanes: row (L>>1)&7, 16-B chunk 4((L>>5)&1) + 2((L>>4)&1) + (L&1)
        e([I("v_lshrrev_b32", t[2], 1, LANE), I("v_and_b32", t[2], 7, t[2]),
           I("v_lshrrev_b32", t[3], 5, LANE), I("v_and_b32", t[3], 1, t[3]), I("v_lshlrev_b32", t[3], 2, t[3]),
           I("v_lshrrev_b32", t[4], 4, LANE), I("v_and_b32", t[4], 1, t[4]), I("v_lshlrev_b32", t[4], 1, t[4]),
           I("v_add_u32", t[3], t[3], t[4]), I("v_and_b32", t[4], 1, LANE), I("v_add_u32", t[3], t[3], t[4]),
           I("v_lshlrev_b32", t[3], 4, t[3])])
        # piece pc = wave of each image: K rows 16((pc>>1)&3) + 8(pc&1), V rows 8 pc
        e([I("s_lshr_b32", sT2, sWPC, 10),
           I("s_lshr_b32", sT3, sT2, 1), I("s_and_b32", sT3, sT3, 3), I("s_lshl_b32", sT3, sT3, 4),
           I("s_and_b32", sT6, sT2, 1), I("s_lshl_b32", sT6, sT6, 3), I("s_add_u32", sT3, sT3, sT6),
           I("s_lshl_b32", sT6, sT2, 3)])
        for (rb, st, dst) in ((sT3, kn, DMAK), (sT6, vn, DMAV)):
            e([I("v_add_u32", t[5], rb, t[2]), I("v_mul_lo_u32", t[5], t[5], st), I("v_add_u32", dst, t[5], t[3])])
        e(K.load_args())
        e([I("v_mov_b32", ONES[k], self.ones) for k in range(4)])

    def block_setup(self):
        e = self.e
        if self.causal:
            e([I("s_load_dword", sOFFT, sKA, 4 * AI["offt"]), I("s_waitcnt", "lgkmcnt(0)")])
        e(block_params_512(sL, self.causal, self.nuid()))
        # K head in s52:53, V head in s94:95, nt in sT8
        e([I("s_mov_b64", sDK, S(K.sT0.i, 2)), I("s_mov_b64", sDV, S(sT2.i, 2)), I("s_mov_b32", sNT, sT8),
           I("s_mov_b32", sDI, 0), I("s_mov_b64", sCOH, sNOH), I("s_mov_b32", sCQ0, sNQ0)])
        e(self.q_loads())
        if self.causal:  # one block per workgroup; the wave's diagonal key tile (q0 + Nk - Nq) / 64
            e([I("s_mov_b32", sHASN, 0), I("s_lshr_b32", sDIAG, sCQ0, 6), I("s_add_u32", sDIAG, sDIAG, sOFFT)])
        else:
            e(self.next_params())
        for j in range(4):
            e(self.dma_tile(j * SLOT))
        e([I("s_mov_b32", sSD, 4 * SLOT), I("s_mov_b32", sSC, (NSLOT - 1) * SLOT)])
        e([I("v_accvgpr_write_b32", A(k), 0) for k in range(64)])
        e([I("v_mov_b32", L_(qb)[r], 0) for qb in range(4) for r in range(4)])

    def group(self, grp):
        """the tile loop of group A (grp 0) or B (1)"""
        e = self.e
        wait = 6 if grp == 0 else 4
        lp, tail = self.L(f"loop{grp}"), self.L(f"tail{grp}")
        e([I("s_waitcnt", f"vmcnt({wait})"), I("s_barrier")])
        if grp == 1:
            e([I("s_barrier")])  # B runs half a period behind A
        if self.causal:
            e([I("s_mov_b32", sT, 0)])  # (the vector phase's tile index)
        e(self.phase_c("first"))
        e([I("s_barrier")])
        e(self.phase_m(True, wait))
        end = self.L(f"end{grp}")
        e([I("s_mov_b32", sT, 1), label(lp), I("s_cmp_ge_u32", sT, sNT), I("s_cbranch_scc1", end)])
        e(self.phase_c("mid"))
        e([I("s_barrier")])
        e(self.phase_m(False, wait))
        e([I("s_add_u32", sT, sT, 1), I("s_branch", lp)])
        # the block's last tile: the next block of the persistent walk, or the tail
        e([label(end), I("s_cmp_eq_u32", sHASN, 0), I("s_cbranch_scc1", tail)])
        e(self.phase_c("trans"))
        e([I("s_barrier")])
        # the block change issued 16 more vector-memory operations (8 Q loads,
        # 8 O stores) after the pieces this wait is for
        e(self.phase_m(True, wait + 16))
        e([I("s_mov_b32", sT, 1), I("s_branch", lp), label(tail)])
        e(self.phase_c("tail"))
        e(self.epilogue())
        if grp == 0:
            e([I("s_barrier")])  # B's last matrix phase
        e([I("s_branch", self.L("exit"))])

    def build(self, in_kernarg="%0", in_wg="%1", in_wave="%2"):
        self.init(in_kernarg, in_wg, in_wave)
        self.block_setup()
        self.e([I("s_lshr_b32", sT6, sWKOFF, 13), I("s_cmp_eq_u32", sT6, 1),
                I("s_cbranch_scc1", self.L("grpB"))])  # waves 4-7: sWKOFF = wave << 11 >= 8192
        self.group(0)
        self.e([label(self.L("grpB"))])
        self.group(1)
        self.e(self.rare())
        self.e([label(self.L("exit")), I("s_mov_b32", M0, sM0)])
        return self.prog


def render(**kw):
    lines = ["// GENERATED by tools/v14/pp64.py -- do not edit (attn_fwd_pp64: head dim 64, two waves per SIMD)",
             "#pragma once", ""]
    # A/B knobs: key=val for the bf16 body, h_key=val for the fp16 one
    kwb = {k: v for k, v in kw.items() if not k.startswith("h_")}
    kwh = {k[2:]: v for k, v in kw.items() if k.startswith("h_")}
    for name, dt, cz in (("PLI_PP64_BODY", "bf16", False), ("PLI_PP64H_BODY", "f16", False),
                         ("PLI_PP64C_BODY", "bf16", True), ("PLI_PP64HC_BODY", "f16", True)):
        kwx = dict(kwh if dt == "f16" else kwb)
        if cz:
            kwx.pop("split", None)
        prog, st = finalize(PP64(dtype=dt, causal=cz, **kwx).build())
        lines.append(f"// {dt}{' causal' if cz else ''}: {len(prog)} instructions, hazard pass: {st['nop_ws']} nop wait states, "
                     f"{st['waits']} waits")
        lines.append(f"#define {name} \\")
        for ins in prog:
            t = ins.text()
            lines.append(f'    "{t}\\n" \\' if ins.op == "label" else f'    "\\t{t}\\n" \\')
        lines.append('    ""')
        lines.append("")
    clob = [f'"v{i}"' for i in range(128)] + [f'"a{i}"' for i in range(128)] + \
           [f'"s{i}"' for i in range(16, 100) if i != 32] + ['"vcc"', '"scc"', '"memory"']
    lines.append("#define PLI_PP64_CLOBBERS \\")
    for k in range(0, len(clob), 16):
        sep = ", \\" if k + 16 < len(clob) else ""
        lines.append("    " + ", ".join(clob[k:k + 16]) + sep)
    lines.append("")
    return "\n".join(lines)


OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                   "physics-llm-inference_amd", "csrc", "flash_pp64_asm.h")

if __name__ == "__main__":
    if "--ab" in sys.argv:  # --ab NAME key=val ...: tools/ab/pp64_NAME_asm.h
        i = sys.argv.index("--ab")
        name, kw = sys.argv[i + 1], {}
        for a in sys.argv[i + 2:]:
            key, val = a.split("=")
            kw[key] = int(val) if val.lstrip("-").isdigit() else val
        out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ab", f"pp64_{name}_asm.h")
        os.makedirs(os.path.dirname(out), exist_ok=True)
        with open(out, "w") as f:
            f.write(render(**kw))
        print(out)
        sys.exit(0)
    txt = render()
    if "--check" in sys.argv:
        with open(OUT) as f:
            sys.exit(0 if f.read() == txt else 1)
    with open(OUT, "w") as f:
        f.write(txt)
    print(OUT)
