"""attn_fwd_v13: flash-attention forward on v_mfma_f32_16x16x32_bf16, one
wave per SIMD, 64 query rows per wave (reference ch06/flash_attention.py:14-74;
gfx950, bf16, D = 128, Nk a multiple of 64 and >= 128; causal -- bottom-right,
(Nk - Nq) % 64 == 0 -- as the second program, Gen(causal=True)).

The whole kernel body is one generated instruction stream (this module
builds it; tools/gen_flash_v13.py prints it into csrc/flash_v13_asm.h, and
tools/v13/emu.py executes the same program on the CPU).

Layout per wave (lane l: i = l & 15, g = l >> 4):
  * S^T = K Q^T as 4 key-blocks kb x 4 query-blocks qb of 16 x 16
    (v_mfma_f32_16x16x32_bf16, A = K fragment from LDS, B = Q^T fragment;
    both in accumulator registers): lane (g, i) holds keys 16kb + 4g + r
    (r = 0..3) of query 16qb + i.
  * P = bf16(exp2(s * c - mu)) straight from S into the B operand of the PV
    MFMA (key order permuted; the V^T operand is read with the same
    permutation by two ds_read_b64_tr_b16 per fragment).
  * O^T = V^T P^T as 8 d-blocks x 4 q-blocks in a[0:127]; the row sum l on
    the matrix core (an all-ones A operand).
  * Defer-max on P itself: mu = (row max) * c + muoff (a launch argument:
    62 in the product since round 4, 7 before; the text below is for 7) when a tile's max is
    taken, so P <= 2^-7 right after; a tile is accepted while every P < 2,
    which is bit 14 of each bf16 half (one v_or3_b32 per two words).  P >= 2
    means the row max grew by 8 in log2 units (the THR 8 rule of v10/v12):
    the rare path recomputes S from the LDS copy of K, moves mu, rescales O
    and l and redoes the P it covers.
  * K / V tiles arrive by LDS-DMA (1 KiB pieces, each 8 rows x one 128-B
    line) into a 5-slot ring two tiles ahead.  The images are laid out so
    that every fragment read is one base register + an immediate offset and
    bank-conflict free (tools/v13/layout.py checks both).
"""
from __future__ import annotations

from .isa import A, EXEC, Ins, M0, Neg, S, SCC, V, VCC, label

MFMA = "v_mfma_f32_16x16x32_bf16"
BF16_ONES = 0x3F803F80
# the element type of Q / K / V / O and of P (Gen(dtype=...)): the MFMA, the
# all-ones row-sum operand and the f32 -> 16-bit pack (both RNE)
DTYPES = {"bf16": {"mfma": "v_mfma_f32_16x16x32_bf16", "ones": BF16_ONES, "cvt": "v_cvt_pk_bf16_f32"},
          "f16": {"mfma": "v_mfma_f32_16x16x32_f16", "ones": 0x3C003C00, "cvt": "v_cvt_pk_f16_f32"}}
DT = dict(DTYPES["bf16"])
# head dim (Gen(hd=...)): 128, or 64 -- the D = 64 tile images are the first
# halves of the D = 128 ones (K: 8 KiB of 64 keys x 128 B rows, V likewise),
# so the same swizzle, fragment offsets and DMA piece map serve both; per
# tile 16 pieces instead of 32 (4 per wave), 32 + 32 MFMAs instead of 64 + 64
GEOM = {"hd": 128}


def NDS():
    """32-wide d slices of Q / K (QK MFMA k steps)"""
    return GEOM["hd"] // 32


def NDB():
    """16-wide d blocks of O / V (PV MFMA rows)"""
    return GEOM["hd"] // 16


def NPW():
    """LDS-DMA pieces per wave per tile (K half, then V half)"""
    return GEOM["hd"] // 16


def WSH():
    """sWKOFF = wave << WSH() = the wave's byte offset in an image (8 pieces of
    1 KiB per wave at D = 128, 4 at D = 64: 32 hd bytes)"""
    return 12 if GEOM["hd"] == 128 else 11

# ---------------------------------------------------------------- registers


def S_(kb, qb):
    return V(4 * (4 * qb + kb), 4)


def P_(X, qb, kp):
    return V(64 + 32 * X + 4 * (2 * qb + kp), 4)


NVF = 3  # V^T fragment buffers (one d-block each)


def VF(b, kp):
    return V(128 + 8 * b + 4 * kp, 4)


def VFh(b, kp, h):
    return V(128 + 8 * b + 4 * kp + 2 * h, 2)


def L_(qb):
    return V(152 + 4 * qb, 4)


ONES = V(168, 4)


def MU(qb):
    return V(172 + qb)


def ACC(X):
    return V(176 + X)


VKL, VVL, VKA, VVA = V(178), V(179), V(180), V(181)


def DMAK(j):
    return V(182 + j)


def DMAV(j):
    return V(186 + j)


def Y(k):
    return V(190 + k)


NY = 16


def MUC(qb):
    """QSCALE: -mu of q-block qb in all four words (the C operand of the
    block's first QK MFMA); shares v190-205 with Y, which QSCALE leaves idle"""
    return V(190 + 4 * qb, 4)


def TRIMU(qb):
    """QSCALE, causal diagonal step: TRI - mu of q-block qb (T(20+4qb) .. +3)"""
    return V(238 + 4 * qb, 4)


def QOFF(qb):
    return V(250 + qb)  # = T(32 + qb): live only while the Q loads issue


def OOFF(qb):
    return V(234 + qb)  # = T(16 + qb): epilogue only


def OOFFY(qb):
    return V(250 + qb)  # = T(32 + qb) = QOFF(qb): epilogue only (OLINE's second 8 rows)


TRI = V(206, 4)   # causal: the 16 x 16 diagonal block's C operand (0 / -inf)
NINF = V(210, 4)  # causal: -inf (C operand of fully masked chains, cndmask source)


def PM(kb, hh):
    """RAGGED (non-causal, so TRI / NINF's registers are free): the AND mask
    of P word (kb, hh) of the last key tile -- its halves hold keys 16 kb +
    4 g + 2 hh (+1), kept iff the key is >= P0"""
    return V(206 + 2 * kb + hh)


LANE, VI, VG = V(214), V(215), V(216)
STAMPV = V(217)  # diagnostic build only


def T(k):
    assert 0 <= k < 38
    return V(218 + k)  # even base: VGPR tuples must be 64-bit aligned


def O_(db, qb):
    return A(4 * (4 * db + qb), 4)


def Q_(qb, ds):
    return A(128 + 4 * (4 * qb + ds), 4)


def K_(kb, ds):
    return A(192 + 4 * (4 * ds + kb), 4)


# SGPRs (hipcc keeps its own in s0..s15)
sKA = S(16, 2)
sWKOFF, sL, sC, sNT, sTBK, sTBV = S(18), S(19), S(20), S(21), S(22), S(23)  # sWKOFF = 32 hd * wave
sCOH, sCQ0, sOFFT = S(24, 2), S(26), S(27)
# (s32 is hipcc's stack pointer and s100 / s101 are reserved too: the
# program uses s16..s31 and s33..s99 only, so hipcc's -Winline-asm check of
# the clobber list is clean)
sNQH, sNOH, sNQ0, sNXNT, sTD, sDNT = S(28, 2), S(30, 2), S(93), S(33), S(34), S(35)
sNXK, sNXV, sNXIDX, sT = S(36, 2), S(38, 2), S(40), S(41)
sDK, sDV, sDIDX = S(42, 2), S(44, 2), S(46)
sSM1, sS0, sSP1, sSP2, sHASN = S(47), S(48), S(49), S(50), S(51)
sDIR = sHASN  # causal: the current block's stream order (1 = reversed), see block_params
sT0, sT1, sT8, sRET = S(52), S(53), S(54), S(55)
ARGS = 56  # block-parameter arguments: s56..s92 (dwords 0..36)


def ARG(k, n=1):
    return S(ARGS + k, n)


sT2, sT3, sT4, sT5, sT6, sT7 = (S(94 + k) for k in range(6))  # sT2 even: sT2:sT3 is a 64-bit pair
SGPR_FIRST = 16
SGPR_LAST = 99
SGPR_SKIP = (32,)
M0SAVE = (V(217), 63)  # m0 is saved in lane 63 of v217 (the stamp build's record: lanes 0-8) and restored at exit

# kernel argument dwords (V13Args in csrc/flash_v13.hip)
# (dwords 0..36 are reloaded into s56..s92 at every block transition -- no
# instruction writes them, and dropping the reload was measured level; 37..
# are read at init or by a single s_load where needed).  "shifts" packs the
# three magic-division shifts and the head count: shq | shh << 5 | shg << 10
# | H << 16 (SALU shifts read bits 4:0 of their count)
ARG_LAYOUT = ["q", "q_hi", "k", "k_hi", "v", "v_hi", "o", "o_hi",
              "qb", "qb_hi", "qh", "qh_hi", "kb", "kb_hi", "kh", "kh_hi",
              "vb", "vb_hi", "vh", "vh_hi", "ob", "ob_hi", "oh", "oh_hi",
              "qn", "on", "nq", "nt", "qblocks", "nblocks", "magq", "magh",
              "magg", "shifts", "cw", "hx", "G",
              "kn", "vn", "c", "muoff", "tbk", "tbv", "stamp", "stamp_hi",
              "offt", "pad1", "pad2", "pad3", "pad4", "pad5", "pad6", "pad7",
              "pad8", "pad9", "pad10", "pad11", "pad12", "pad13", "pad14", "pad15",
              "pad16", "pad17", "pad18"]
assert len(ARG_LAYOUT) == 64
AI = {n: i for i, n in enumerate(ARG_LAYOUT)}

SLOT = 32768  # one ring slot: K image (16 KiB) then V image (16 KiB)
NSLOT = 5
VIMG = 16384


def I(op, *ops, mods="", note=""):
    return Ins(op, *ops, mods=mods, note=note)


def mfma(d, a, b, c):
    return I(DT["mfma"], d, a, b, c)


# ---------------------------------------------------------------- scheduler


class Fill:
    """filler work for the gaps between MFMAs: a few instructions with an
    issue cost (cycles), dependencies on other fills, an earliest gap and an
    optional deadline gap"""
    __slots__ = ("ins", "cost", "trans", "deps", "sep", "earliest", "deadline", "gap", "tag", "hard", "lds")

    def __init__(self, ins, cost, trans=False, deps=(), sep=1, earliest=0, deadline=None, tag="", hard=False):
        self.ins = ins if isinstance(ins, list) else [ins]
        # LDS bytes this fill reads per wave (a gap of 16 cycles moves at most
        # 1 KiB per wave when all four SIMDs read: 256 B/clk per CU)
        self.lds = sum(1024 if i.op == "ds_read_b128" else 512 if i.op == "ds_read_b64_tr_b16" else 0
                       for i in self.ins)
        self.cost, self.trans, self.deps, self.sep = cost, trans, list(deps), sep
        self.earliest, self.deadline, self.gap, self.tag = earliest, deadline, None, tag
        self.hard = hard  # the deadline is a correctness bound (checked)


LDS_GAP = 1024  # LDS bytes per wave per 16-cycle gap (256 B/clk per CU, 4 waves)
TRANS_PER_GAP = [1]  # transcendental fills per gap (Gen(trans=...), A/B knob)

# timing-only A/B knobs (tools/build_v13_ab.sh; Gen(abl=..., dma_cost=...)):
# ABL "dma" drops the LDS-DMA loads, "exp" turns v_exp_f32 into v_mov_b32,
# "check" drops the defer-max branch, "or" the v_or3_b32 that gather its bits; in the step loop only: "kread" / "vread"
# drop the K / V fragment reads, "barrier" the per-step barrier, "soft" the
# softmax stream -- results wrong, timing only
ABL = set()
DMA_COST = 8
# QSCALE (Gen(qscale=True)): Q is scaled by c = scale * log2(e) once per
# block (bf16, RNE) and -mu enters as the first QK MFMA's C operand, so the
# softmax stream is exp2(S) in place + cvt: no v_fma_f32 per score
QSCALE = [False]
# LCHECK (Gen(lcheck=True), the product since round 5): the defer-max check
# reads the row sums l instead of OR-ing the bits of every P word.  P =
# bf16(exp2(s c - mu)) with v_exp_f32's clamp (P <= 1: never inf), the row-sum
# MFMAs of tile t-1 run at the end of QK(t) (before the check, not in PV(t-1)),
# and a tile takes the rare path once some row's l >= 1.  In the normal regime
# l <= Nk 2^(growth - muoff) << 1; l >= 1 needs a row max grown by about muoff
# - log2(Nk) -- the same event the P >= 2 bit test caught at muoff + 1, a
# little earlier.  A clamped P (growth > muoff) is caught the same way (it
# adds 1 to l) and redone by the rare path, which first takes the tile's old
# sums back out of l.  Saves the 16 v_or3_b32 + v_and + v_cmp per wave-tile
# (3 VALU instead).
LCHECK = [True]
NEGONES = 0xBF80BF80
# SHORTFIRST (Gen(causal=True, short_first=True), A/B knob): the pair walk
# runs each workgroup's short block (height a) first and its long block
# (QB-1-a) second, both streamed forward, so a tile's second read comes at
# most 4a+4 tile-times after its first (the round-4 order reads it again up
# to 64 later, the reversed second block about 67-2u later)
SHORTFIRST = [False]
# RAGGED (Gen(ragged=True), non-causal, Nk % 64 != 0): the last key tile is
# streamed from key Nk - 64 (it overlaps the one before by P0 = 64 - Nk % 64
# keys, so every K / V read stays inside the head); its first P0 keys were
# already counted, so their P is ANDed to 0 before the row sums and PV read
# it.  Their scores are real scores of keys the row max has already seen, so
# mu and the check are unaffected.  P0 rides in the cw argument (unused by the
# non-causal walk).
RAGGED = [False]
# OLINE (Gen(oline=True), A/B knob): the epilogue stores O as whole 128-B
# lines -- 8 rows x 128 B per global_store_dwordx4 instead of the 16 rows x 64
# B the MFMA output layout gives, the halves exchanged between lanes j and j +
# 8 by DPP (3 VALU per word pair).  Bitwise equal and level in throughput
# (profiles/r05/flash/ab_oline.jsonl: the stores drain behind the next
# block), so the product keeps the half-line stores
OLINE = [False]
# SEAMWAIT (Gen(seam_wait=True), A/B knob): the wait before the block's
# first barrier retires only key tile 0's DMA pieces (vmcnt(NPW + 4 NDS))
# instead of every vector-memory operation in flight (vmcnt(0)), so neither
# the last block's O stores nor the Q loads are waited for there (the Q loads
# get the hazard pass's counted wait before the first MFMA that reads them).
# Bitwise equal and level (profiles/r05/flash/ab_seam_wait.jsonl): the seam's
# stores and Q loads cost time (dropping either is +2 % at S 4096, +6 % at
# S 1024: ab_seam_ablation.jsonl), but not through this wait or the stores'
# line count (OLINE) -- so the product keeps vmcnt(0)
SEAMWAIT = [False]
# BEYOND (Gen(beyond=...), the product since round 5): causal, a key tile
# past the wave's diagonal (every score masked) skips QK(t) and the softmax
# of t -- P(t) is set to 0 and the S words its deferred slices read next step
# to -inf -- instead of running them on -inf C operands; PV(t) next step
# still runs on the zeros.  Bitwise equal; causal +0.8-1.4 % at S 4096, +2.3
# % at S 1024 (profiles/r05/flash/ab_beyond.jsonl).  BEYOND 2 also skips
# PV(t-1) when tile t-1 was past the diagonal too (step_idle: only the K/V
# stream and the barrier) and the tail's PV when the last tile is
# (tail_dispatch); 3 adds skipping an idle step's K reads when tile t+1 is
# past the diagonal too (level alone); 4 (the product) adds dropping the
# diagonal tile's all -inf blocks (kb > qb: 24 QK MFMAs) and, in the light
# step after it, its all-zero P(qb 0-1, kp 1) from PV and the row sums (18
# MFMAs): bitwise equal, +0.2-1.3 % (profiles/r05/flash/ab_beyond_diag.jsonl)
BEYOND = [4]
# BALANCED (Gen(causal=True, balanced=True), non-ragged causal): the wave's
# four 16-row q-blocks are interleaved over the block's 256 rows -- q-block qb
# of wave w holds rows 64 qb + 16 w + i instead of 64 w + 16 qb + i -- so
# every wave has one q-block on each of the four diagonal key tiles.  Key tile
# sTD + m (m = 0..3) is then the same work for all four waves: q-blocks qb < m
# are past the diagonal (no QK chains, no softmax, P = 0; the next step drops
# their PV MFMAs), q-block m is the diagonal one (its scores masked by VALU
# against LIMW = 16 w + i - 4 g), q-blocks above it are whole.  In the
# row-contiguous layout the waves reach their diagonal tiles one tile apart
# and wait for each other at every step's barrier (the diagonal group costs
# ~3.7 tile-times per block; balanced ~2.5)
BALANCED = [False]


def RS():
    """row stride between a wave's q-blocks (BALANCED: 64, else 16)"""
    return 64 if BALANCED[0] else 16


def WROW():
    """log2 of the row offset of wave w's first row (BALANCED: 16 w, else 64 w)"""
    return 4 if BALANCED[0] else 6


LIMW = V(206)  # BALANCED: 16 w + i - 4 g (TRI's register: no diagonal C operand)

# NORELOAD (Gen(noreload=True), A/B knob): the block transition does not
# reload argument dwords 0..36 into s56..s92 (no instruction writes them; the
# reload's s_load + lgkmcnt(0) sits on the seam's critical path)
NORELOAD = [False]
# PROPIPE (Gen(propipe=True), non-causal, A/B knob): the first tile's row
# max, mu and P of q-block qb run in the gaps of QK(0)'s later q-blocks
# instead of straight-line after QK(0)
PROPIPE = [False]
# QSPLIT (Gen(qscale=True, qsplit=True), bf16, head dim 64): Q c held as
# two bf16 parts, hi = bf16(q c) and lo = bf16(q c - hi), and every QK chain
# runs both (S = K hi^T + K lo^T, -mu as the first C operand): QSCALE's fma
# saving with the score error of a 16-bit mantissa instead of bf16's 8 --
# twice the QK MFMAs, which only the head-dim-64 form (MFMA busy ~0.5, the
# AGPRs a64-127 free) can pay for
QSPLIT = [False]
# TAILEPI (Gen(tailepi=True), the row-sum-check programs): the epilogue's
# normalise / pack / store of O runs in the gaps of the tail's PV(T), one
# unit per (q-block, d-block pair) as soon as PV(T) has finished those d-blocks
# (l is final before PV(T) under LCHECK; S's registers are dead after the
# tail's check and hold the epilogue's temporaries), instead of after it
TAILEPI = [False]
EP_R = [V(k) for k in range(8)]      # TAILEPI: O values of one unit (in S's registers)
EP_W = V(8, 4)                       # TAILEPI: the unit's packed store words
EP_ROW, EP_LANE = V(12), V(13)


def EP_OOFF(qb):
    return V(16 + qb)


def EP_RCP(qb):
    return V(20 + qb)


# QSEP (Gen(qsep=k), A/B knob): the tail's 16 (D 64: 8) Q loads of the next
# block spaced k MFMA gaps apart, one per gap, instead of packed into the
# first few gaps (0, the round-5 program)
QSEP = [0]
# cache-policy bits of the seam's memory operations (A/B: Gen(o_bits=...,
# q_bits=...), e.g. "nt" / "sc1" / "sc0 sc1"); the product issues them plain
CACHEBITS = {"o": "", "q": ""}


def schedule(mfmas, fills, budget=8, gap_offset=0, lds_gap=LDS_GAP):
    """place fills into the gaps after each MFMA (gap k follows MFMA k);
    returns (instructions, unplaced fills).  Gap indices are shifted by
    gap_offset for the fills' earliest/deadline/dependency bookkeeping, so
    several phases can share one gap numbering."""
    out = []
    for k0, m in enumerate(mfmas):
        k = k0 + gap_offset
        out.append(m)
        used, trans, lds = 0, 0, 0
        for f in fills:
            if f.gap is not None or f.earliest > k:
                continue
            if any(d.gap is None or d.gap + f.sep > k for d in f.deps):
                continue
            forced = f.deadline is not None and f.deadline <= k
            if not forced:
                if f.trans and trans >= TRANS_PER_GAP[0]:
                    continue
                if f.lds and lds + f.lds > lds_gap:
                    continue
                if used + f.cost > budget and not (used == 0 and f.cost > budget) and \
                        not (f.cost <= 2 and used + f.cost <= budget + 2):
                    continue
            f.gap = k
            out.extend(f.ins)
            used += f.cost
            lds += f.lds
            trans += int(bool(f.trans))
    for f in fills:
        if f.hard and (f.gap is None or f.gap > f.deadline):
            raise RuntimeError(f"fill {f.tag} {f.ins[0]} missed its hard deadline {f.deadline} (gap {f.gap})")
    left = [f for f in fills if f.gap is None]
    return out, left


def chain(ins_list, earliest=0, cost=None):
    """fills that keep program order (each depends on the one before)"""
    out, prev = [], None
    for ins in ins_list:
        c = cost(ins) if cost else (4 if ins.op.startswith("v_") else 2)
        f = Fill(ins, c, deps=[prev] if prev else [], sep=0, earliest=earliest, tag="chain")
        out.append(f)
        prev = f
    return out


def drain(fills, k):
    """emit unplaced fills in dependency order after the last gap k"""
    out = []
    pending = [f for f in fills if f.gap is None]
    while pending:
        progressed = False
        for f in pending:
            if all(d.gap is not None for d in f.deps):
                f.gap = k
                out.extend(f.ins)
                progressed = True
        pending = [f for f in pending if f.gap is None]
        assert progressed, "fill dependency cycle"
    return out


# ---------------------------------------------------------------- pieces


def NQK():
    """MFMAs per QK chain: one per 32-wide d slice, two with QSPLIT (Q hi and lo)"""
    return NDS() * (2 if QSPLIT[0] else 1)


def QL_(qb, ds):
    """QSPLIT (head dim 64): the low bf16 part of Q c, a64.. (O uses a0-63)"""
    return A(64 + 4 * (4 * qb + ds), 4)


def qk_mfmas(mask=None, muc=False):
    """QK^T of one tile, q-block major.  mask (causal): the C operand of each
    chain's first MFMA -- 'diag' (the wave's diagonal tile: 0 below the
    diagonal blocks, the triangular pattern on them, -inf above), 'beyond'
    (every score -inf: P = 0)"""
    def c0(kb, qb):
        if mask == "beyond" or (mask == "diag" and kb > qb):
            return NINF
        if mask == "diag" and kb == qb:
            return TRIMU(qb) if muc else TRI
        return MUC(qb) if muc else 0
    if QSPLIT[0]:
        return [mfma(S_(kb, qb), K_(kb, j >> 1), (QL_ if j & 1 else Q_)(qb, j >> 1), S_(kb, qb) if j else c0(kb, qb))
                for qb in range(4) for j in range(NQK()) for kb in range(4)]
    return [mfma(S_(kb, qb), K_(kb, ds), Q_(qb, ds), S_(kb, qb) if ds else c0(kb, qb))
            for qb in range(4) for ds in range(NDS()) for kb in range(4)]


def qk_done_gap(kb, qb):
    """QK phase gap after which S(kb, qb) is complete"""
    return 4 * NQK() * qb + 4 * (NQK() - 1) + kb


def qk_first(kb, qb):
    """QK phase index of the MFMA that starts S(kb, qb) (it overwrites S)"""
    return 4 * NQK() * qb + kb


def rowsum_mfmas(X, ones=None):
    """l(qb) += 1^T P(X, qb, kp) for the tile in P state X (all-ones A operand)"""
    ones = ONES if ones is None else ones
    return [mfma(L_(qb), ones, P_(X, qb, kp), L_(qb)) for qb in range(4) for kp in range(2)]


def qk_with_rowsums(mask=None, muc=False, Xr=None):
    """LCHECK: QK(t) with the row sums of tile t-1 (state Xr) interleaved
    into its last 8 MFMAs (after every deferred slice of t-1 is due, so the
    check right after the phase reads complete sums); returns the MFMA list,
    done(kb, qb) -> the gap after which S(kb, qb) is complete and first(kb,
    qb) -> the index of the MFMA that starts S(kb, qb)"""
    qk = qk_mfmas(mask, muc)
    n = len(qk)
    if Xr is None:
        return qk, lambda kb, qb: qk_done_gap(kb, qb), lambda kb, qb: qk_first(kb, qb)
    if "rsum" in ABL:  # timing only: no row-sum MFMAs
        return qk, lambda kb, qb: qk_done_gap(kb, qb), lambda kb, qb: qk_first(kb, qb)
    rs = rowsum_mfmas(Xr)
    out, pos = qk[:n - 8], {}
    for j in range(n - 8, n):
        out += [rs[j - (n - 8)], qk[j]]
    for j in range(n):
        pos[j] = j if j < n - 8 else 2 * j - (n - 9)
    # the deferred slices of t-1 (q-block 3) are due before their S blocks are
    # overwritten -- before the row sums of q-block 3 (rs[6], rs[7]) read them
    assert pos[qk_first(3, 3)] - 1 < out.index(rs[6])
    return out, lambda kb, qb: pos[qk_done_gap(kb, qb)], lambda kb, qb: pos[qk_first(kb, qb)]


def pv_mfmas(X):
    out = []
    per = 8 // NDB()  # P-bit check: the 8 row sums spread over the d-blocks
    for db in range(NDB()):
        for kp in range(2):
            for qb in range(4):
                out.append(mfma(O_(db, qb), VF(db % NVF, kp), P_(X, qb, kp), O_(db, qb)))
        if not LCHECK[0]:
            for r in range(per * db, per * db + per):
                qb, kp = r % 4, r // 4
                out.append(mfma(L_(qb), ONES, P_(X, qb, kp), L_(qb)))
    return out


def pv_first_gap(db):
    return (8 if LCHECK[0] else 8 + 8 // NDB()) * db


def vbuf_free(db):
    """earliest PV gap for d-block db's V^T reads: its buffer (db mod 3) is
    d-block db-3's, free one MFMA after that block's last use"""
    if GEOM["hd"] == 128:
        return pv_first_gap(db - 3) + 9  # (the D = 128 schedules as built in round 4)
    return pv_first_gap(db - 3) + pv_first_gap(1) + 1


def k_reads():
    return [I("ds_read_b128", K_(kb, ds), VKA, mods=f"offset:{512 * (ds & 1) + 2048 * kb + 8192 * (ds >> 1)}")
            for ds in range(NDS()) for kb in range(4)]


def v_reads(db):
    b = db % NVF
    return [I("ds_read_b64_tr_b16", VFh(b, kp, h), VVA,
              mods=f"offset:{256 * (db & 1) + 512 * ((db >> 1) & 1) + 2048 * h + 4096 * kp + 8192 * (db >> 2)}")
            for kp in range(2) for h in range(2)]


def slice_list():
    """softmax slices of one tile: (qb, kb, hh) in stream order"""
    return [(qb, kb, hh) for qb in range(4) for kb in range(4) for hh in range(2)]


def softmax_fills(X, slices, earliest_of, deadline_of=None, ytag=0, prev_cv=None, extra_deps=None):
    """fills for the given slices of the tile in P state X: per slice two
    v_fma_f32 (s * c - mu), two v_exp_f32, one v_cvt_pk_bf16_f32; one
    v_or3_b32 per two slices into ACC(X).  Temporaries Y rotate over 8 slots
    (a slot is reused once its cvt has issued)."""
    fills, cvs, groups = [], [], []
    last_or = None
    slot_cv = dict(prev_cv or {})
    for n, (qb, kb, hh) in enumerate(slices):
        slot = (ytag + n) % (NY // 2)
        y0, y1 = Y(2 * slot), Y(2 * slot + 1)
        s = S_(kb, qb)
        deps = [slot_cv[slot]] if slot in slot_cv else []
        if extra_deps is not None:  # (the ragged causal mask of S(kb, qb))
            deps = deps + extra_deps(qb, kb)
        ea, dl = earliest_of(qb, kb), deadline_of(qb, kb) if deadline_of else None
        f0 = Fill(I("v_fma_f32", y0, s[2 * hh], sC, Neg(MU(qb))), 4, deps=deps, sep=0, earliest=ea, deadline=dl,
                  tag="fma", hard=dl is not None)
        f1 = Fill(I("v_fma_f32", y1, s[2 * hh + 1], sC, Neg(MU(qb))), 4, deps=deps, sep=0, earliest=ea,
                  deadline=dl, tag="fma", hard=dl is not None)
        if QSCALE[0]:  # P = bf16(exp2(S)), S already c s - mu: in place, no temporaries
            dle = None if dl is None else dl - 1
            xd = extra_deps(qb, kb) if extra_deps is not None else []  # (a VALU mask of S(kb, qb) first)
            xm = "clamp" if LCHECK[0] else ""
            e0 = Fill(I("v_exp_f32", s[2 * hh], s[2 * hh], mods=xm), 8, trans=True, deps=xd, sep=0, earliest=ea,
                      deadline=dle, tag="exp", hard=dl is not None)
            e1 = Fill(I("v_exp_f32", s[2 * hh + 1], s[2 * hh + 1], mods=xm), 8, trans=True, deps=xd, sep=0,
                      earliest=ea, deadline=dle, tag="exp", hard=dl is not None)
            f0 = f1 = None
            y0, y1 = s[2 * hh], s[2 * hh + 1]
        elif "exp" in ABL:
            e0 = Fill(I("v_mov_b32", y0, y0), 4, deps=[f0], sep=1, tag="exp")
            e1 = Fill(I("v_mov_b32", y1, y1), 4, deps=[f1], sep=1, tag="exp")
        elif "fma" in ABL:  # exp straight from S (no s * c - mu)
            e0 = Fill(I("v_exp_f32", y0, s[2 * hh]), 8, trans=True, deps=deps, sep=0, earliest=ea, deadline=dl,
                      tag="exp", hard=dl is not None)
            e1 = Fill(I("v_exp_f32", y1, s[2 * hh + 1]), 8, trans=True, deps=deps, sep=0, earliest=ea, deadline=dl,
                      tag="exp", hard=dl is not None)
            f0 = f1 = None
        else:
            xm = "clamp" if LCHECK[0] else ""
            e0 = Fill(I("v_exp_f32", y0, y0, mods=xm), 8, trans=True, deps=[f0], sep=1, tag="exp")
            e1 = Fill(I("v_exp_f32", y1, y1, mods=xm), 8, trans=True, deps=[f1], sep=1, tag="exp")
        fm = f1
        w = P_(X, qb, kb >> 1)[2 * (kb & 1) + hh]
        cdeps = [e0, e1]
        rsv = []
        if "rsumv" in ABL:  # timing only: the row sums as VALU adds of the fp32 P (no row-sum MFMAs)
            a0 = Fill(I("v_add_f32", L_(qb)[0], L_(qb)[0], y0), 4, deps=[e0], sep=1, tag="rsumv")
            a1 = Fill(I("v_add_f32", L_(qb)[0], L_(qb)[0], y1), 4, deps=[a0, e1], sep=1, tag="rsumv")
            rsv, cdeps = [a0, a1], [e0, e1, a1]
        cv = Fill(I(DT["cvt"], w, y0, y1), 4, deps=cdeps, sep=1, tag="cvt",
                  deadline=dl if QSCALE[0] else None, hard=QSCALE[0] and dl is not None)
        slot_cv[slot] = cv
        grp = [f for f in (f0, f1, e0, e1, *rsv, cv) if f is not None]
        fills += grp
        groups.append(grp)
        cvs.append((cv, w))
        if len(cvs) == 2 and ("or" in ABL or LCHECK[0]):  # LCHECK / timing-only "or": no defer-max bits
            cvs = []
        if len(cvs) == 2:
            (c0, w0), (c1, w1) = cvs
            od = [c0, c1] + ([last_or] if last_or else [])
            last_or = Fill(I("v_or3_b32", ACC(X), ACC(X), w0, w1), 4, deps=od, sep=1, tag="or")
            fills.append(last_or)
            cvs = []
    assert not cvs
    softmax_fills.groups = groups  # per-slice fills of the last call
    return fills, slot_cv, last_or


# ---------------------------------------------------------------- SALU helpers


def div_magic(out, x, mag, shpos):
    """out = x / d for x < 2^31 (mag and the shift from the host:
    Granlund-Montgomery with N = 31): ((x * mag) >> 31) >> sh, sh at bit
    shpos of the packed "shifts" argument"""
    sh = ARG(AI["shifts"])
    c = [I("s_mul_hi_u32", sT6, x, mag), I("s_mul_i32", sT7, x, mag), I("s_lshl_b32", sT6, sT6, 1),
         I("s_lshr_b32", sT7, sT7, 31), I("s_or_b32", sT6, sT6, sT7)]
    if shpos:
        c += [I("s_lshr_b32", sT7, sh, shpos)]
        sh = sT7
    return c + [I("s_lshr_b32", out, sT6, sh)]


def mad64(out, base, x, st, y, st2):
    """out = base + x * st + y * st2 (64-bit; x, y 32-bit unsigned)"""
    c = []
    for (m, stv, b) in ((x, st, base), (y, st2, out)):
        c += [I("s_mul_i32", sT6, m, stv[0]), I("s_mul_hi_u32", sT7, m, stv[0]),
              I("s_add_u32", out[0], b[0], sT6), I("s_addc_u32", out[1], b[1], sT7),
              I("s_mul_i32", sT6, m, stv[1]), I("s_add_u32", out[1], out[1], sT6)]
    return c


def block_params(sx, causal=False, uid=0, rev=0):
    """block index sx -> sNQH, sNOH (Q / O heads), sNQ0 (the wave's first
    row), sT8 (the block's key-tile count), the K head in sT0:sT1 (s52:s53)
    and the V head in s96:s97; needs the arguments in s56..s95.  sx is read
    by the first instructions only (it may be a scratch register the rest
    overwrites).

    Walk (non-causal): each XCD walks a contiguous range of blocks (the
    xcd_remap of pli_common.h), lb = x * (nb >> 3) + min(x, nb & 7) + (l >> 3).
    Causal (the cw argument's low byte): 1 = the pair walk of attn_fwd_v12
    (workgroup i of XCD x runs query heights QB-1-a then a of one head, so
    every workgroup does the same triangular work and the QB/2 workgroups of a
    head share its K/V in L2); 2 = the remap walk, heaviest block of a head
    first (one block per workgroup)."""
    NB, QB, CW = ARG(AI["nblocks"]), ARG(AI["qblocks"]), ARG(AI["cw"])
    c = []
    pair, done = f"v13_pair_{uid}_%=", f"v13_walked_{uid}_%="
    if causal:
        c += [I("s_and_b32", sT6, CW, 0xFF), I("s_cmp_eq_u32", sT6, 1), I("s_cbranch_scc1", pair)]
    # the remap walk: lb in sT4, bh in sT5, qblk in sT2
    c += [I("s_lshr_b32", sT4, NB, 3), I("s_and_b32", sT5, NB, 7), I("s_cmp_lt_u32", NB, 8),
          I("s_cselect_b32", sT4, 0, sT4), I("s_cselect_b32", sT5, 8, sT5),
          I("s_and_b32", sT2, sx, 7), I("s_lshr_b32", sT3, sx, 3), I("s_mul_i32", sT4, sT2, sT4),
          I("s_min_u32", sT2, sT2, sT5), I("s_add_u32", sT4, sT4, sT2), I("s_add_u32", sT4, sT4, sT3)]
    c += div_magic(sT5, sT4, ARG(AI["magq"]), 0)
    c += [I("s_mul_i32", sT2, sT5, QB), I("s_sub_u32", sT2, sT4, sT2)]
    if causal:
        # heaviest first: query height QB-1-r
        c += [I("s_sub_u32", sT3, QB, 1), I("s_sub_u32", sT2, sT3, sT2)] + \
            ([I("s_mov_b32", sRET, 0)] if rev else []) + [I("s_branch", done)]
        # the pair walk: x = l & 7, l8 = l >> 3, j = l8 >> lgG8, wg = l8 mod G8,
        # wgq = wg >> lghq, a = wg mod hq, bh = x hx + wgq + per (j >> 1),
        # qblk = j odd ? a : QB-1-a
        c += [label(pair),
              I("s_and_b32", sT2, sx, 7), I("s_lshr_b32", sT3, sx, 3),
              I("s_lshr_b32", sT6, CW, 8), I("s_and_b32", sT6, sT6, 0xFF),
              I("s_lshr_b32", sT4, sT3, sT6), I("s_lshl_b32", sT5, sT4, sT6), I("s_sub_u32", sT5, sT3, sT5),
              *([I("s_and_b32", sT6, ARG(AI["hx"]), 0xFFFFFF), I("s_mul_i32", sT2, sT2, sT6)] if RAGGED[0] else
                [I("s_mul_i32", sT2, sT2, ARG(AI["hx"]))]),
              I("s_lshr_b32", sT6, CW, 16), I("s_and_b32", sT6, sT6, 0xFF),
              I("s_lshr_b32", sT3, sT5, sT6), I("s_lshl_b32", sT7, sT3, sT6), I("s_sub_u32", sT5, sT5, sT7),
              I("s_add_u32", sT2, sT2, sT3),
              I("s_lshr_b32", sT6, CW, 24), I("s_lshr_b32", sT7, sT4, 1), I("s_mul_i32", sT7, sT7, sT6),
              I("s_add_u32", sT2, sT2, sT7),
              I("s_sub_u32", sT6, QB, 1), I("s_sub_u32", sT6, sT6, sT5),
              I("s_and_b32", sT4, sT4, 1)] + ([I("s_cselect_b32", sRET, 1, 0)] if rev else []) + [
              I("s_cselect_b32", sT4, sT6, sT5) if SHORTFIRST[0] else I("s_cselect_b32", sT4, sT5, sT6),
              I("s_mov_b32", sT5, sT2), I("s_mov_b32", sT2, sT4), label(done)]
        # key tiles the block's last row sees: min(nt, 4 qblk + 4 + off / 64)
        c += [I("s_lshl_b32", sT8, sT2, 2), I("s_add_u32", sT8, sT8, 4), I("s_add_u32", sT8, sT8, sOFFT),
              I("s_min_u32", sT8, sT8, ARG(AI["nt"]))]
        if rev:  # reversed order (the second block of a pair) needs 4 tiles
            c += [I("s_cmp_ge_u32", sT8, 4), I("s_cselect_b32", sRET, sRET, 0)]
    else:
        c += [I("s_mov_b32", sT8, ARG(AI["nt"]))]
    # q0 = qblk * 256 + 64 * wave (BALANCED: + 16 * wave)
    c += [I("s_lshl_b32", sT2, sT2, 8), I("s_lshr_b32", sT3, sWKOFF, WSH() - WROW()), I("s_add_u32", sNQ0, sT2, sT3)]
    # b = bh / H, h = bh - b * H, hk = h / group
    c += div_magic(sT4, sT5, ARG(AI["magh"]), 5)
    c += [I("s_lshr_b32", sT2, ARG(AI["shifts"]), 16), I("s_mul_i32", sT2, sT4, sT2), I("s_sub_u32", sT3, sT5, sT2)]
    c += div_magic(sT5, sT3, ARG(AI["magg"]), 10)
    # heads: b in sT4, h in sT3, hk in sT5
    c += mad64(sNQH, ARG(AI["q"], 2), sT4, ARG(AI["qb"], 2), sT3, ARG(AI["qh"], 2))
    c += mad64(sNOH, ARG(AI["o"], 2), sT4, ARG(AI["ob"], 2), sT3, ARG(AI["oh"], 2))
    c += mad64(S(sT0.i, 2), ARG(AI["k"], 2), sT4, ARG(AI["kb"], 2), sT5, ARG(AI["kh"], 2))
    c += mad64(S(sT2.i, 2), ARG(AI["v"], 2), sT4, ARG(AI["vb"], 2), sT5, ARG(AI["vh"], 2))
    if causal and rev:
        # reversed block: the stream starts at tile nt - 4 (see Gen.tile_of);
        # the order rides in bit 16 of the tile count
        fwd = f"v13_fwd_{uid}_%="
        c += [I("s_cmp_eq_u32", sRET, 0), I("s_cbranch_scc1", fwd),
              I("s_sub_u32", sT4, sT8, 4),
              I("s_mul_i32", sT5, sT4, sTBK), I("s_add_u32", sT0, sT0, sT5), I("s_addc_u32", sT1, sT1, 0),
              I("s_mul_i32", sT5, sT4, sTBV), I("s_add_u32", sT2, sT2, sT5), I("s_addc_u32", sT3, sT3, 0),
              I("s_or_b32", sT8, sT8, 0x10000), label(fwd)]
    return c  # K head in sT0:sT1, V head in sT2:sT3, nt in sT8 (causal: | reversed << 16)


def load_args():
    return [I("s_load_dwordx16", ARG(0, 16), sKA, 0), I("s_load_dwordx16", ARG(16, 16), sKA, 64),
            I("s_load_dwordx4", ARG(32, 4), sKA, 128), I("s_load_dword", ARG(36), sKA, 144),
            I("s_waitcnt", "lgkmcnt(0)")]


# ---------------------------------------------------------------- DMA


def dma_fills(slot_reg, earliest0=2, spacing=6, rev=False):
    """the NPW() LDS-DMA pieces (8 at D = 128, 4 at D = 64) of the stream's
    next tile into slot slot_reg (K pieces NPW/2 w .. of the K image, V
    pieces of the V image; one M0 write per half), the stream switch before
    and the advance after"""
    swi = [I("s_cmp_eq_u32", sDIDX, sDNT), I("s_cselect_b64", sDK, sNXK, sDK),
           I("s_cselect_b64", sDV, sNXV, sDV), I("s_cselect_b32", sDIDX, sNXIDX, sDIDX),
           I("s_cselect_b32", sDNT, sNXNT, sDNT)]
    cost = 2
    if RAGGED[0] and rev:
        # causal: the last key tile streams from key Nk - 64 (P0 keys back);
        # sT3 keeps the shift until the advance undoes it
        swi += p0_to(sT3, True) + is_last_tile() + [I("s_cselect_b32", sT3, sT3, 0)] + rag_shift(sDK, sDV, True)
        cost = 8
    sw = Fill(swi, cost, earliest=earliest0 - 1, tag="dmasw")
    fills = [sw]
    prev = sw
    half = NPW() // 2
    for j in range(NPW()):
        ins = []
        if j == 0:
            ins.append(I("s_add_u32", M0, slot_reg, sWKOFF))
        if j == half:
            ins += [I("s_add_u32", M0, slot_reg, sWKOFF), I("s_add_u32", M0, M0, VIMG)]
        src = sDK if j < half else sDV
        off = DMAK(j) if j < half else DMAV(j - half)
        if "dma" not in ABL:
            ins.append(I("global_load_lds_dwordx4", off, src, mods=f"offset:{1024 * (j % half)}"))
        f = Fill(ins, DMA_COST, deps=[prev], sep=1 if j else 0, earliest=earliest0 + spacing * j, tag="dma")
        fills.append(f)
        prev = f
    if rev:
        # causal: sDIDX bit 16 = the streamed block's order.  Reversed, the
        # positions 0..3 are tiles nt-4 .. nt-1 and position p >= 4 is tile
        # nt-1-p: the step into position p is +1, -4 (p = 4) or -1 tiles
        undo = rag_shift(sDK, sDV, False) if RAGGED[0] else []
        adv = Fill(undo + [I("s_add_u32", sDIDX, sDIDX, 1), I("s_and_b32", sT2, sDIDX, 0xFFFF),
                    I("s_cmp_eq_u32", sT2, 4), I("s_cselect_b32", sT3, -4, -1),
                    I("s_cmp_lt_u32", sT2, 4), I("s_cselect_b32", sT3, 1, sT3),
                    I("s_bitcmp1_b32", sDIDX, 16), I("s_cselect_b32", sT3, sT3, 1),
                    I("s_mul_i32", sT2, sT3, sTBK), I("s_ashr_i32", sT4, sT2, 31),
                    I("s_add_u32", sDK[0], sDK[0], sT2), I("s_addc_u32", sDK[1], sDK[1], sT4),
                    I("s_mul_i32", sT2, sT3, sTBV), I("s_ashr_i32", sT4, sT2, 31),
                    I("s_add_u32", sDV[0], sDV[0], sT2), I("s_addc_u32", sDV[1], sDV[1], sT4)],
                   8, deps=[prev], sep=0, tag="dmaadv")
    else:
        ains = [I("s_add_u32", sDK[0], sDK[0], sTBK), I("s_addc_u32", sDK[1], sDK[1], 0),
                I("s_add_u32", sDV[0], sDV[0], sTBV), I("s_addc_u32", sDV[1], sDV[1], 0),
                I("s_add_u32", sDIDX, sDIDX, 1)]
        cost = 2
        if RAGGED[0]:
            # the stream's next tile is the last one: P0 keys back
            ains += [I("s_sub_u32", sT2, sDNT, 1), I("s_cmp_eq_u32", sDIDX, sT2)] + rag_back(sDK, sDV)
            cost = 6
        adv = Fill(ains, cost, deps=[prev], sep=0, tag="dmaadv")
    fills.append(adv)
    return fills


def rag_back(k, v):
    """RAGGED: with SCC set, the K / V stream pointers k, v move back by P0
    keys (P0 tbk / 64 and P0 tbv / 64 bytes); uses sT2, sT3"""
    c = [I("s_cselect_b32", sT3, ARG(AI["cw"]), 0)]
    for (ptr, tb) in ((k, sTBK), (v, sTBV)):
        c += [I("s_mul_i32", sT2, sT3, tb), I("s_lshr_b32", sT2, sT2, 6),
              I("s_sub_u32", ptr[0], ptr[0], sT2), I("s_subb_u32", ptr[1], ptr[1], 0)]
    return c


def p_mask(X):
    """RAGGED: the last tile's P (state X) with its first P0 keys zeroed"""
    return [I("v_and_b32", P_(X, qb, kb >> 1)[2 * (kb & 1) + hh], P_(X, qb, kb >> 1)[2 * (kb & 1) + hh], PM(kb, hh))
            for qb in range(4) for kb in range(4) for hh in range(2)]


def dma_now(slot_reg, rev=False):
    """the same as straight-line code (prologue of the first block)"""
    out = []
    for f in dma_fills(slot_reg, rev=rev):
        out += f.ins
    return out


def rotate_slots():
    """slot(t-1) <- slot(t) <- slot(t+1) <- slot(t+2) <- slot(t+2) + 1"""
    return [I("s_mov_b32", sSM1, sS0), I("s_mov_b32", sS0, sSP1), I("s_mov_b32", sSP1, sSP2),
            I("s_add_u32", sSP2, sSP2, SLOT), I("s_cmp_ge_u32", sSP2, SLOT * NSLOT),
            I("s_cselect_b32", sSP2, 0, sSP2)]


# ---------------------------------------------------------------- softmax bits


def row_max(qb, m, t1, t2):
    """m = max over the row (query 16qb + i) of S(., qb): 16 values per lane,
    then across the four lanes l, l^16, l^32, l^48"""
    c = []
    vals = [S_(kb, qb)[r] for kb in range(4) for r in range(4)]
    c.append(I("v_max3_f32", m, vals[0], vals[1], vals[2]))
    k = 3
    while k + 1 < 16:
        c.append(I("v_max3_f32", m, m, vals[k], vals[k + 1]))
        k += 2
    c.append(I("v_max_f32", m, m, vals[15]))
    for sw in ("v_permlane32_swap_b32", "v_permlane16_swap_b32"):
        c += [I("v_mov_b32", t1, m), I("v_mov_b32", t2, m), I(sw, t1, t2), I("v_max_f32", m, t1, t2)]
    return c


def exps_all(X, also_or=False, shifted=False):
    """every P of the tile in S with the current mu (straight line);
    QSCALE: S = c s (C operand 0) unless shifted (S = c s - mu already)"""
    c = []
    for n, (qb, kb, hh) in enumerate(slice_list()):
        y0, y1 = T(0 + 2 * (n % 8)), T(1 + 2 * (n % 8))
        s = S_(kb, qb)
        w = P_(X, qb, kb >> 1)[2 * (kb & 1) + hh]
        xm = "clamp" if LCHECK[0] else ""
        if QSCALE[0] and shifted:
            c += [I("v_exp_f32", y0, s[2 * hh], mods=xm), I("v_exp_f32", y1, s[2 * hh + 1], mods=xm)]
        elif QSCALE[0]:
            # S = c s - mu written back in place: the next step's deferred
            # slices of this tile exp S in place and expect it shifted
            c += [I("v_sub_f32", s[2 * hh], s[2 * hh], MU(qb)), I("v_sub_f32", s[2 * hh + 1], s[2 * hh + 1], MU(qb)),
                  I("v_exp_f32", y0, s[2 * hh], mods=xm), I("v_exp_f32", y1, s[2 * hh + 1], mods=xm)]
        else:
            c += [I("v_fma_f32", y0, s[2 * hh], sC, Neg(MU(qb))), I("v_fma_f32", y1, s[2 * hh + 1], sC, Neg(MU(qb))),
                  I("v_exp_f32", y0, y0, mods=xm), I("v_exp_f32", y1, y1, mods=xm)]
        c += [I(DT["cvt"], w, y0, y1)]
        if also_or and not LCHECK[0]:
            c.append(I("v_or_b32", ACC(X), ACC(X), w))
    return c


def p0_to(dst, causal):
    """RAGGED: dst = P0 = 64 - Nk % 64 (the non-causal program has it in
    the cw argument, the causal one -- whose walk uses cw -- in the top byte
    of hx)"""
    if causal:
        return [I("s_lshr_b32", dst, ARG(AI["hx"]), 24)]
    return [I("s_mov_b32", dst, ARG(AI["cw"]))]


def qshift(dst, tmp):
    """causal: dst = s = (Nk - Nq) & 63 = (-(Nq + P0)) & 63, the virtual-row
    shift that puts the bottom-right diagonal on 64-key tile boundaries: row q
    is processed as q + s of Nq + s rows (the launcher sizes the blocks and
    the diagonal tile offset for Nq + s)"""
    c = [I("s_sub_u32", dst, 0, ARG(AI["nq"]))]
    if RAGGED[0]:
        c += p0_to(tmp, True) + [I("s_sub_u32", dst, dst, tmp)]
    return c + [I("s_and_b32", dst, dst, 63)]


def is_last_tile():
    """RAGGED causal: SCC = the stream's current position is key tile NT - 1
    (forward: position NT - 1; reversed: position 3 of a block whose tile
    count is NT); uses sT4 .. sT7"""
    return [I("s_and_b32", sT4, sDIDX, 0xFFFF), I("s_and_b32", sT5, sDNT, 0xFFFF),
            I("s_cmp_eq_u32", sT5, ARG(AI["nt"])), I("s_cselect_b32", sT7, 3, 0xFFFF),
            I("s_sub_u32", sT6, ARG(AI["nt"]), 1), I("s_bitcmp1_b32", sDIDX, 16),
            I("s_cselect_b32", sT6, sT7, sT6), I("s_cmp_eq_u32", sT4, sT6)]


def rag_shift(k, v, sub):
    """RAGGED causal: K / V stream pointers k, v moved back (sub) or forward
    by sT3 keys (sT3 = P0 or 0); uses sT2"""
    c = []
    for (ptr, tb) in ((k, sTBK), (v, sTBV)):
        c += [I("s_mul_i32", sT2, sT3, tb), I("s_lshr_b32", sT2, sT2, 6)]
        c += ([I("s_sub_u32", ptr[0], ptr[0], sT2), I("s_subb_u32", ptr[1], ptr[1], 0)] if sub else
              [I("s_add_u32", ptr[0], ptr[0], sT2), I("s_addc_u32", ptr[1], ptr[1], 0)])
    return c


def mask_tile(tile):
    """causal, straight line (prologue and rare path): scores of the tile
    whose index is in SGPR `tile` with key > row + off set to -inf.  Lane
    (g, i) holds key 64 tile + 16 kb + 4 g + r of row q0 + RS qb + i (RS 16,
    BALANCED 64): masked iff 16 kb - RS qb + r > lim = q0 + 64 (off - tile)
    + i - 4 g"""
    lim = T(37)
    c = [I("s_sub_u32", sT7, sOFFT, tile), I("s_lshl_b32", sT7, sT7, 6), I("s_add_u32", sT7, sT7, sCQ0),
         I("v_add_u32", lim, sT7, VI), I("v_lshlrev_b32", T(36), 2, VG), I("v_sub_u32", lim, lim, T(36))]
    for qb in range(4):
        for kb in range(4):
            for r in range(4):
                c += [I("v_cmp_gt_i32_e32", VCC, 16 * kb - RS() * qb + r, lim),
                      I("v_cndmask_b32_e32", S_(kb, qb)[r], S_(kb, qb)[r], NINF[0], VCC)]
    return c


def grp_block(kb, qb):
    """BALANCED: S(kb, qb) of the q-block on its diagonal tile masked to -inf
    where the key is past the row: key 16 kb + 4 g + r of the tile against
    row 16 w + i of the q-block's 64-row group (masked iff 16 kb + r > LIMW)"""
    c = []
    for r in range(4):
        c += [I("v_cmp_gt_i32_e32", VCC, 16 * kb + r, LIMW),
              I("v_cndmask_b32_e32", S_(kb, qb)[r], S_(kb, qb)[r], NINF[0], VCC)]
    return c


def rag_setup():
    """RAGGED causal, key tile NT - 1 (keys Nk - 64 + p at position p):
    T(26) = 4 g - P0, T(27) = i + 64 (sTD - NT + 1) (sTD >= NT - 1 here);
    uses sT0, sT1"""
    return p0_to(sT1, True) + [
        I("s_sub_u32", sT0, sTD, ARG(AI["nt"])), I("s_add_u32", sT0, sT0, 1), I("s_lshl_b32", sT0, sT0, 6),
        I("v_lshlrev_b32", T(26), 2, VG), I("v_subrev_u32", T(26), sT1, T(26)), I("v_add_u32", T(27), sT0, VI)]


def rag_block(kb, qb):
    """RAGGED causal: S(kb, qb) of key tile NT - 1 masked to -inf where the
    key is already counted (p < P0) or past the row's diagonal: with x =
    p - P0 and y = (row's last visible key) - (Nk - 64) - P0, masked iff x >u
    y (x wraps for p < P0)"""
    c = [I("v_add_u32", T(29), 16 * qb, T(27))]
    for r in range(4):
        c += [I("v_add_u32", T(28), 16 * kb + r, T(26)), I("v_cmp_gt_u32_e32", VCC, T(28), T(29)),
              I("v_cndmask_b32_e32", S_(kb, qb)[r], S_(kb, qb)[r], NINF[0], VCC)]
    return c


# ---------------------------------------------------------------- program


class Gen:
    """the whole kernel program (list of Ins); causal=True builds the
    bottom-right-masked kernel (attn_fwd_v13c)"""

    def __init__(self, ndef=4, budget=8, dma_spacing=6, tag="%=", stamp=False, causal=False, abl=(), dma_cost=8,
                 rev=True, qscale=False, dma_pv=0, dma_pv_spacing=16, budget_pv=None, lcheck=None, dtype="bf16",
                 hd=128, short_first=False, ragged=False, oline=False, seam_wait=False, o_bits=0, q_bits=0,
                 beyond=4, qsep=0, balanced=False, noreload=False, propipe=False, trans=1, qsplit=False,
                 tailepi=False, pad=0):
        global DMA_COST
        TAILEPI[0] = int(tailepi)  # 1: one fill per unit, 2: four (reads + muls x 2, pack, store)
        # (head dim 64 only: the AGPRs for Q lo; other forms ignore it)
        QSPLIT[0] = bool(qsplit) and bool(qscale) and dtype == "bf16" and hd == 64
        TRANS_PER_GAP[0] = int(trans)
        PROPIPE[0] = bool(propipe)
        NORELOAD[0] = bool(noreload)
        QSEP[0] = int(qsep)
        # (balanced applies to the non-ragged causal programs; the others ignore it)
        BALANCED[0] = bool(balanced) and causal and not ragged
        OLINE[0] = bool(oline)
        BEYOND[0] = int(beyond)
        bits = {0: "", 1: "nt", 2: "sc1", 3: "sc0 sc1", 4: "sc0 sc1 nt"}
        CACHEBITS["o"], CACHEBITS["q"] = bits[o_bits], bits[q_bits]
        SEAMWAIT[0] = bool(seam_wait)
        assert not (ragged and causal and not rev), "ragged causal: the pair-walk program (rev=True)"
        RAGGED[0] = bool(ragged)
        SHORTFIRST[0] = bool(short_first)
        assert not (short_first and rev and causal), "short_first streams both blocks forward (rev=False)"
        assert hd in (64, 128)
        GEOM["hd"] = hd
        # fp16: P keeps the bit check (P < 2: bit 14 of an fp16 half too) --
        # the l >= 1 test needs muoff >> log2 Nk, which fp16 P (normal down to
        # 2^-14, zero below 2^-24) cannot give; the launcher passes muoff 4
        DT.clear()
        DT.update(DTYPES[dtype])
        if lcheck is None:
            lcheck = dtype == "bf16"
        assert not (dtype == "f16" and lcheck), "fp16 runs the P-bit check"
        QSCALE[0] = bool(qscale)
        LCHECK[0] = bool(lcheck)
        TAILEPI[0] = TAILEPI[0] if LCHECK[0] and not OLINE[0] else 0
        # causal: the second block of each pair streams its tiles in the
        # reversed order of tile_of (its 8 workgroups then read every K/V
        # tile at the same time)
        self.rev = causal and rev
        # dma_pv > 0: the V half of each tile's DMA in the PV phase from gap
        # dma_pv on, dma_pv_spacing apart (A/B knob; 0 = all in the QK phase)
        self.dma_pv, self.dma_pv_spacing = dma_pv, dma_pv_spacing
        self.budget_pv = budget if budget_pv is None else budget_pv  # the steps' PV-phase issue budget
        assert not (dma_pv and GEOM["hd"] != 128), "dma_pv: D = 128 only"
        self.ndef, self.budget, self.dma_spacing, self.tag = ndef, budget, dma_spacing, tag
        ABL.clear()
        ABL.update(abl)
        DMA_COST = dma_cost
        self.stamp = stamp  # diagnostic build: s_memtime / s_memrealtime at entry and exit
        self.pad = int(pad)  # A/B knob: s_nop 0 before the step loop (moves the loop's code address)
        self.causal = causal
        self.prog = []
        self.sites = []  # (site id, rare block name, return label)
        self.uid = 0

    def L(self, name):
        return f"v13_{name}_{self.tag}"

    def emit(self, c):
        self.prog.extend(c)

    def new_uid(self):
        self.uid += 1
        return self.uid

    # ---- init ------------------------------------------------------------
    def init(self, in_kernarg, in_wg, in_wave):
        e = self.emit
        e([I("v_writelane_b32", M0SAVE[0], M0, M0SAVE[1])])  # m0 is not on the clobber list
        e([I("s_mov_b64", sKA, in_kernarg), I("s_mov_b32", sL, in_wg), I("s_lshl_b32", sWKOFF, in_wave, WSH())])
        # dwords 37..44 (kn, vn, c, muoff, tbk, tbv, stamp) into s88..s95 first
        e([I("s_load_dwordx8", S(88, 8), sKA, 4 * AI["kn"])])
        if self.causal:
            e([I("s_load_dword", sOFFT, sKA, 4 * AI["offt"])])
        e([I("s_waitcnt", "lgkmcnt(0)")])
        kn, vn = S(88), S(89)
        e([I("s_mov_b32", sC, S(90)), I("s_mov_b32", sTBK, S(92)), I("s_mov_b32", sTBV, S(93))])
        # lane constants
        e([I("v_mbcnt_lo_u32_b32", LANE, -1, 0), I("v_mbcnt_hi_u32_b32", LANE, -1, LANE),
           I("v_and_b32", VI, 15, LANE), I("v_lshrrev_b32", VG, 4, LANE)])
        t = [T(k) for k in range(12)]
        # K read base: 16 (g&1) + 32 (i&7) + 256 (g>>1) + 1024 (i>>3)
        e([I("v_and_b32", t[0], 1, VG), I("v_lshlrev_b32", t[0], 4, t[0]),
           I("v_and_b32", t[1], 7, VI), I("v_lshlrev_b32", t[1], 5, t[1]), I("v_add_u32", t[0], t[0], t[1]),
           I("v_lshrrev_b32", t[1], 1, VG), I("v_lshlrev_b32", t[1], 8, t[1]), I("v_add_u32", t[0], t[0], t[1]),
           I("v_lshrrev_b32", t[1], 3, VI), I("v_lshlrev_b32", t[1], 10, t[1]), I("v_add_u32", VKL, t[0], t[1])])
        # V read base: 8 i + 128 (g&1) + 1024 (g>>1) + 16384
        e([I("v_lshlrev_b32", t[0], 3, VI), I("v_and_b32", t[1], 1, VG), I("v_lshlrev_b32", t[1], 7, t[1]),
           I("v_add_u32", t[0], t[0], t[1]), I("v_lshrrev_b32", t[1], 1, VG), I("v_lshlrev_b32", t[1], 10, t[1]),
           I("v_add_u32", t[0], t[0], t[1]), I("v_add_u32", VVL, VIMG, t[0])])
        # DMA lane parts: row (L>>1)&7, chunk 4((L>>5)&1) + 2((L>>4)&1) + (L&1)
        e([I("v_lshrrev_b32", t[2], 1, LANE), I("v_and_b32", t[2], 7, t[2]),          # laneRow
           I("v_lshrrev_b32", t[3], 5, LANE), I("v_and_b32", t[3], 1, t[3]), I("v_lshlrev_b32", t[3], 2, t[3]),
           I("v_lshrrev_b32", t[4], 4, LANE), I("v_and_b32", t[4], 1, t[4]), I("v_lshlrev_b32", t[4], 1, t[4]),
           I("v_add_u32", t[3], t[3], t[4]), I("v_and_b32", t[4], 1, LANE), I("v_add_u32", t[3], t[3], t[4]),
           I("v_lshlrev_b32", t[3], 4, t[3])])                                          # 16 * laneCh
        for j in range(NPW() // 2):
            # K piece pc = (NPW/2) w + j: rowbase 16((pc>>1)&3) + 8(pc&1), chbase 8(pc>>3)
            # V piece: rowbase 8(pc&7), chbase 8(pc>>3) (D = 64: pc < 8, chbase 0)
            e([I("s_lshr_b32", sT2, sWKOFF, 10), I("s_add_u32", sT2, sT2, j),           # pc = (NPW/2) wave + j
               I("s_lshr_b32", sT3, sT2, 1), I("s_and_b32", sT3, sT3, 3), I("s_lshl_b32", sT3, sT3, 4),
               I("s_and_b32", sT4, sT2, 1), I("s_lshl_b32", sT4, sT4, 3), I("s_add_u32", sT3, sT3, sT4),  # K rowbase
               I("s_and_b32", sT4, sT2, 7), I("s_lshl_b32", sT4, sT4, 3),               # V rowbase
               I("s_lshr_b32", sT5, sT2, 3), I("s_lshl_b32", sT5, sT5, 7),              # 16 * chbase
               I("s_sub_u32", sT5, sT5, 1024 * j)])
            for (rb, st, dst) in ((sT3, kn, DMAK(j)), (sT4, vn, DMAV(j))):
                e([I("v_add_u32", t[5], rb, t[2]), I("v_mul_lo_u32", t[5], t[5], st),
                   I("v_add_u32", t[5], t[5], t[3]), I("v_add_u32", dst, sT5, t[5])])
        e(load_args())
        if RAGGED[0] and not self.causal:
            # PM(kb, hh): keep the half whose key 16 kb + 4 g + 2 hh (+1) >= P0
            e([I("v_lshlrev_b32", T(0), 2, VG), I("v_mov_b32", T(4), 0xFFFF), I("v_mov_b32", T(5), 0xFFFF0000)])
            for kb in range(4):
                for hh in range(2):
                    e([I("v_add_u32", T(1), 16 * kb + 2 * hh, T(0)),
                       I("v_cmp_le_u32_e32", VCC, ARG(AI["cw"]), T(1)),
                       I("v_cndmask_b32_e32", T(2), 0, T(4), VCC),
                       I("v_add_u32", T(1), 1, T(1)),
                       I("v_cmp_le_u32_e32", VCC, ARG(AI["cw"]), T(1)),
                       I("v_cndmask_b32_e32", T(3), 0, T(5), VCC),
                       I("v_or_b32", PM(kb, hh), T(2), T(3))])
        if self.stamp:
            # STAMP: lanes 0-3 of v217 = entry s_memtime / s_memrealtime, lane 8
            # = this wave's record index (workgroup x 4 + wave)
            e([I("s_memtime", S(96, 2)), I("s_memrealtime", S(98, 2)), I("s_waitcnt", "lgkmcnt(0)")])
            e([I("v_writelane_b32", STAMPV, S(96 + k), k) for k in range(4)])
            e([I("s_lshl_b32", sT6, sL, 2), I("s_lshr_b32", sT7, sWKOFF, WSH()), I("s_add_u32", sT6, sT6, sT7),
               I("v_writelane_b32", STAMPV, sT6, 8)])
            # seam sums (lanes 16-21) from 0, the last point (lane 15) = entry
            e([I("v_writelane_b32", STAMPV, 0, 16 + k) for k in range(6)] +
              [I("v_writelane_b32", STAMPV, S(96), 15)])
        # ones selector, ring slots, causal mask operands
        e([I("v_mov_b32", ONES[k], DT["ones"]) for k in range(4)])
        e([I("s_mov_b32", sS0, 0), I("s_mov_b32", sSP1, SLOT), I("s_mov_b32", sSP2, 2 * SLOT),
           I("s_mov_b32", sSM1, 4 * SLOT)])
        if self.causal:
            e([I("v_mov_b32", NINF[k], 0xFF800000) for k in range(4)])
            if BALANCED[0]:
                # LIMW = 16 w + i - 4 g: the diagonal q-block's key 16 kb + 4 g + r
                # is past row 16 w + i iff 16 kb + r > LIMW
                e([I("v_lshlrev_b32", T(0), 2, VG), I("s_lshr_b32", sT2, sWKOFF, WSH() - 4),
                   I("v_add_u32", T(1), sT2, VI), I("v_sub_u32", LIMW, T(1), T(0))])
            else:
                # diagonal block: key 4g + r of the block masked above query i
                e([I("v_lshlrev_b32", T(0), 2, VG)])
                for r in range(4):
                    e([I("v_add_u32", T(1), r, T(0)), I("v_cmp_lt_i32_e32", VCC, VI, T(1)),
                       I("v_cndmask_b32_e32", TRI[r], 0, NINF[0], VCC)])

    # ---- per-block scalar setup -----------------------------------------
    def q_offsets(self, q0, qh, loads=True):
        """QOFF(qb) = min(q0 + 16 qb + i, Nq - 1) * qn + 16 g; Q loads.
        Causal: rows are virtual, q' = q + s with s = (-Nq) & 63 (QSHIFT),
        so the load row is min(max(q', s) - s, Nq - 1)"""
        c = [I("s_sub_u32", sT0, ARG(AI["nq"]), 1)]
        if self.causal:
            c += qshift(sT1, sT2)
        for qb in range(4):
            c += [I("v_add_u32", T(0), q0, VI), I("v_add_u32", T(0), RS() * qb, T(0))]
            if self.causal:
                c += [I("v_max_u32", T(0), sT1, T(0)), I("v_subrev_u32", T(0), sT1, T(0))]
            c += [I("v_min_u32", T(0), sT0, T(0)), I("v_mul_lo_u32", T(0), T(0), ARG(AI["qn"])),
                  I("v_lshlrev_b32", T(1), 4, VG), I("v_add_u32", QOFF(qb), T(0), T(1))]
        for qb in range(4):
            for ds in range(NDS()):
                if loads:
                    c.append(I("global_load_dwordx4", Q_(qb, ds), QOFF(qb), qh,
                               mods=f"offset:{64 * ds} {CACHEBITS['q']}".rstrip()))
        return c

    def block_setup_first(self):
        """first block: params, DMA tiles 0 and 1, Q loads, next-block params"""
        e = self.emit
        e(block_params(sL, self.causal, self.new_uid(), rev=int(self.rev)))
        if self.rev:
            e([I("s_mov_b64", sCOH, sNOH), I("s_mov_b32", sCQ0, sNQ0), I("s_and_b32", sNT, sT8, 0xFFFF),
               I("s_lshr_b32", sDIR, sT8, 16),
               I("s_mov_b64", sDK, S(sT0.i, 2)), I("s_mov_b64", sDV, S(sT2.i, 2)),
               I("s_and_b32", sDIDX, sT8, 0xFFFF0000), I("s_mov_b32", sDNT, sT8)])
            e(self.q_offsets(sNQ0, sNQH))
            # the stream is at position 2 when the next block's params are made
            e(dma_now(sS0, rev=True))
            e(dma_now(sSP1, rev=True))
            e(self._next_params())
            e(self.first_wait())
            return
        e([I("s_mov_b64", sCOH, sNOH), I("s_mov_b32", sCQ0, sNQ0), I("s_mov_b32", sNT, sT8),
           I("s_mov_b64", sDK, S(sT0.i, 2)), I("s_mov_b64", sDV, S(sT2.i, 2)), I("s_mov_b32", sDIDX, 0),
           I("s_mov_b32", sDNT, sT8)])
        e(self.q_offsets(sNQ0, sNQH))
        e(self._next_params())
        e(dma_now(sS0))
        e(dma_now(sSP1))
        e(self.first_wait())

    def first_wait(self):
        """SEAMWAIT: the first block issues its Q loads before key tiles 0 and
        1, so tile 0 is retired here (vmcnt(NPW): only tile 1 may stay in
        flight) and the block's first barrier's vmcnt(NPW + 4 NDS), counted
        for the seam's order (tile 0, tile 1, Q loads, O stores), waits for
        nothing more on this path"""
        return [I("s_waitcnt", f"vmcnt({NPW()})")] if SEAMWAIT[0] else []

    def _next_params(self):
        """sHASN = L + G < nblocks; if so the next block's params into sNQH,
        sNOH, sNQ0, its K / V heads into sNXK / sNXV with sNXIDX = 0 and its
        tile count in sNXNT; else the stream parks on the current block's
        last tile (sNXK = its address, sNXIDX = nt - 1, sNXNT = nt).  The
        stream pointer sDK / sDV is at tile sDIDX of the current block."""
        skip = self.L(f"nonext{self.new_uid()}")
        if self.rev:
            # (causal) park: the tile of stream position 1 of the current
            # block (the stream is at position 2: one tile back in either
            # order), a one-tile stream that repeats
            c = [I("s_sub_u32", sNXK[0], sDK[0], sTBK), I("s_subb_u32", sNXK[1], sDK[1], 0),
                 I("s_sub_u32", sNXV[0], sDV[0], sTBV), I("s_subb_u32", sNXV[1], sDV[1], 0)]
            if RAGGED[0]:
                # a forward block's position 1 may be key tile NT - 1, whose
                # unshifted rows run past the head: park on tile 0 instead
                c += [I("s_cmp_eq_u32", sDIR, 0), I("s_cselect_b32", sT2, sTBK, 0),
                      I("s_sub_u32", sNXK[0], sNXK[0], sT2), I("s_subb_u32", sNXK[1], sNXK[1], 0),
                      I("s_cmp_eq_u32", sDIR, 0), I("s_cselect_b32", sT2, sTBV, 0),
                      I("s_sub_u32", sNXV[0], sNXV[0], sT2), I("s_subb_u32", sNXV[1], sNXV[1], 0)]
            c += [I("s_mov_b32", sNXIDX, 0), I("s_mov_b32", sNXNT, 1),
                 I("s_add_u32", sT2, sL, ARG(AI["G"])), I("s_cmp_ge_u32", sT2, ARG(AI["nblocks"])),
                 I("s_cbranch_scc1", skip),
                 I("s_add_u32", sT7, sL, ARG(AI["G"]))]
            c += block_params(sT7, self.causal, self.new_uid(), rev=1)
            c += [I("s_mov_b64", sNXK, S(sT0.i, 2)), I("s_mov_b64", sNXV, S(sT2.i, 2)),
                  I("s_and_b32", sNXIDX, sT8, 0xFFFF0000), I("s_mov_b32", sNXNT, sT8)]
            c += [label(skip)]
            return c
        c = [I("s_add_u32", sT2, sL, ARG(AI["G"])), I("s_cmp_lt_u32", sT2, ARG(AI["nblocks"])),
             I("s_cselect_b32", sHASN, 1, 0)]
        # parking place: sDK + (nt - 1 - sDIDX) tiles (signed: -1 when nt = 2
        # and both tiles were already issued)
        c += [I("s_sub_u32", sT4, sNT, 1), I("s_sub_u32", sT4, sT4, sDIDX)]
        for (dst, src, tb) in ((sNXK, sDK, sTBK), (sNXV, sDV, sTBV)):
            c += [I("s_mul_i32", sT5, sT4, tb), I("s_ashr_i32", sT3, sT5, 31),
                  I("s_add_u32", dst[0], src[0], sT5), I("s_addc_u32", dst[1], src[1], sT3)]
        if RAGGED[0]:
            # (sDK already points P0 keys back once the stream is at or past
            # the last tile)
            c += [I("s_sub_u32", sT4, sNT, 1), I("s_sub_u32", sT4, sT4, sDIDX), I("s_cmp_gt_i32", sT4, 0)]
            c += rag_back(sNXK, sNXV)
        c += [I("s_sub_u32", sNXIDX, sNT, 1), I("s_mov_b32", sNXNT, sNT)]
        c += [I("s_cmp_eq_u32", sHASN, 0), I("s_cbranch_scc1", skip)]
        # the next block's index in s101 (block_params reads it first)
        c += [I("s_add_u32", sT7, sL, ARG(AI["G"]))]
        c += block_params(sT7, self.causal, self.new_uid())
        c += [I("s_mov_b64", sNXK, S(sT0.i, 2)), I("s_mov_b64", sNXV, S(sT2.i, 2)), I("s_mov_b32", sNXIDX, 0),
              I("s_mov_b32", sNXNT, sT8)]
        c += [label(skip)]
        return c

    # ---- the tile loop ---------------------------------------------------
    def block_body(self):
        """O, l zero; tile 0 (QK, exact max, P); the step loop; the tail; the
        epilogue; the walk to the next block"""
        e, Lb = self.emit, self.L
        e([label(Lb("common"))])
        e(self.seam_stamp(3))
        e([I("s_load_dword", sT8, sKA, 4 * AI["muoff"])])
        if self.causal:
            e([I("s_lshr_b32", sTD, sCQ0, 6), I("s_add_u32", sTD, sTD, sOFFT)])  # the wave's diagonal tile
        # (zeroing O and l in QK(0)'s gaps instead: level -- the gaps it frees
        # here it takes from QK(0); profiles/r05/flash/seam/)
        e([I("v_accvgpr_write_b32", A(k), 0) for k in range(16 * NDB())])  # O
        e([I("v_mov_b32", L_(qb)[r], 0) for qb in range(4) for r in range(4)])
        if not LCHECK[0]:
            e([I("v_mov_b32", ACC(0), 0), I("v_mov_b32", ACC(1), 0)])
        # this wave's pieces of the block's key tile 0 have landed: on both
        # paths here the VMEM operations after them are tile 1's NPW pieces and
        # the NDS x 4 Q loads (and, at a seam, the last block's O stores after
        # those).  SEAMWAIT 0 waited for everything, the O stores' write-back
        # and all the Q loads included (timing: profiles/r05/flash/)
        n_after = NPW() + 4 * NDS()
        e([I("s_waitcnt", f"vmcnt({n_after})" if SEAMWAIT[0] else "vmcnt(0)"), I("s_barrier")])
        e(self.seam_stamp(4))
        if QSCALE[0]:
            e(self.q_prescale())
        # tile 0: K(0) fragments, QK(0) with tile 2's DMA beside it
        e([I("v_add_u32", VKA, sS0, VKL)])
        e(k_reads())
        fills = dma_fills(sSP2, earliest0=1, spacing=4, rev=self.rev)
        qk0 = qk_mfmas()
        if PROPIPE[0] and not self.causal:
            # non-causal: q-block qb's exact row max, mu and P in the gaps of
            # QK(0)'s later q-blocks (QK runs q-block major)
            fills += self.prologue_fills()
            body, left = schedule(qk0, fills, self.budget)
            e(body)
            e(drain(left, len(qk0)))
            e([I("s_waitcnt", f"vmcnt({NPW()})"), I("s_barrier"), I("v_add_u32", VKA, sSP1, VKL)])
            e(k_reads())
            e([I("s_mov_b32", sT, 1)])
            e(self.seam_stamp(5))
            self.loop_and_tails()
            return
        body, left = schedule(qk0, fills, self.budget)
        e(body)
        e(drain(left, len(qk0)))
        if self.rev:
            # only the wave whose diagonal tile this is has masked scores in it
            # (a first tile is never past a wave's diagonal)
            skip = Lb(f"nomask{self.new_uid()}")
            e(self.tile_of(sT0, 0))
            e([I("s_cmp_lt_u32", sT0, sTD), I("s_cbranch_scc1", skip)])
            e(self.mask_rt(sT0))
            e([label(skip)])
        elif self.causal:
            e(self.mask_rt(0))
        # exact row max -> mu = max * c + muoff; P(0) into state 0
        for qb in range(4):
            e(row_max(qb, T(20 + qb), T(30), T(31)))
            if QSCALE[0]:  # S = c s already
                e([I("v_add_f32", MU(qb), sT8, T(20 + qb))] +
                  [I("v_sub_f32", MUC(qb)[r], 0, MU(qb)) for r in range(4)])
            else:
                e([I("v_mul_f32", T(20 + qb), sC, T(20 + qb)), I("v_add_f32", MU(qb), sT8, T(20 + qb))])
        e(exps_all(0))
        # tile 1 landed (tile 2 in flight): K(1) fragments
        e([I("s_waitcnt", f"vmcnt({NPW()})"), I("s_barrier"), I("v_add_u32", VKA, sSP1, VKL)])
        e(k_reads())
        e([I("s_mov_b32", sT, 1)])
        e(self.seam_stamp(5))
        self.loop_and_tails()

    def prologue_fills(self):
        """PROPIPE: per q-block, the row max of tile 0 and mu (one fill after
        its S blocks complete), then its P slices (the 4 deferred slices are
        left to step 1, which computes them from S; QSCALE shifts their S in
        place, S = c s - mu, as step 1 expects)"""
        dfr, now = self.deferred()
        fills, prev_rm, cv = [], None, {}
        for qb in range(4):
            ins = row_max(qb, T(20 + qb), T(30), T(31))
            if QSCALE[0]:
                ins += [I("v_add_f32", MU(qb), sT8, T(20 + qb))] + \
                    [I("v_sub_f32", MUC(qb)[r], 0, MU(qb)) for r in range(4)]
            else:
                ins += [I("v_mul_f32", T(20 + qb), sC, T(20 + qb)), I("v_add_f32", MU(qb), sT8, T(20 + qb))]
            rm = Fill(ins, 16, deps=[prev_rm] if prev_rm else [], sep=0, earliest=qk_done_gap(3, qb) + 3,
                      tag="rowmax")
            fills.append(rm)
            prev_rm = rm
            mine = [sl for sl in now if sl[0] == qb]
            if QSCALE[0]:
                n = 0
                for (q_, kb, hh) in [sl for sl in dfr + now if sl[0] == qb]:
                    sw = S_(kb, qb)
                    sh = Fill([I("v_sub_f32", sw[2 * hh], sw[2 * hh], MU(qb)),
                               I("v_sub_f32", sw[2 * hh + 1], sw[2 * hh + 1], MU(qb))], 8, deps=[rm], sep=1,
                              tag="shift")
                    fills.append(sh)
                    if (q_, kb, hh) in dfr:
                        continue
                    slot = (8 * qb + n) % (NY // 2)
                    n += 1
                    y0, y1 = Y(2 * slot), Y(2 * slot + 1)
                    dep = [sh] + ([cv[slot]] if slot in cv else [])
                    xm = "clamp" if LCHECK[0] else ""
                    e0 = Fill(I("v_exp_f32", y0, sw[2 * hh], mods=xm), 8, trans=True, deps=dep, sep=1, tag="exp")
                    e1 = Fill(I("v_exp_f32", y1, sw[2 * hh + 1], mods=xm), 8, trans=True, deps=dep, sep=1, tag="exp")
                    w = P_(0, qb, kb >> 1)[2 * (kb & 1) + hh]
                    cv[slot] = Fill(I(DT["cvt"], w, y0, y1), 4, deps=[e0, e1], sep=1, tag="cvt")
                    fills += [e0, e1, cv[slot]]
            else:
                f, cv, _ = softmax_fills(0, mine, lambda q_, kb: 0, ytag=8 * qb, prev_cv=cv,
                                         extra_deps=lambda q_, kb: [rm])
                fills += [x for x in f if x.tag != "or"]
        return fills

    def loop_and_tails(self):
        e, Lb = self.emit, self.L
        # steps t = 1 .. nt-1, two per iteration (P states 1 / 0)
        if self.pad:
            e([I("s_nop", 0)] * self.pad)
        e([label(Lb("loop"))])
        self.step_dispatch(1)
        e([I("s_add_u32", sT, sT, 1), I("s_cmp_ge_u32", sT, sNT), I("s_cbranch_scc1", Lb("tail1"))])
        self.step_dispatch(0)
        e([I("s_add_u32", sT, sT, 1), I("s_cmp_lt_u32", sT, sNT), I("s_cbranch_scc1", Lb("loop"))])
        # tails: the last tile T = nt - 1 is in state (T & 1)
        self.tail_dispatch(0)
        e([I("s_branch", Lb("epi"))])
        e([label(Lb("tail1"))])
        self.tail_dispatch(1)
        e([label(Lb("epi"))])
        self.epilogue()

    def deferred(self):
        sl = slice_list()
        return sl[len(sl) - self.ndef:], sl[:len(sl) - self.ndef]

    def q_prescale(self):
        """QSCALE: every Q word (two bf16) in the accumulator file times c,
        rounded to bf16 (RNE); eight rotating temporaries"""
        c = []
        n = 0
        for qb in range(4):
            for ds in range(NDS()):
                for r in range(4):
                    a = Q_(qb, ds)[r]
                    t0, t1, t2 = T(3 * (n % 8)), T(3 * (n % 8) + 1), T(3 * (n % 8) + 2)
                    if DT["cvt"] == "v_cvt_pk_f16_f32":  # fp16 halves: widen, scale, RNE back
                        c += [I("v_accvgpr_read_b32", t0, a), I("v_cvt_f32_f16", t1, t0),
                              I("v_lshrrev_b32", t2, 16, t0), I("v_cvt_f32_f16", t2, t2)]
                    else:
                        c += [I("v_accvgpr_read_b32", t0, a), I("v_lshlrev_b32", t1, 16, t0),
                              I("v_and_b32", t2, 0xFFFF0000, t0)]
                    c += [I("v_mul_f32", t1, sC, t1), I("v_mul_f32", t2, sC, t2),
                          I(DT["cvt"], t0, t1, t2), I("v_accvgpr_write_b32", a, t0)]
                    if QSPLIT[0]:
                        # lo = bf16(q c - hi): the residual of each half, RNE
                        h1, h2 = T(24 + 2 * (n % 4)), T(25 + 2 * (n % 4))
                        c += [I("v_lshlrev_b32", h1, 16, t0), I("v_and_b32", h2, 0xFFFF0000, t0),
                              I("v_sub_f32", t1, t1, h1), I("v_sub_f32", t2, t2, h2),
                              I("v_cvt_pk_bf16_f32", t0, t1, t2), I("v_accvgpr_write_b32", QL_(qb, ds)[r], t0)]
                    n += 1
        return c

    def seam_stamp(self, k):
        """STAMP build: s_memtime now; lane 16 + k of STAMPV += now - (lane
        15), lane 15 = now (cycles since the previous seam point; points: 0
        tail start, 1 epilogue, 2 after the O stores, 3 the next block's
        common code, 4 after its first barrier, 5 the tile loop).  Uses
        s96..s99 (free at every point)"""
        if not self.stamp:
            return []
        return [I("s_memtime", S(96, 2)), I("s_waitcnt", "lgkmcnt(0)"),
                I("v_readlane_b32", S(98), STAMPV, 15), I("s_sub_u32", S(99), S(96), S(98)),
                I("v_readlane_b32", S(98), STAMPV, 16 + k), I("s_add_u32", S(98), S(98), S(99)),
                I("v_writelane_b32", STAMPV, S(98), 16 + k), I("v_writelane_b32", STAMPV, S(96), 15)]

    def mask_rt(self, tile):
        """causal, straight line (prologue and rare path): the mask of the
        tile whose index is in `tile` (SGPR or 0); RAGGED: key tile NT - 1
        holds shifted keys and takes the rag mask (or all -inf when the
        wave's diagonal is before it)"""
        if not RAGGED[0]:
            return mask_tile(tile)
        u = self.new_uid()
        normal, allinf, done = self.L(f"mnorm{u}"), self.L(f"minf{u}"), self.L(f"mdone{u}")
        c = [I("s_sub_u32", sT6, ARG(AI["nt"]), 1), I("s_cmp_eq_u32", tile, sT6), I("s_cbranch_scc0", normal),
             I("s_cmp_lt_u32", sTD, sT6), I("s_cbranch_scc1", allinf)]
        c += rag_setup()
        for qb in range(4):
            for kb in range(4):
                c += rag_block(kb, qb)
        c += [I("s_branch", done), label(allinf)]
        c += [I("v_mov_b32", S_(kb, qb)[r], NINF[0]) for qb in range(4) for kb in range(4) for r in range(4)]
        c += [I("s_branch", done), label(normal)] + mask_tile(tile) + [label(done)]
        return c

    def tile_of(self, dst, pos):
        """causal: the key tile at stream position pos (SGPR or 0) of the
        current block: pos, or reversed (sDIR) nt-4+pos for pos < 4 and
        nt-1-pos after (the diagonal group first -- every wave's first tile
        then has an unmasked key in every row -- then down to tile 0)"""
        if not self.rev:
            return [I("s_mov_b32", dst, pos)]
        if pos == 0:
            return [I("s_sub_u32", sT2, sNT, 4), I("s_cmp_eq_u32", sDIR, 0), I("s_cselect_b32", dst, 0, sT2)]
        return [I("s_add_u32", sT2, sNT, pos), I("s_sub_u32", sT2, sT2, 4), I("s_sub_u32", sT3, sNT, 1),
                I("s_sub_u32", sT3, sT3, pos), I("s_cmp_lt_u32", pos, 4), I("s_cselect_b32", sT3, sT2, sT3),
                I("s_cmp_eq_u32", sDIR, 0), I("s_cselect_b32", dst, pos, sT3)]

    def step_dispatch(self, X):
        """causal: the wave's tiles below its diagonal run the plain step,
        the diagonal tile the masked one, tiles past it the all -inf one (the
        workgroup's last row sees them; this wave's rows do not)"""
        if not self.causal:
            self.step(X, None)
            return
        e, Lb = self.emit, self.L
        u = self.new_uid()
        n, d, cont = Lb(f"plain{u}"), Lb(f"diag{u}"), Lb(f"stepped{u}")
        tl = sT
        if self.rev:
            e(self.tile_of(sT0, sT))
            tl = sT0
        if BALANCED[0]:
            # tiles below the diagonal group: the plain step; tile sTD + m:
            # group step m (every block ends at sTD + 3 or before)
            gl = [Lb(f"grp{m}_{u}") for m in range(4)]
            e([I("s_cmp_lt_u32", tl, sTD), I("s_cbranch_scc1", n), I("s_sub_u32", sT1, tl, sTD)] +
              [x for m in range(3) for x in (I("s_cmp_eq_u32", sT1, m), I("s_cbranch_scc1", gl[m]))] +
              [I("s_branch", gl[3])])
            e([label(n)])
            self.step(X, None)
            for m in range(4):
                e([I("s_branch", cont), label(gl[m])])
                self.step(X, ("grp", m))
            e([label(cont)])
            return
        rg, by = Lb(f"rag{u}"), Lb(f"beyond{u}")
        if RAGGED[0]:
            # key tile NT - 1 holds keys Nk - 64 .. Nk - 1: the rag step (a
            # VALU mask on the shifted keys) unless the wave's diagonal is
            # before it (then every score is masked: the beyond step)
            e([I("s_sub_u32", sT2, ARG(AI["nt"]), 1), I("s_cmp_eq_u32", tl, sT2), I("s_cbranch_scc1", rg)])
        e([I("s_cmp_lt_u32", tl, sTD), I("s_cbranch_scc1", n), I("s_cmp_eq_u32", tl, sTD),
           I("s_cbranch_scc1", d)] + ([label(by)] if RAGGED[0] else []))
        b2 = Lb(f"beyond2{u}")
        if BEYOND[0] >= 2:
            # the tile before (position t - 1) past the diagonal too: its P is
            # 0, so PV(t-1) is skipped as well -- the idle step
            e([I("s_sub_u32", sT1, sT, 1)])
            if self.rev:
                e(self.tile_of(sT1, sT1))
            e([I("s_cmp_gt_u32", sT1, sTD), I("s_cbranch_scc1", b2)])
        self.step(X, "beyond")
        e([I("s_branch", cont), label(n)])
        self.step(X, None)
        e([I("s_branch", cont), label(d)])
        self.step(X, "diag")
        if RAGGED[0]:
            e([I("s_branch", cont), label(rg), I("s_cmp_lt_u32", sTD, sT2), I("s_cbranch_scc1", by)])
            self.step(X, "rag")
        if BEYOND[0] >= 2:
            e([I("s_branch", cont), label(b2)])
            self.step_idle(X)
        e([label(cont)])

    def step_idle(self, X):
        """causal, tiles t and t-1 both past this wave's diagonal (BEYOND):
        nothing of either reaches O or l (P = 0), so only the stream moves --
        tile t+2's DMA, the barrier, K(t+1)'s fragments -- and P(t) = 0, the S
        words its deferred slices would read = -inf (for a light step or the
        tail after this one)"""
        e = self.emit
        dfr, _ = self.deferred()
        e(rotate_slots())
        for f in dma_fills(sSP2, earliest0=1, spacing=self.dma_spacing, rev=self.rev):
            e(f.ins)
        e([I("v_mov_b32", P_(X, qb, kp)[r], 0) for qb in range(4) for kp in range(2) for r in range(4)])
        e([I("v_mov_b32", S_(kb, qb)[2 * hh + j], NINF[0]) for (qb, kb, hh) in dfr for j in range(2)])
        if not LCHECK[0]:
            e([I("v_mov_b32", ACC(X), 0)])
        e([I("s_waitcnt", f"vmcnt({NPW()})")] + ([] if "barrier" in ABL else [I("s_barrier")]))
        skip = None
        if BEYOND[0] >= 3:
            # K(t+1) is read only if tile t+1 is not past the diagonal too
            # (forward blocks: never; reversed: position 4 after the group)
            skip = self.L(f"nokread{self.new_uid()}")
            e([I("s_add_u32", sT1, sT, 1)])
            if self.rev:
                e(self.tile_of(sT1, sT1))
            e([I("s_cmp_gt_u32", sT1, sTD), I("s_cbranch_scc1", skip)])
        e([I("v_add_u32", VKA, sSP1, VKL)])
        e(k_reads())
        if skip:
            e([label(skip)])

    def tail_dispatch(self, X):
        """causal (BEYOND): the last tile past this wave's diagonal (forward
        blocks of waves 0-2) adds nothing to O or l -- only the next block's
        Q loads run"""
        if BALANCED[0]:
            # the last tile of a forward block is normally group tile sTD + 3,
            # whose q-blocks 0-2 are dead: the tail's PV runs on q-block 3 only
            e, Lb = self.emit, self.L
            u = self.new_uid()
            g3, done = Lb(f"tailg3_{u}"), Lb(f"tailed{u}")
            e([I("s_sub_u32", sT1, sNT, 1)])
            if self.rev:
                e(self.tile_of(sT1, sT1))
            e([I("s_add_u32", sT2, sTD, 3), I("s_cmp_eq_u32", sT1, sT2), I("s_cbranch_scc1", g3)])
            self.tail(X)
            e([I("s_branch", done), label(g3)])
            self.tail(X, dead=3)
            e([label(done)])
            return
        if not (self.causal and BEYOND[0] >= 2):
            self.tail(X)
            return
        e, Lb = self.emit, self.L
        u = self.new_uid()
        light, done = Lb(f"taillight{u}"), Lb(f"tailed{u}")
        e([I("s_sub_u32", sT1, sNT, 1)])
        if self.rev:
            e(self.tile_of(sT1, sT1))
        e([I("s_cmp_gt_u32", sT1, sTD), I("s_cbranch_scc1", light)])
        self.tail(X)
        e([I("s_branch", done), label(light)])
        e(self.seam_stamp(0))
        e(rotate_slots())
        e(self.q_offsets(sNQ0, sNQH, loads="qload" not in ABL))
        e([label(done)])

    def check(self, Xc, rare_block):
        """the defer-max check of the tile in P state Xc (some P >= 2: bit 14
        of a bf16 half); the rare block returns to the label emitted here"""
        e, Lb = self.emit, self.L
        k = len(self.sites)
        ret = Lb(f"ret{k}")
        self.sites.append((k, rare_block, ret))
        if "check" in ABL:
            e([label(ret)])
            return
        if LCHECK[0]:  # some row's l >= 1 (its row sums ran right before)
            e([I("v_max3_f32", T(37), L_(0)[0], L_(1)[0], L_(2)[0]), I("v_max_f32", T(37), T(37), L_(3)[0]),
               I("v_cmp_le_f32_e32", VCC, 1.0, T(37)),  # 1 <= l: a clamped P (= 1) alone trips it
               I("s_mov_b32", sRET, k), I("s_cbranch_vccnz", Lb(rare_block)), label(ret)])
            return
        e([I("v_and_b32", T(37), 0x40004000, ACC(Xc)), I("v_cmp_ne_u32_e32", VCC, 0, T(37)),
           I("s_mov_b32", sRET, k), I("s_cbranch_vccnz", Lb(rare_block)), label(ret)])

    def step(self, X, mask):
        """step t (state X = t & 1): QK(t) || the deferred slices of t-1,
        tile t+2's DMA, V(t-1) d-blocks 0-1, softmax(t); the defer-max check
        of t-1; barrier; PV(t-1) + row sums || K(t+1), V(t-1) d-blocks 2-7,
        softmax(t)"""
        e = self.emit
        Xp = 1 - X
        dfr, now = self.deferred()
        e(rotate_slots())
        e([I("v_add_u32", VVA, sSM1, VVL)])
        # ---- QK phase
        fills = []
        # deferred slices of tile t-1 (they read S(., 3): before QK(t) overwrites it)
        qk, done, first = qk_with_rowsums(mask, QSCALE[0], Xp if LCHECK[0] else None)
        dl = lambda qb, kb: first(kb, qb) - 1  # noqa: E731
        # BEYOND: a tile past this wave's diagonal has every score masked --
        # no QK(t) and no softmax(t): P(t) = 0 and the S words its deferred
        # slices read next step = -inf, written after t-1's deferred slices
        light = mask == "beyond" and BEYOND[0]
        if light:
            qk = []  # (t-1's row sums run below, after its deferred slices)
            dl = None
        diag_skip = mask == "diag" and BEYOND[0] >= 4
        if diag_skip:
            # the diagonal tile's blocks kb > qb are -inf whole: S = -inf by
            # v_mov instead of their 4 chained MFMAs (qb 3 is never among
            # them, so t-1's deferred slices, which read S(., 3), are unaffected)
            dead = {S_(kb, qb).i for qb in range(4) for kb in range(4) if kb > qb}
            keep = [j for j, m in enumerate(qk) if not (m.op == DT["mfma"] and m.ops[0].i in dead)]
            newpos = {j: n for n, j in enumerate(keep)}
            qk = [qk[j] for j in keep]
            done0, first0 = done, first
            done = lambda kb, qb: newpos[done0(kb, qb)] if kb <= qb else -3  # noqa: E731
            first = lambda kb, qb: newpos[first0(kb, qb)]  # noqa: E731
            dl = lambda qb, kb: first(kb, qb) - 1  # noqa: E731
            e([I("v_mov_b32", S_(kb, qb)[r], NINF[0]) for qb in range(4) for kb in range(4) if kb > qb
               for r in range(4)])
        grp = mask[1] if isinstance(mask, tuple) and mask[0] == "grp" else None
        if grp is not None:
            # BALANCED, tile sTD + grp: q-blocks below grp are past the
            # diagonal (no QK chains; their P = 0 below), q-block grp is masked
            # by VALU as its S blocks complete
            dead = {S_(kb, qb).i for qb in range(grp) for kb in range(4)}
            keep = [j for j, m in enumerate(qk) if not (m.op == DT["mfma"] and m.ops[0].i in dead)]
            newpos = {j: n for n, j in enumerate(keep)}
            qk = [qk[j] for j in keep]
            done0, first0 = done, first
            done = lambda kb, qb: newpos[done0(kb, qb)] if qb >= grp else -3  # noqa: E731
            first = lambda kb, qb: newpos[first0(kb, qb)] if qb >= grp else 0  # noqa: E731
            dl = lambda qb, kb: first(kb, qb) - 1  # noqa: E731
            now = [sl for sl in now if sl[0] >= grp]
        f_def, cvd, last_or_prev = softmax_fills(Xp, dfr, lambda qb, kb: 0, dl, ytag=0)
        if "soft" in ABL:
            f_def = []
        fills += f_def
        dma = dma_fills(sSP2, earliest0=1, spacing=self.dma_spacing, rev=self.rev)
        dma_pv = []
        if self.dma_pv:
            # the V pieces (4-7, their own M0 write) and the advance go to the
            # PV phase: tile t+2 only has to land by step t+1's barrier
            dma, dma_pv = dma[:5], dma[5:]
            for n, f in enumerate(dma_pv[:4]):
                f.earliest = 64 + self.dma_pv + self.dma_pv_spacing * n
                f.deps = [] if n == 0 else [dma_pv[n - 1]]
            dma_pv[4].deps = [dma_pv[3]]
        fills += dma
        # V(t-1) d-blocks 0, 1 (from 32 MFMAs before the phase ends)
        for db in (0, 1):
            for ins in v_reads(db):
                if "vread" not in ABL and light:
                    fills.append(Fill(ins, 2, earliest=0, tag="vread0"))
                elif "vread" not in ABL:
                    fills.append(Fill(ins, 2, earliest=(40 if GEOM["hd"] == 128 and not diag_skip and grp is None
                                                        else len(qk) - 32) + 8 * db, tag="vread"))
        # softmax(t), zero ACC(X) first (P-bit check)
        z = Fill(I("v_mov_b32", ACC(X), 0), 4, tag="zero")
        if not LCHECK[0]:
            fills.append(z)
        rag = {}
        if mask == "rag":
            # key tile NT - 1 (shifted keys): S(kb, qb) masked by VALU as it
            # completes, before its softmax slices read it
            rsetup = Fill(rag_setup(), 8, earliest=0, tag="ragsetup")
            fills.append(rsetup)
            for qb in range(4):
                for kb in range(4):
                    rag[(kb, qb)] = Fill(rag_block(kb, qb), 16, deps=[rsetup], sep=1, earliest=done(kb, qb) + 3,
                                         tag="ragmask")
                    fills.append(rag[(kb, qb)])
        if grp is not None:
            for kb in range(4):
                rag[(kb, grp)] = Fill(grp_block(kb, grp), 16, earliest=done(kb, grp) + 3, tag="ragmask")
                fills.append(rag[(kb, grp)])
        f_now, cvn, last_or = softmax_fills(X, now, lambda qb, kb: done(kb, qb) + 3, ytag=len(dfr),
                                            prev_cv=cvd,
                                            extra_deps=(lambda qb, kb: [rag[(kb, qb)]] if (kb, qb) in rag else [])
                                            if rag else None)
        now_groups = softmax_fills.groups
        if "soft" in ABL or light:
            f_now, now_groups = [], []
        for f in f_now:
            if f.tag == "or" and not any(d.tag == "or" for d in f.deps):
                f.deps.append(z)
        fills += f_now
        if QSCALE[0] and mask == "diag":
            e([I("v_add_f32", TRIMU(qb)[r], TRI[r], MUC(qb)[r]) for qb in range(4) for r in range(4)])
        body, left = schedule(qk, fills, self.budget)
        e(body)
        # everything of tile t-1 must be done before its check
        pend_prev = [f for f in left if f in f_def or f.tag.startswith("dma") or f.tag.startswith("rag") or
                     f.tag == "vread0"]
        # a slice of tile t that has started finishes before the check: the
        # rare path redoes every P of t from S, and a slice whose fma ran
        # with the old mu must not write its P after that
        for sg in now_groups:
            if any(f.gap is not None for f in sg):
                pend_prev += [f for f in sg if f.gap is None]
        e(drain(pend_prev, len(qk) - 1))
        left = [f for f in left if f.gap is None]
        # light (BEYOND >= 4): tile t-1 is the diagonal one, whose P(qb, kp = 1)
        # for qb 0, 1 (rows 0-31 x keys 32-63) is all zero: no row sums or PV
        # MFMAs on them
        pdead = {P_(Xp, qb, 1).i for qb in (0, 1)} if light and BEYOND[0] >= 4 else set()
        if grp is not None:
            # BALANCED: this tile's dead q-blocks have P = 0; tile t-1 was
            # group step grp - 1 (either stream order), whose q-blocks below
            # grp - 1 were dead: no PV MFMAs on them
            e([I("v_mov_b32", P_(X, qb, kp)[r], 0) for qb in range(grp) for kp in range(2) for r in range(4)])
            pdead = {P_(Xp, qb, kp).i for qb in range(grp - 1) for kp in range(2)}
        if light:
            if LCHECK[0]:
                e([m for m in rowsum_mfmas(Xp) if m.ops[2].i not in pdead])
            e([I("v_mov_b32", P_(X, qb, kp)[r], 0) for qb in range(4) for kp in range(2) for r in range(4)])
            e([I("v_mov_b32", S_(kb, qb)[2 * hh + j], NINF[0]) for (qb, kb, hh) in dfr for j in range(2)])
            if not LCHECK[0]:
                e([I("v_mov_b32", ACC(X), 0)])
        # ---- defer-max check of tile t-1
        self.check(Xp, f"rare_s{Xp}")
        e([I("s_waitcnt", f"vmcnt({NPW()})")] + ([] if "barrier" in ABL else [I("s_barrier")]))
        # ---- PV phase (gaps numbered on from the QK phase's, so the
        # leftover softmax keeps its dependency distances)
        B0 = len(qk)
        fills = left
        ka = Fill(I("v_add_u32", VKA, sSP1, VKL), 4, earliest=B0, tag="kaddr")
        pv = pv_mfmas(Xp)
        if pdead:
            pv = [m for m in pv if m.ops[2].i not in pdead]
        kr = [Fill(ins, 2, deps=[ka], sep=1, earliest=B0 + n // 2, deadline=B0 + min(40, len(pv) - 8), tag="kread")
              for n, ins in enumerate(k_reads())] if "kread" not in ABL else []
        # V d-block db (2..) reads: after d-block db-3's MFMAs (same buffer), well before db's
        vr = []
        if pdead:  # (positions from the shortened list; a missed deadline is an error)
            use = {}
            for j, m in enumerate(pv):
                if m.ops[0].f == "a":
                    use.setdefault(m.ops[0].i // 16, []).append(j)
        for db in range(2 if "vread" not in ABL else NDB(), NDB()):
            for ins in v_reads(db):
                if pdead:
                    vr.append(Fill(ins, 2, earliest=B0 + (use[db - 3][-1] + 2 if db >= 3 else 0),
                                   deadline=B0 + use[db][0] - 6, tag="vread", hard=True))
                else:
                    vr.append(Fill(ins, 2, earliest=B0 + (vbuf_free(db) if db >= 3 else 0),
                                   deadline=B0 + pv_first_gap(db) - 6, tag="vread"))
        fills = [ka] + kr + vr + fills + dma_pv
        body, left = schedule(pv, fills, self.budget_pv, gap_offset=B0)
        e(body)
        e(drain(left, B0 + len(pv) - 1))

    def tail(self, X, dead=0):
        """last tile T (state X): its deferred slices, its check, PV(T) with
        the next block's Q loads beside it (BALANCED: q-blocks below `dead`
        have P = 0 -- no PV MFMAs on them)"""
        e = self.emit
        e(self.seam_stamp(0))
        dfr, _ = self.deferred()
        e(rotate_slots())
        e([I("v_add_u32", VVA, sSM1, VVL)])
        f_def, _, _ = softmax_fills(X, dfr, lambda qb, kb: 0, ytag=0)
        e(drain(f_def, 0))
        if RAGGED[0] and not self.causal:
            e(p_mask(X))
        if LCHECK[0]:
            e(rowsum_mfmas(X))
        self.check(X, f"rare_t{X}")
        fills = []
        if dead:
            # BALANCED tail on group tile sTD + 3: only q-blocks >= dead are
            # live, so PV(T) is 2 (4 - dead) MFMAs per d-block -- too few to
            # hide the V^T reads behind the 3-buffer rotation; every d-block
            # is read up front into its own buffer instead (the three V^T
            # buffers, the other P state and this state's dead P words)
            bufs = [V(128 + 8 * b) for b in range(NVF)] + \
                [V(64 + 32 * (1 - X) + 8 * j) for j in range(4)] + [V(64 + 32 * X + 8 * j) for j in range(dead)]
            assert len(bufs) >= NDB()
            for db in range(NDB()):
                for ins in v_reads(db):
                    d = ins.ops[0]
                    e([I(ins.op, V(bufs[db].i + (d.i - 128) % 8, 2), ins.ops[1], mods=ins.mods)])
            pv = [mfma(O_(db, qb), V(bufs[db].i + 4 * kp, 4), P_(X, qb, kp), O_(db, qb))
                  for db in range(NDB()) for kp in range(2) for qb in range(dead, 4)]
            if not LCHECK[0]:  # (the P-bit check's row sums run with PV)
                pv += [mfma(L_(qb), ONES, P_(X, qb, kp), L_(qb)) for qb in range(dead, 4) for kp in range(2)]
        else:
            e(v_reads(0) + v_reads(1))
            pv = pv_mfmas(X)
            for db in range(2, NDB()):
                for ins in v_reads(db):
                    fills.append(Fill(ins, 2, earliest=vbuf_free(db) if db >= 3 else 0,
                                      deadline=pv_first_gap(db) - 6, tag="vread"))
        # the next block's Q rows (or this block's again past the last block)
        # (ABL "qload", timing only: no Q loads here -- every block reuses the
        # first block's Q)
        qf = chain(self.q_offsets(sNQ0, sNQH, loads="qload" not in ABL), earliest=4)
        if QSEP[0]:
            for f in qf:
                if f.ins[0].op == "global_load_dwordx4":
                    f.sep, f.cost = QSEP[0], 8
        fills += qf
        tailepi = TAILEPI[0] and not dead
        if tailepi:
            fills += self.epi_units(pv)
        body, left = schedule(pv, fills, self.budget)
        e(body)
        e(drain(left, len(pv) - 1))
        if tailepi:
            e([I("s_branch", self.L("epinext"))])

    def epi_units(self, pv):
        """TAILEPI: the epilogue as fills of the tail's PV(T): a setup (1 / l,
        the O row offsets) and one unit per (q-block, d-block pair) -- read the
        pair's 8 accumulators, times 1 / l, pack, swap halves, store (rows past
        Nq masked) -- placed after PV(T)'s last MFMA on those d-blocks.  Uses
        S's registers (dead after the tail's check) and sT4:sT7, never the
        SGPRs of the Q-load chain beside it"""
        setup = [I("v_rcp_f32", EP_RCP(qb), L_(qb)[0]) for qb in range(4)]
        if self.causal:
            setup += qshift(sT4, sT5)
        setup += [I("v_and_b32", EP_LANE, 1, VG), I("v_lshlrev_b32", EP_LANE, 5, EP_LANE),
                  I("v_lshrrev_b32", EP_ROW, 1, VG), I("v_lshlrev_b32", EP_ROW, 4, EP_ROW),
                  I("v_add_u32", EP_LANE, EP_LANE, EP_ROW)]
        row = lambda qb: [I("v_add_u32", EP_ROW, sCQ0, VI), I("v_add_u32", EP_ROW, RS() * qb, EP_ROW)] + \
            ([I("v_subrev_u32", EP_ROW, sT4, EP_ROW)] if self.causal else [])  # noqa: E731
        for qb in range(4):
            setup += row(qb) + [I("v_mul_lo_u32", EP_OOFF(qb), EP_ROW, ARG(AI["on"])),
                                I("v_add_u32", EP_OOFF(qb), EP_OOFF(qb), EP_LANE)]
        fsetup = Fill(setup, 16, earliest=1, tag="episetup")
        last = {}
        for j, m in enumerate(pv):
            if m.ops[0].f == "a":
                last[m.ops[0].i] = j
        fills = [fsetup]
        prev = fsetup
        for dbp in range(NDB() // 2):
            for qb in range(4):
                parts = []
                for half, db in enumerate((2 * dbp, 2 * dbp + 1)):
                    rr = EP_R[4 * half:4 * half + 4]
                    parts.append([I("v_accvgpr_read_b32", rr[r], O_(db, qb)[r]) for r in range(4)] +
                                 [I("v_mul_f32", rr[r], rr[r], EP_RCP(qb)) for r in range(4)])
                parts.append([I(DT["cvt"], EP_W[2 * h], EP_R[4 * h], EP_R[4 * h + 1]) for h in (0, 1)] +
                             [I(DT["cvt"], EP_W[2 * h + 1], EP_R[4 * h + 2], EP_R[4 * h + 3]) for h in (0, 1)] +
                             [I("v_permlane16_swap_b32", EP_W[0], EP_W[2]),
                              I("v_permlane16_swap_b32", EP_W[1], EP_W[3])])
                st = row(qb) + [I("v_cmp_gt_u32_e32", VCC, ARG(AI["nq"]), EP_ROW),
                                I("s_and_saveexec_b64", S(sT6.i, 2), VCC)]
                if "epi_store" not in ABL:
                    st += [I("global_store_dwordx4", EP_OOFF(qb), EP_W, sCOH,
                             mods=f"offset:{64 * dbp} {CACHEBITS['o']}".rstrip())]
                parts.append(st + [I("s_mov_b64", EXEC, S(sT6.i, 2))])
                if TAILEPI[0] != 2:  # one fill per unit
                    parts = [[x for pt in parts for x in pt]]
                ready = max(last[O_(db, qb).i] for db in (2 * dbp, 2 * dbp + 1)) + 1
                for pt in parts:
                    f = Fill(pt, 4 * len(pt), deps=[prev], sep=0, earliest=ready, tag="epiunit")
                    fills.append(f)
                    prev = f
        return fills

    # ---- epilogue ---------------------------------------------------------
    def epilogue(self):
        e, Lb = self.emit, self.L
        e(self.seam_stamp(1))
        e([I("s_nop", 7), I("s_nop", 7)])
        for qb in range(4):
            e([I("v_rcp_f32", T(20 + qb), L_(qb)[0])])
        if self.causal:
            e(qshift(sT1, sT2))
        if OLINE[0]:
            e([I("s_lshl_b32", sT5, ARG(AI["on"]), 3)])  # 8 rows of O
        for qb in range(4):
            # O offsets and the row mask of this q-block (causal: the real
            # row q' - s; a virtual row below s wraps and is not stored).
            # OLINE: the X stores hold rows j & 7 (lanes j < 8: the first 64 B
            # of a 128-B line, j >= 8: the second), the Y stores rows 8 + (j & 7)
            if OLINE[0]:
                e([I("v_and_b32", T(24), 7, VI), I("v_add_u32", T(24), sCQ0, T(24)),
                   I("v_add_u32", T(24), RS() * qb, T(24))])
            else:
                e([I("v_add_u32", T(24), sCQ0, VI), I("v_add_u32", T(24), RS() * qb, T(24))])
            if self.causal:
                e([I("v_subrev_u32", T(24), sT1, T(24))])
            e([I("v_mul_lo_u32", T(25), T(24), ARG(AI["on"])),
               I("v_and_b32", T(26), 1, VG), I("v_lshlrev_b32", T(26), 5, T(26)),
               I("v_lshrrev_b32", T(27), 1, VG), I("v_lshlrev_b32", T(27), 4, T(27)),
               I("v_add3_u32", OOFF(qb), T(25), T(26), T(27))])
            if OLINE[0]:
                e([I("v_lshrrev_b32", T(26), 3, VI), I("v_lshlrev_b32", T(26), 6, T(26)),
                   I("v_add_u32", OOFF(qb), OOFF(qb), T(26)), I("v_add_u32", OOFFY(qb), sT5, OOFF(qb))])
            # packed words of the q-block (W = Y for odd q-blocks, so the next
            # q-block's packing leaves the data of stores in flight alone, was
            # measured level: profiles/r05/flash/seam/)
            W = T
            for dbp in range(NDB() // 2):
                w = 4 * dbp  # words W(w) .. W(w+3)
                for half, db in enumerate((2 * dbp, 2 * dbp + 1)):
                    if "epi_read" not in ABL:  # (timing-only A/B knobs: epi_read / epi_perm / epi_store)
                        for r in range(4):
                            e([I("v_accvgpr_read_b32", T(28 + r), O_(db, qb)[r])])
                    for r in range(4):
                        e([I("v_mul_f32", T(28 + r), T(28 + r), T(20 + qb))])
                    e([I(DT["cvt"], W(w + 2 * half), T(28), T(29)),
                       I(DT["cvt"], W(w + 2 * half + 1), T(30), T(31))])
                if "epi_perm" not in ABL:
                    e([I("v_permlane16_swap_b32", W(w), W(w + 2)), I("v_permlane16_swap_b32", W(w + 1), W(w + 3))])
            if OLINE[0]:
                # whole 128-B lines: per pair of 64-B halves (Wa: bytes 128 p ..,
                # Wb: 128 p + 64 ..), lanes j >= 8 of Wa take Wb of lane j - 8
                # (X: rows j & 7, whole lines) and lanes j < 8 of Wb take Wa of
                # lane j + 8 (Y: rows 8 + (j & 7)), by DPP row_ror:8 + bank masks
                for pr in range(NDB() // 4):
                    Wa, Wb = [W(8 * pr + r) for r in range(4)], [W(8 * pr + 4 + r) for r in range(4)]
                    e([I("v_mov_b32", T(28 + r), Wb[r]) for r in range(4)])
                    e([I("v_mov_b32_dpp", Wb[r], Wa[r], mods="row_ror:8 row_mask:0xf bank_mask:0x3")
                       for r in range(4)])
                    e([I("v_mov_b32_dpp", Wa[r], T(28 + r), mods="row_ror:8 row_mask:0xf bank_mask:0xc")
                       for r in range(4)])
                for y in (0, 1):
                    if y:
                        e([I("v_add_u32", T(25), 8, T(24))])
                    e([I("v_cmp_gt_u32_e32", VCC, ARG(AI["nq"]), T(25) if y else T(24)),
                       I("s_and_saveexec_b64", S(sT2.i, 2), VCC)])
                    for pr in range(NDB() // 4):
                        if "epi_store" not in ABL:
                            e([I("global_store_dwordx4", OOFFY(qb) if y else OOFF(qb), V(W(8 * pr + 4 * y).i, 4),
                                 sCOH, mods=f"offset:{128 * pr}")])
                    e([I("s_mov_b64", EXEC, S(sT2.i, 2))])
                continue
            e([I("v_cmp_gt_u32_e32", VCC, ARG(AI["nq"]), T(24)), I("s_and_saveexec_b64", S(sT2.i, 2), VCC)])
            if "epi_fullline" in ABL:
                # timing only (wrong layout): each store covers 4 rows x 256 B
                # (whole 128-B lines), lane l -> row 4 dbp + l / 16, chunk l % 16
                e([I("v_lshrrev_b32", T(25), 4, LANE), I("v_add_u32", T(25), sCQ0, T(25)),
                   I("v_add_u32", T(25), 16 * qb, T(25)), I("v_mul_lo_u32", T(25), T(25), ARG(AI["on"])),
                   I("v_and_b32", T(26), 15, LANE), I("v_lshlrev_b32", T(26), 4, T(26)),
                   I("v_add_u32", OOFF(qb), T(25), T(26))])
            for dbp in range(NDB() // 2):
                if "epi_store" not in ABL:
                    off = 64 * dbp if "epi_fullline" not in ABL else 0
                    e([I("global_store_dwordx4", OOFF(qb), V(W(4 * dbp).i, 4), sCOH,
                         mods=f"offset:{off} {CACHEBITS['o']}".rstrip())])
            e([I("s_mov_b64", EXEC, S(sT2.i, 2))])
        if TAILEPI[0]:
            e([label(Lb("epinext"))])
        e(self.seam_stamp(2))
        # next block
        if self.rev:
            e([I("s_add_u32", sT2, sL, ARG(AI["G"])), I("s_cmp_ge_u32", sT2, ARG(AI["nblocks"])),
               I("s_cbranch_scc1", Lb("end"))])
            e([I("s_add_u32", sL, sL, ARG(AI["G"])), I("s_mov_b64", sCOH, sNOH), I("s_mov_b32", sCQ0, sNQ0),
               I("s_and_b32", sNT, sNXNT, 0xFFFF), I("s_lshr_b32", sDIR, sNXNT, 16)])
        else:
            e([I("s_cmp_eq_u32", sHASN, 0), I("s_cbranch_scc1", Lb("end"))])
            e([I("s_add_u32", sL, sL, ARG(AI["G"])), I("s_mov_b64", sCOH, sNOH), I("s_mov_b32", sCQ0, sNQ0),
               I("s_mov_b32", sNT, sNXNT)])
        if not NORELOAD[0]:
            e(load_args())
        e(self._next_params())
        e([I("s_branch", Lb("common"))])

    # ---- rare path --------------------------------------------------------
    def rare(self, name, X, has_next):
        """tile t (state X) raised some row's max by >= 8 (log2): recompute
        S(t) from K(t) in slot sSM1, mu_new = max(mu, rowmax * c + muoff),
        rescale O and l by exp2(mu - mu_new), redo P(t); then S(t+1) (slot
        sS0) and every P(t+1) so far, ACC(t+1) from them.  Returns to the
        site whose id is in sRET."""
        e, Lb = self.emit, self.L
        e([label(Lb(name)), I("s_nop", 7), I("s_nop", 7), I("s_load_dword", sT1, sKA, 4 * AI["muoff"])])
        if LCHECK[0]:
            # the tile's old P (still in state X) out of l: l -= 1^T P(X)
            neg = V(T(32).i, 4)
            e([I("v_mov_b32", neg[r], NEGONES) for r in range(4)])
            e(rowsum_mfmas(X, neg))
        for tile_slot, Xs, redo in ((sSM1, X, True), (sS0, 1 - X, has_next)):
            if not redo:
                continue
            e([I("v_add_u32", T(36), tile_slot, VKL)])
            e([I("ds_read_b128", K_(kb, ds), T(36), mods=f"offset:{512 * (ds & 1) + 2048 * kb + 8192 * (ds >> 1)}")
               for ds in range(NDS()) for kb in range(4)])
            # QSCALE: the checked tile with C = 0 (its exact max), the next one
            # shifted by the new mu (its later slices exp S in place)
            e(qk_mfmas(muc=QSCALE[0] and Xs != X))
            if self.causal:
                if Xs == X:  # tile at position sT - 1
                    e([I("s_sub_u32", sT0, sT, 1)])
                    if self.rev:
                        e(self.tile_of(sT0, sT0))
                    e(self.mask_rt(sT0))
                elif self.rev:
                    e(self.tile_of(sT0, sT))
                    e(self.mask_rt(sT0))
                else:
                    e(self.mask_rt(sT))
            if Xs == X:
                for qb in range(4):
                    m = T(20 + qb)
                    e(row_max(qb, m, T(30), T(31)))
                    if not QSCALE[0]:
                        e([I("v_mul_f32", m, sC, m)])
                    e([I("v_add_f32", m, sT1, m), I("v_max_f32", m, m, MU(qb)),
                       I("v_sub_f32", T(24), MU(qb), m), I("v_exp_f32", T(24), T(24)), I("v_mov_b32", MU(qb), m)])
                    if QSCALE[0]:
                        e([I("v_sub_f32", MUC(qb)[r], 0, m) for r in range(4)])
                    for db in range(NDB()):
                        for r in range(4):
                            e([I("v_accvgpr_read_b32", T(25), O_(db, qb)[r]),
                               I("v_mul_f32", T(25), T(25), T(24)),
                               I("v_accvgpr_write_b32", O_(db, qb)[r], T(25))])
                    e([I("v_mul_f32", L_(qb)[r], L_(qb)[r], T(24)) for r in range(4)])
                e(exps_all(X))
                if RAGGED[0] and not self.causal and name.startswith("rare_t"):  # the last tile
                    e(p_mask(X))
                if LCHECK[0]:  # its new sums (the step's row sums of this tile already ran)
                    e(rowsum_mfmas(X))
            else:
                if not LCHECK[0]:
                    e([I("v_mov_b32", ACC(Xs), 0)])
                e(exps_all(Xs, also_or=True, shifted=QSCALE[0]))
        if not LCHECK[0]:
            e([I("v_mov_b32", ACC(X), 0)])
        e([I("s_nop", 4)])
        for k, blk, ret in self.sites:
            if blk == name:
                e([I("s_cmp_eq_u32", sRET, k), I("s_cbranch_scc1", ret)])
        e([I("s_endpgm")])  # unreachable: every site that branches here is listed above

    # ---- whole kernel -----------------------------------------------------
    def build(self, in_kernarg="%0", in_wg="%1", in_wave="%2"):
        self.init(in_kernarg, in_wg, in_wave)
        self.block_setup_first()
        self.block_body()
        e, Lb = self.emit, self.L
        e([label(Lb("end")), I("s_waitcnt", "vmcnt(0)")])
        if self.stamp:
            # exit stamps into lanes 4-7; lanes 0-7 stored at stamp + 32 * record
            e([I("s_memtime", S(96, 2)), I("s_memrealtime", S(98, 2)), I("s_waitcnt", "lgkmcnt(0)")])
            e([I("v_writelane_b32", STAMPV, S(96 + k), 4 + k) for k in range(4)])
            e([I("v_readlane_b32", sT6, STAMPV, 8), I("s_load_dwordx2", S(88, 2), sKA, 4 * AI["stamp"]),
               I("s_waitcnt", "lgkmcnt(0)"), I("s_lshl_b32", sT6, sT6, 7),
               I("v_lshlrev_b32", T(0), 2, LANE), I("v_add_u32", T(0), sT6, T(0)),
               I("s_mov_b64", EXEC, 0xFFFFFFFF), I("global_store_dword", T(0), STAMPV, S(88, 2)),
               I("s_mov_b64", EXEC, -1), I("s_waitcnt", "vmcnt(0)")])
        e([I("s_branch", Lb("exit"))])
        for X in (0, 1):
            self.rare(f"rare_s{X}", X, True)
            self.rare(f"rare_t{X}", X, False)
        e([label(Lb("exit")), I("v_readlane_b32", sT7, M0SAVE[0], M0SAVE[1]), I("s_mov_b32", M0, sT7)])
        return self.prog
