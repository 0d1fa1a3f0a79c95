// attn_fwd_v12: flash-attention forward, one wave per SIMD, 64 query rows per
// wave (reference ch06/flash_attention.py:14-74; gfx950, bf16, D = 128, Nk a
// multiple of 64; causal as a second instantiation -- other cases take
// attn_fwd_v10).
//
// The structure of cdna_hip_programming.md's 4-wave persistent example: one
// workgroup per CU walks blocks L, L + G, ... (G = the grid), each block 4
// waves x 64 rows (two 32-row blocks A
// and B per wave), one workgroup per CU, and each wave owns the whole
// 512-entry register file.  O^T (128 registers), Q^T (64) and the K
// fragments of one tile (64) live in the accumulator file, named literally
// by the inline-asm MFMAs of flash_v12_asm.h; hipcc keeps S, P and the
// softmax in the architectural VGPRs.  One K fragment feeds the QK^T MFMAs of
// both blocks and one V^T fragment both blocks' PV MFMAs, so LDS bytes per
// MFMA are half of attn_fwd_v10's.
//
// Per tile t (steady state), two MFMA phases with the VALU work beside them:
//   phase Q:  S(t) = K(t) Q^T, block A's chain then block B's (32 MFMAs);
//             beside B's chain, block A's softmax slices (running max,
//             speculative exps with the current m, packed P into P(t&1))
//   barrier (tile t+1 landed; every wave past PV(t-2)), DMA of tile t+2
//   phase P:  O += V(t-1)^T P(t-1) (32 MFMAs) + the row-sum MFMAs of P(t-1)
//             || block B's softmax slices || K(t+1) fragments -> AGPR
// then the defer-max ballot of tile t (rare path: drain, rescale O and l,
// recompute S(t) from the LDS copy of K(t), redo its exps and P).  One S
// state, two P states (t even / odd).  K/V tiles arrive by LDS-DMA into a
// 5-slot ring of XOR-swizzled images (attn_fwd_v10's layout), two tiles
// ahead; the stream continues across block seams.
//
// Arithmetic is attn_fwd_v10's (exact scaling, same MFMA chains and orders,
// same defer-max rule per row), so outputs are bitwise those of variant 55.
//
// hipcc does not see the asm statements as MFMAs or loads, so this file
// carries its own hazard padding (s_nop after MFMA results before VALU or
// accumulator reads, before MFMAs reading freshly written P) and its own LDS
// counts (every LDS access of the loop is asm, in a fixed order).
#include <type_traits>
#include <utility>

#include "flash_v7.h"
#include "pli_common.h"
#ifdef V12_ASM_HDR
#include V12_ASM_HDR  // timing diagnostics only (tools/gen_flash_v12.py V12_MFMA16)
#else
#include "flash_v12_asm.h"
#endif

// A/B switches (tools/build_v12_ab.sh); the defaults are the product
#ifndef V12_DMA_IMM
#define V12_DMA_IMM 1  // LDS-DMA pieces by instruction offset, one M0 write per 4 pieces
#endif
// ablations (timing diagnostics only, results wrong): drop one kind of work
#ifndef V12_ABL_DMA
#define V12_ABL_DMA 0
#endif
#ifndef V12_ABL_EXP
#define V12_ABL_EXP 0
#endif
#ifndef V12_ABL_KREAD
#define V12_ABL_KREAD 0
#endif
#ifndef V12_ABL_SEL
#define V12_ABL_SEL 0
#endif
#ifndef V12_ABL_SETTLE
#define V12_ABL_SETTLE 0
#endif
#ifndef V12_ABL_BAR
#define V12_ABL_BAR 0
#endif
#ifndef V12_ABL_OSTORE
#define V12_ABL_OSTORE 0  // no O stores at block seams
#endif
#ifndef V12_ABL_QLOAD
#define V12_ABL_QLOAD 0  // no Q reload at block seams (the first block's Q reused)
#endif
#ifndef V12_FM_AHEAD
#define V12_FM_AHEAD 1  // each slice's s*c - m a gap pair ahead of its exps
#endif
#ifndef V12_SETTLE2
#define V12_SETTLE2 1  // defer-max decision on half-row maxes, no permlane on the common path
#endif
#ifndef V12_SEL8
#define V12_SEL8 1  // both blocks' row-sum selector MFMAs in one asm statement
#endif
#ifndef V12_UNROLL4
#define V12_UNROLL4 0  // four steps per loop iteration (A/B)
#endif
#ifndef V12_MF16SPLIT
#define V12_MF16SPLIT 0  // timing only (with a V12_MF16SPLIT asm header): each loop MFMA as two 16x16x32, fillers between
#endif
#ifndef V12_SLOT_INC
#define V12_SLOT_INC 0  // 1: ring slots stepped incrementally (no modulo per use): spills (hipcc parks O in a0/a1)
#endif

namespace pli {
namespace {

template <int... I, class Fn>
__device__ __forceinline__ void v12_for(std::integer_sequence<int, I...>, Fn&& fn) {
    (fn(std::integral_constant<int, I>{}), ...);
}
template <int N, class Fn> __device__ __forceinline__ void sfor(Fn&& fn) {
    v12_for(std::make_integer_sequence<int, N>{}, fn);
}

template <int N> __device__ __forceinline__ void lgkm() { asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory"); }

struct V12Frag { i32x2 lo, hi; };

// V^T fragment (two tr-reads); `ro` an immediate byte offset
template <int RO> __device__ __forceinline__ void v12_vread(V12Frag& f, uint32_t alo, uint32_t ahi) {
    asm volatile("ds_read_b64_tr_b16 %0, %2 offset:%4\n\tds_read_b64_tr_b16 %1, %3 offset:%4"
                 : "=&v"(f.lo), "=&v"(f.hi) : "v"(alo), "v"(ahi), "n"(RO) : "memory");
}
// wait until at most N LDS accesses are outstanding; the fragment's registers
// are "written" here as far as hipcc knows, so nothing reads them earlier
template <int N> __device__ __forceinline__ void v12_vwait(V12Frag& f) {
    asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(f.lo), "+v"(f.hi) : "n"(N) : "memory");
}

// row sums: the four selector MFMAs of one block in ONE statement, strictly
// back to back (an MFMA takes the previous result as C without wait states
// only as the very next instruction; an s_nop between them lost a step's sum);
// the leading s_nop covers a hipcc v_mov of l right before the statement, the
// trailing ones a v_mov of the result right after it (4-pass XDL -> VALU)
// LDS accesses issued after V^T fragment I's two reads by the time step I
// waits for it: pre-loop reads V0..V(D-1); step s reads V(s+D) (if < 16) and
// the K fragment s (if KR)
template <int I, bool KR, int D> constexpr int v12_vwait_n() {
    int n = 0;
    bool after = false;
    for (int v = 0; v < D; ++v) {
        if (after) n += 2;
        if (v == I) after = true;
    }
    for (int s = 0; s <= I; ++s) {
        if (s + D < 16) {
            if (after) n += 2;
            if (s + D == I) after = true;
        }
        if (KR && after) n += 1;
    }
    return n;
}

__device__ __forceinline__ void v12_sel4(f32x4& l, i32x4 sel, i32x4 p0, i32x4 p1, i32x4 p2, i32x4 p3) {
    asm volatile("s_nop 2\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0\n\t"
                 "v_mfma_f32_16x16x32_bf16 %0, %1, %3, %0\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %4, %0\n\t"
                 "v_mfma_f32_16x16x32_bf16 %0, %1, %5, %0\n\ts_nop 7\n\ts_nop 2"
                 : "+v"(l) : "v"(sel), "v"(p0), "v"(p1), "v"(p2), "v"(p3));
}

// both blocks' four selector MFMAs in one statement: block B's chain right
// behind block A's (independent accumulators), one set of pads
__device__ __forceinline__ void v12_sel8(f32x4& la, f32x4& lb, i32x4 sel, const i32x4 (&p)[2][2][2]) {
    asm volatile("s_nop 2\n\tv_mfma_f32_16x16x32_bf16 %0, %2, %3, %0\n\t"
                 "v_mfma_f32_16x16x32_bf16 %0, %2, %4, %0\n\tv_mfma_f32_16x16x32_bf16 %0, %2, %5, %0\n\t"
                 "v_mfma_f32_16x16x32_bf16 %0, %2, %6, %0\n\t"
                 "v_mfma_f32_16x16x32_bf16 %1, %2, %7, %1\n\t"
                 "v_mfma_f32_16x16x32_bf16 %1, %2, %8, %1\n\tv_mfma_f32_16x16x32_bf16 %1, %2, %9, %1\n\t"
                 "v_mfma_f32_16x16x32_bf16 %1, %2, %10, %1\n\ts_nop 7\n\ts_nop 2"
                 : "+v"(la), "+v"(lb)
                 : "v"(sel), "v"(p[0][0][0]), "v"(p[0][0][1]), "v"(p[0][1][0]), "v"(p[0][1][1]), "v"(p[1][0][0]),
                   "v"(p[1][0][1]), "v"(p[1][1][0]), "v"(p[1][1][1]));
}

// MFMA results -> VALU reads: 8-pass XDL needs 12 wait states
__device__ __forceinline__ void v12_sfence(f32x16 (&s)[2][2]) {
    asm volatile("s_nop 7\n\ts_nop 4" : "+v"(s[0][0]), "+v"(s[0][1]), "+v"(s[1][0]), "+v"(s[1][1]));
}

__device__ __forceinline__ float v12_xor32_max(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float v12_xor32_sum(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

typedef __attribute__((ext_vector_type(2))) float v12f2;
// defer-max threshold THR (log2 units, a template argument so the shipped
// instantiation's register allocation is not touched): the shipped kernel
// runs 64 since round 4 (8 before; P <= 2^64 is a normal bf16 / fp32 value,
// and the rescale path all but vanishes where the scaled scores spread wide,
// as for v13's offset 62, csrc/flash_attn.hip PLI_V13_MUOFF); variant 72
// (tests only) runs 0, a rescale whenever a tile raises a row's max

#ifdef PLI_FLASH_STAMPS
// diagnostic build only (tools/build_diag.sh): per-segment s_memtime sums
__device__ unsigned long long g_v12_stamps[24];
#endif

// STAMP (diagnostic build only): 0 none, 1 per-segment s_memtime sums, 2 the
// in-kernel clock (s_memtime / s_memrealtime once at entry and exit)
// causal mask of one 32x32 score half in place: element r sits at key
// offset (r&3) + 8(r>>2) of the lane's key group; -inf unless offset <= lim.
// Compare into VCC and select, element by element in asm: hipcc hoists no
// compares (their SGPR masks would not fit beside the kernel's scalars).
template <int R> __device__ __forceinline__ void v12_mask1(f32x16& s, int lim, float ninf) {
    float e = s[R];
    asm volatile("v_cmp_le_i32_e32 vcc, %1, %2\n\tv_cndmask_b32_e32 %0, %3, %0"
                 : "+v"(e) : "n"((R & 3) + 8 * (R >> 2)), "v"(lim), "v"(ninf) : "vcc");
    s[R] = e;
}
template <int... R>
__device__ __forceinline__ void v12_mask_seq(f32x16& s, int lim, float ninf, std::integer_sequence<int, R...>) {
    (v12_mask1<R>(s, lim, ninf), ...);
}
// (-inf comes in a VGPR: a literal beside the VCC read of v_cndmask_b32_e32
// breaks gfx9's one-constant-bus rule)
__device__ __forceinline__ void v12_mask_half(f32x16& s, int lim, float ninf) {
    v12_mask_seq(s, lim, ninf, std::make_integer_sequence<int, 16>{});
}

// Causal block order.  Persistent (G = gridDim.x < nblocks), the pair walk
// (V12_CAUSAL_PAIR 2, the default; the launcher checks QB even, (G/8) %
// (QB/2) == 0, BH % 8 == 0, (BH/8) % ((G/8)/(QB/2)) == 0, nblocks % G == 0
// and nblocks/G even): workgroup i of XCD x owns, at pair step p = j/2 of its
// walk (j = l / G), head x*BH/8 + i/(QB/2) + p*(G/8)/(QB/2) and runs query
// block QB-1-a then a (a = i % (QB/2)) of it.  Every pair is the same work
// (QB+1 key-tile heights), so the QB/2 workgroups of a head stay in step and
// share its K/V in the XCD's L2 -- the long blocks read the same tile at the
// same time, the short ones re-read tiles a few tile-times apart.  B8 H32
// S4096: FETCH 1.33 GB per launch vs 3.94 for the rotation walk below
// (V12_CAUSAL_PAIR 0: QB workgroups run all blocks of one head per step,
// one query height each, but desynchronise as the heights differ), 1049 vs
// 1016 TF/s (profiles/r03/flash/ab_causal_pair.log); short block first
// (V12_CAUSAL_PAIR 1) read 1.9 GB.  One block per workgroup: xcd_remap order,
// the heaviest query block of a head first.
#ifndef V12_CAUSAL_PAIR
#define V12_CAUSAL_PAIR 2
#endif
__device__ __forceinline__ void causal_block(int l, int G, int nblocks, int qb, int& bh, int& qblk) {
#if V12_CAUSAL_PAIR
    if (G < nblocks) {
        const int x = l % 8, wg = (l / 8) % (G / 8), j = l / G, hq = qb / 2;
        const int per = (G / 8) / hq, hx = nblocks / qb / 8, a = wg % hq;
        bh = x * hx + wg / hq + per * (j >> 1);
        qblk = ((j & 1) == (V12_CAUSAL_PAIR == 1 ? 1 : 0)) ? qb - 1 - a : a;
        return;
    }
#endif
    if (G < nblocks) {
        const int x = l % 8, wg = (l / 8) % (G / 8), j = l / G;
        const int per = (G / 8) / qb, hx = nblocks / qb / 8;
        bh = x * hx + wg / qb + per * j;
        qblk = (wg % qb + j) % qb;
    } else {
        const int lb = xcd_remap(l, nblocks);
        bh = lb / qb;
        qblk = qb - 1 - lb % qb;
    }
}

// CAUSAL: the bottom-right mask of ch01/attention.py:66-67 / ch02's cached
// prefill (row i sees keys j <= i + Nk - Nq; the launcher requires Nq <= Nk):
// a block runs only the key tiles its last row sees, the scores of tiles from
// the wave's first masked one on are masked in place (-inf) right after their
// QK^T chains, and the persistent walk is causal_block's pair walk (every
// workgroup the same triangular share).
template <int STAMP = 0, int THR = 64, bool CAUSAL = false>
__global__ __launch_bounds__(256, 1) void attn_fwd_v12(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k, const uint16_t* __restrict__ v,
    uint16_t* __restrict__ o, int H, int group, int Nq, int Nk, V7Strides st, float c, int qblocks,
    int nblocks) {
    constexpr int KT = 64, IMG = KT * 256, BUFB = 2 * IMG, NBUF = 5, PPW = 4;
    __shared__ __attribute__((aligned(1024))) char smem[NBUF * BUFB];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int h32 = lane >> 5, l32 = lane & 31;
    // persistent form: workgroup w walks the blocks w, w + G, w + 2G, ...
    // (G = gridDim.x, a multiple of 8, so every block of one walk stays on
    // the workgroup's XCD and xcd_remap keeps a head's blocks together)
    int L = blockIdx.x, b = 0, hq = 0, q0 = 0;
    const uint16_t *qp = q, *kp = k, *vp = v;
    auto block_ptrs = [&](int l, int& bb, int& hh, int& r0, const uint16_t*& qq, const uint16_t*& kk,
                          const uint16_t*& vv) __attribute__((always_inline)) {
        int bh, qblk;
        if constexpr (CAUSAL) {
            causal_block(l, (int)gridDim.x, nblocks, qblocks, bh, qblk);
        } else {
            const int lb = xcd_remap(l, nblocks);
            bh = lb / qblocks;
            qblk = lb % qblocks;
        }
        bb = bh / H;
        hh = bh % H;
        const int hk = hh / group;
        r0 = qblk * 256 + wave * 64;
        qq = q + bb * st.qb + hh * st.qh;
        kk = k + bb * st.kb + hk * st.kh;
        vv = v + bb * st.vb + hk * st.vh;
    };
    block_ptrs(L, b, hq, q0, qp, kp, vp);
    // key tiles of the block (causal: those its last row sees) and the
    // wave's first tile with a masked score
    auto block_nt = [&](int r0) __attribute__((always_inline)) {
        return CAUSAL ? min(Nk / KT, (r0 - 64 * wave + 256 + Nk - Nq + KT - 1) / KT) : Nk / KT;
    };
    int nt = block_nt(q0);
    int tdiag = CAUSAL ? (q0 + Nk - Nq + 1) / KT : 1 << 30;
    unsigned long long st_sum[20] = {}, st_last = 0;
    auto stamp = [&](int seg) __attribute__((always_inline)) {
        if constexpr (STAMP == 1) {
            unsigned long long now;
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(now)::"memory");
            __builtin_amdgcn_sched_barrier(0);
            if (seg >= 0) st_sum[seg] += now - st_last;
            st_last = now;
        }
    };
    stamp(-1);
    unsigned long long clk_t0 = 0, clk_r0 = 0;
    if constexpr (STAMP == 2)
        asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(clk_t0), "=s"(clk_r0)::"memory");

    // ---- LDS-DMA plan (attn_fwd_v10's, 4 waves: 4 K + 4 V pieces per wave)
    auto fsw = [](int row) __attribute__((always_inline)) { return ((row & 3) << 2) | ((row >> 2) & 3); };
    uint32_t koff[PPW], voff[PPW];
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
        const int drow = 4 * (PPW * wave + i) + (lane >> 4);
        const int ch = (lane & 15) ^ fsw(drow);
        // V12_DMA_IMM: piece i reaches its LDS quarter through the
        // instruction offset i * 1024, which the hardware adds to the global
        // address too -- bias the source offset by -i * 1024 (drow >= 4i and
        // a row is >= 256 B, so the offset stays >= 0)
        koff[i] = (uint32_t)(drow * (int)st.kn + 8 * ch) * 2u - (V12_DMA_IMM ? 1024u * i : 0u);
        voff[i] = (uint32_t)(drow * (int)st.vn + 8 * ch) * 2u - (V12_DMA_IMM ? 1024u * i : 0u);
    }
#if V12_DMA_IMM
    // one M0 per group of four pieces (a tile's K or V quarter of this wave):
    // piece 0 of a group writes M0, pieces 1-3 reach their LDS quarter by the
    // instruction offset.  hipcc itself never touches M0 in this kernel (the
    // CPU build test checks it), so M0 is not saved or restored.
    auto dma_first = [&](const uint16_t* tbase, uint32_t off, uint32_t lds) __attribute__((always_inline)) {
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(lds), "v"(off),
                     "s"(tbase) : "memory");
    };
    auto dma_next = [&](auto i_tag, const uint16_t* tbase, uint32_t off) __attribute__((always_inline)) {
        asm volatile("global_load_lds_dwordx4 %0, %1 offset:%2" ::"v"(off), "s"(tbase),
                     "n"(1024 * decltype(i_tag)::value) : "memory");
    };
#else
    auto dma = [&](const uint16_t* tbase, uint32_t off, uint32_t lds) __attribute__((always_inline)) {
        uint32_t keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %3\n\t"
                     "s_mov_b32 m0, %0"
                     : "=&s"(keep) : "s"(lds), "v"(off), "s"(tbase) : "memory");
    };
#endif
    const uint32_t lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem;
    // DMA piece j of a tile: V12_DMA_IMM K pieces 0-3 then V pieces 0-3;
    // else even j K piece j/2, odd j V piece j/2
    auto dma_piece = [&](auto j_tag, const uint16_t* kt, const uint16_t* vt, uint32_t base) __attribute__((always_inline)) {
        constexpr int j = decltype(j_tag)::value;
#if V12_DMA_IMM
        constexpr int i = j % 4;
        const uint16_t* src = j < 4 ? kt : vt;
        const uint32_t off = j < 4 ? koff[i] : voff[i];
        if constexpr (i == 0) dma_first(src, off, base + (j < 4 ? 0 : IMG));
        else dma_next(std::integral_constant<int, i>{}, src, off);
#else
        if constexpr (j % 2 == 0) dma(kt, koff[j / 2], base + (j / 2) * 1024);
        else dma(vt, voff[j / 2], base + IMG + (j / 2) * 1024);
#endif
    };
    auto dma_tile = [&](int t, int slot) __attribute__((always_inline)) {
        const uint16_t* kt = kp + (int64_t)t * KT * st.kn;
        const uint16_t* vt = vp + (int64_t)t * KT * st.vn;
        const uint32_t base = lds0 + slot * BUFB + (PPW * wave) * 1024;
        sfor<8>([&](auto J) { dma_piece(J, kt, vt, base); });
    };

    // ---- tiles 0 and 1 in flight first, then the Q^T fragments (VGPRs;
    // into the accumulators at the block's prologue)
    if (nt > 0) dma_tile(0, 0);
    if (nt > 1) dma_tile(1, 1);
    i32x4 qa[8], qb[8];
    auto load_q = [&](const uint16_t* qbase, int r0) __attribute__((always_inline)) {
        const int ra = r0 + l32, rb = r0 + 32 + l32;
        const uint16_t* sa = qbase + (int64_t)(ra < Nq ? ra : 0) * st.qn + 8 * h32;
        const uint16_t* sb = qbase + (int64_t)(rb < Nq ? rb : 0) * st.qn + 8 * h32;
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
            qa[kk] = *reinterpret_cast<const i32x4*>(sa + 16 * kk);
            qb[kk] = *reinterpret_cast<const i32x4*>(sb + 16 * kk);
        }
    };
    load_q(qp, q0);

    // ---- fragment addresses (LDS byte addresses; + slot * BUFB per tile)
    const int A0 = l32 * 256 + ((h32 ^ fsw(l32)) << 4);
    uint32_t kaddr[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) kaddr[kk] = lds0 + (uint32_t)(A0 ^ (kk << 5));
    const int g = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;
    const int c0 = 2 * (g & 1) + (pp >> 1);
    const int B0 = IMG + (4 * h32 + qq) * 256 + ((c0 ^ ((qq << 2) | h32)) << 4) + 8 * (pp & 1);
    uint32_t valo[4], vahi[4];
#pragma unroll
    for (int db = 0; db < 4; ++db) {
        const int alo = B0 ^ (db << 6);
        valo[db] = lds0 + (uint32_t)alo;
        vahi[db] = lds0 + (uint32_t)((alo ^ 32) + 2048);
    }
    const bool sel_on = (i16 == 0 && (g & 1) == 0) || (i16 == 4 && (g & 1) == 1);
    const int one = sel_on ? 0x3F803F80 : 0;
    const i32x4 sel = {one, one, one, one};

    float mA = -1e30f, mB = -1e30f;
    f32x4 lA = {0.f, 0.f, 0.f, 0.f}, lB = {0.f, 0.f, 0.f, 0.f};
    // stream position: the block's tile t sits in LDS slot (s0 + t) % NBUF
    int s0 = 0;
    bool has_next = false;
    f32x16 S[2][2];               // [block][key half]: one tile's scores
    i32x4 P0[2][2][2], P1[2][2][2];  // [block][key half][16-key step]; tile t in P(t&1)
    float mxA = -INFINITY, mxB = -INFINITY;

    // ---- softmax slice i (elements 2i, 2i+1 of a lane's row) of block X as
    // five single-issue stages placed one by one into MFMA gaps: MX (running
    // max), FM (two v_fma_f32: s*c - m; v_pk_fma_f32 costs ~22 cycles more
    // beside an MFMA), E0 / E1 (one v_exp_f32 each: at most one 8-cycle
    // instruction per gap), CV (packed bf16 pair into P).  Each result is
    // pinned where it is made (an empty volatile asm), or hipcc sinks the
    // exps to their use in the next tile's PV.
    v12f2 sy[2][4], se[2][4];
    auto opMX = [&](auto x_tag, auto i_tag) __attribute__((always_inline)) {
        constexpr int X = decltype(x_tag)::value, i = decltype(i_tag)::value, tt = i / 8, r = 2 * (i % 8);
        float& mx = X == 0 ? mxA : mxB;
        mx = max3(mx, S[X][tt][r], S[X][tt][r + 1]);
        asm volatile("" : "+v"(mx));
    };
    auto opFM = [&](auto x_tag, auto i_tag) __attribute__((always_inline)) {
        constexpr int X = decltype(x_tag)::value, i = decltype(i_tag)::value, tt = i / 8, r = 2 * (i % 8);
        const float m = X == 0 ? mA : mB;
        const float s0 = S[X][tt][r], s1 = S[X][tt][r + 1], cc = c;
        float y0, y1;
        asm volatile("v_fma_f32 %0, %2, %4, -%5\n\tv_fma_f32 %1, %3, %4, -%5"
                     : "=&v"(y0), "=&v"(y1) : "v"(s0), "v"(s1), "v"(cc), "v"(m));
        sy[X][i % 4] = v12f2{y0, y1};
    };
    auto opE = [&](auto x_tag, auto i_tag, auto h_tag) __attribute__((always_inline)) {
        constexpr int X = decltype(x_tag)::value, i = decltype(i_tag)::value, h = decltype(h_tag)::value;
        if constexpr (h == 0) {
            se[X][i % 4].x = V12_ABL_EXP ? sy[X][i % 4].x : __builtin_amdgcn_exp2f(sy[X][i % 4].x);
            asm volatile("" : "+v"(se[X][i % 4].x));
        } else {
            se[X][i % 4].y = V12_ABL_EXP ? sy[X][i % 4].y : __builtin_amdgcn_exp2f(sy[X][i % 4].y);
            asm volatile("" : "+v"(se[X][i % 4].y));
        }
    };
    auto opCV = [&](auto x_tag, auto i_tag, i32x4 (&Pc)[2][2][2]) __attribute__((always_inline)) {
        constexpr int X = decltype(x_tag)::value, i = decltype(i_tag)::value;
        constexpr int tt = i / 8, s2 = (i % 8) / 4, j = i % 4;
        Pc[X][tt][s2][j] = (int)pack2<bf16_t>(se[X][i % 4].x, se[X][i % 4].y);
        asm volatile("" : "+v"(Pc[X][tt][s2]));
    };
    using X0 = std::integral_constant<int, 0>;
    using X1 = std::integral_constant<int, 1>;
    using H0 = std::integral_constant<int, 0>;
    using H1 = std::integral_constant<int, 1>;
    // slice stream: slice I0 + a over gaps 2a (FM, E0) and 2a + 1 (E1, CV of
    // the slice before); gap g of the stream.  The CV of the stream's last
    // slice is left to the caller.
    auto stream = [&](auto x_tag, auto i0_tag, auto g_tag, i32x4 (&Pc)[2][2][2]) __attribute__((always_inline)) {
        constexpr int g = decltype(g_tag)::value, I0 = decltype(i0_tag)::value, i = I0 + g / 2;
        if constexpr (g % 2 == 0) {
#if V12_FM_AHEAD
            // the FM of slice i was issued a gap pair earlier (by the caller
            // for the stream's first slice): hipcc pads any instruction that
            // reads an asm statement's result right after it with s_nop 0
            // (it cannot tell the asm is no transcendental), so the exp
            // never follows its own FM
            opE(x_tag, std::integral_constant<int, i>{}, H0{});
            if constexpr (g / 2 + 1 < 8) opFM(x_tag, std::integral_constant<int, i + 1>{});
#else
            opFM(x_tag, std::integral_constant<int, i>{});
            opE(x_tag, std::integral_constant<int, i>{}, H0{});
#endif
        } else {
            opE(x_tag, std::integral_constant<int, i>{}, H1{});
            if constexpr (g > 1) opCV(x_tag, std::integral_constant<int, i - 1>{}, Pc);
        }
    };
    // V12_FM_AHEAD: the first slice's FM of a stream, ahead of the phase's
    // first MFMA
    auto prefm = [&](auto x_tag, auto i_tag) __attribute__((always_inline)) {
        if constexpr (V12_FM_AHEAD) {
            opFM(x_tag, i_tag);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    // VALU-written P -> MFMA operands: pin P here and pad
    auto pfence = [&](i32x4 (&Pc)[2][2][2]) __attribute__((always_inline)) {
        asm volatile("s_nop 1" : "+v"(Pc[0][0][0]), "+v"(Pc[0][0][1]), "+v"(Pc[0][1][0]), "+v"(Pc[0][1][1]),
                     "+v"(Pc[1][0][0]), "+v"(Pc[1][0][1]), "+v"(Pc[1][1][0]), "+v"(Pc[1][1][1]));
    };
    // exps (current m) and P of every element of S (first tile, rare path)
    auto expo_cvt_all = [&](i32x4 (&Pc)[2][2][2]) __attribute__((always_inline)) {
        sfor<16>([&](auto I) {
            constexpr int i = I;
            constexpr int tt = i / 8, r = 2 * (i % 8), s2 = (i % 8) / 4, j = i % 4;
#pragma unroll
            for (int X = 0; X < 2; ++X) {
                const float m = X == 0 ? mA : mB;
                const v12f2 y = __builtin_elementwise_fma(v12f2{S[X][tt][r], S[X][tt][r + 1]}, v12f2{c, c},
                                                          v12f2{-m, -m});
                Pc[X][tt][s2][j] = (int)pack2<bf16_t>(__builtin_amdgcn_exp2f(y.x), __builtin_amdgcn_exp2f(y.y));
            }
        });
    };
    // block B's slices 8..15 (key half 1) of a tile, no MFMAs (epilogue)
    auto tailB = [&](i32x4 (&Pc)[2][2][2]) __attribute__((always_inline)) {
        sfor<8>([&](auto A) {
            constexpr int i = 8 + A;
            opFM(X1{}, std::integral_constant<int, i>{});
            opE(X1{}, std::integral_constant<int, i>{}, H0{});
            opE(X1{}, std::integral_constant<int, i>{}, H1{});
            opCV(X1{}, std::integral_constant<int, i>{}, Pc);
        });
    };

    // phase QA: block A's QK^T chains (16 MFMAs); beside them block B's slices
    // 8..15 of the previous tile (m already settled) into Pp, and the 8 DMA
    // pieces of a tile two ahead (one per odd gap)
    auto phaseQA = [&](i32x4 (&Pp)[2][2][2], auto sm_tag, const uint16_t* kt, const uint16_t* vt, uint32_t dbase)
        __attribute__((always_inline)) {
        constexpr bool SM = decltype(sm_tag)::value;
        if constexpr (SM) prefm(X1{}, std::integral_constant<int, 8>{});
        sfor<16>([&](auto FF) {
            constexpr int F = FF;
#if V12_MF16SPLIT
            v12::qk1h<F, 0, 0>(S[0][F / 8]);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (SM) stream(X1{}, std::integral_constant<int, 8>{}, FF, Pp);
            __builtin_amdgcn_sched_barrier(0);
            v12::qk1h<F, 0, 1>(S[0][F / 8]);
#else
            v12::qk1<F, 0>(S[0][F / 8]);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (SM) stream(X1{}, std::integral_constant<int, 8>{}, FF, Pp);
#endif
            if constexpr (F % 2 == 1 && !V12_ABL_DMA) dma_piece(std::integral_constant<int, F / 2>{}, kt, vt, dbase);
            __builtin_amdgcn_sched_barrier(0);
        });
    };
    // V^T fragments of d-block db of the tile at LDS byte offset vs: fragment
    // k is two tr-reads
    V12Frag vf[2][4];
    auto vread1 = [&](auto db_tag, auto k_tag, uint32_t vs) __attribute__((always_inline)) {
        constexpr int db = decltype(db_tag)::value, k = decltype(k_tag)::value;
        v12_vread<((k / 2) * 32 + 16 * (k & 1)) * 256>(vf[db & 1][k], valo[db] + vs, vahi[db] + vs);
    };
    // phase QB: block B's QK^T chains (16 MFMAs); beside them the last P pair
    // of phase QA, block A's slices 0..7 (key half 0, written 8 MFMAs ago),
    // the running max over key half 1 (odd gaps) and (VR) the V^T d-block 0
    // fragments of the tile in slot sv for the next phase P (gaps 1, 3, 5, 7)
    auto phaseQB = [&](i32x4 (&Pp)[2][2][2], i32x4 (&Pc)[2][2][2], auto sm_tag, int sv) __attribute__((always_inline)) {
        constexpr bool SM = decltype(sm_tag)::value;
        const uint32_t vs = (uint32_t)sv * BUFB;
        mxA = -INFINITY;
        if constexpr (SM) prefm(X0{}, std::integral_constant<int, 0>{});
        sfor<16>([&](auto FF) {
            constexpr int F = FF;
#if V12_MF16SPLIT
            v12::qk1h<F, 1, 0>(S[1][F / 8]);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (SM) {
                if constexpr (F == 0) opCV(X1{}, std::integral_constant<int, 15>{}, Pp);
                if constexpr (F % 2 == 0) opMX(X0{}, std::integral_constant<int, F / 2>{});
                else opMX(X0{}, std::integral_constant<int, 8 + F / 2>{});
            }
            __builtin_amdgcn_sched_barrier(0);
            v12::qk1h<F, 1, 1>(S[1][F / 8]);
#else
            v12::qk1<F, 1>(S[1][F / 8]);
#endif
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (SM) {
#if !V12_MF16SPLIT
                if constexpr (F == 0) opCV(X1{}, std::integral_constant<int, 15>{}, Pp);
                if constexpr (F % 2 == 0) opMX(X0{}, std::integral_constant<int, F / 2>{});
                else opMX(X0{}, std::integral_constant<int, 8 + F / 2>{});
#endif
                stream(X0{}, std::integral_constant<int, 0>{}, FF, Pc);
                if constexpr (F % 2 == 1 && F < 8)
                    vread1(std::integral_constant<int, 0>{}, std::integral_constant<int, F / 2>{}, vs);
            }
            __builtin_amdgcn_sched_barrier(0);
        });
    };

    // phase P: PV of the tile in slot sv with Pv (PV) as 8 accumulator chains
    // of 4 (d-block major: O_A[db] then O_B[db], sharing db's 4 V^T fragments,
    // the next d-block's fragments read under the current chains); beside them
    // (SM) block A's slices 8..15, block B's running max and slices 0..7 into
    // Pc, one stage per gap, and the K fragments of the tile in slot sk into
    // AGPR (KR, 4 per d-block)
    auto phaseP = [&](int sv, i32x4 (&Pv)[2][2][2], i32x4 (&Pc)[2][2][2], int sk, auto pv_tag,
                      auto sm_tag, auto kr_tag, auto vpre_tag) __attribute__((always_inline)) {
        constexpr bool PV = decltype(pv_tag)::value, SM = decltype(sm_tag)::value, KR = decltype(kr_tag)::value;
        constexpr bool VPRE = decltype(vpre_tag)::value;  // d-block 0 fragments already issued (phase QB)
        const uint32_t vs = (uint32_t)sv * BUFB, ks = (uint32_t)sk * BUFB;
        mxB = -INFINITY;
        if constexpr (SM) prefm(X0{}, std::integral_constant<int, 8>{});
        if constexpr (PV && !VPRE)
            sfor<4>([&](auto KS) { vread1(std::integral_constant<int, 0>{}, KS, vs); });
        sfor<4>([&](auto DBB) {
            constexpr int db = DBB;
            if constexpr (PV) {
                // d-block db's 8 reads were issued before the K reads of the
                // previous d-block's gaps 4..7
                constexpr int N = (KR && db > 0) ? 4 : 0;
                V12Frag* f = vf[db & 1];
                asm volatile("s_waitcnt lgkmcnt(%8)"
                             : "+v"(f[0].lo), "+v"(f[0].hi), "+v"(f[1].lo), "+v"(f[1].hi), "+v"(f[2].lo),
                               "+v"(f[2].hi), "+v"(f[3].lo), "+v"(f[3].hi)
                             : "n"(N) : "memory");
            }
            sfor<8>([&](auto JJ) {
                constexpr int j = JJ, X = j / 4, k = j % 4, slot = 8 * db + j;
#if V12_MF16SPLIT
                if constexpr (PV) {
                    const V12Frag& ff = vf[db & 1][k];
                    v12::pv1h<X, db, 0>(i32x4{ff.lo.x, ff.lo.y, ff.hi.x, ff.hi.y}, Pv[X][k / 2][k & 1]);
                }
                __builtin_amdgcn_sched_barrier(0);
                if constexpr (PV && j < 4 && db + 1 < 4)
                    vread1(std::integral_constant<int, db + 1>{}, std::integral_constant<int, j>{}, vs);
                if constexpr (KR && j >= 4 && !V12_ABL_KREAD) v12::kread<4 * db + j - 4>(kaddr[(4 * db + j - 4) % 8] + ks);
                __builtin_amdgcn_sched_barrier(0);
                if constexpr (PV) {
                    const V12Frag& ff = vf[db & 1][k];
                    v12::pv1h<X, db, 1>(i32x4{ff.lo.x, ff.lo.y, ff.hi.x, ff.hi.y}, Pv[X][k / 2][k & 1]);
                }
                __builtin_amdgcn_sched_barrier(0);
#else
                if constexpr (PV) {
                    const V12Frag& ff = vf[db & 1][k];
                    v12::pv1<X, db>(i32x4{ff.lo.x, ff.lo.y, ff.hi.x, ff.hi.y}, Pv[X][k / 2][k & 1]);
                }
                __builtin_amdgcn_sched_barrier(0);
                // gaps 0..3: the next d-block's fragment j; gaps 4..7: K fragment
                if constexpr (PV && j < 4 && db + 1 < 4)
                    vread1(std::integral_constant<int, db + 1>{}, std::integral_constant<int, j>{}, vs);
                if constexpr (KR && j >= 4 && !V12_ABL_KREAD) v12::kread<4 * db + j - 4>(kaddr[(4 * db + j - 4) % 8] + ks);
#endif
                if constexpr (SM) {
                    if constexpr (slot == 0) opCV(X0{}, std::integral_constant<int, 7>{}, Pc);
                    if constexpr (slot % 2 == 1) opMX(X1{}, std::integral_constant<int, slot / 2>{});
                    if constexpr (slot < 16) {
                        stream(X0{}, std::integral_constant<int, 8>{}, std::integral_constant<int, slot>{}, Pc);
                        if constexpr (V12_FM_AHEAD && slot == 14) opFM(X1{}, std::integral_constant<int, 0>{});
                    } else {
                        if constexpr (slot == 16) opCV(X0{}, std::integral_constant<int, 15>{}, Pc);
                        stream(X1{}, std::integral_constant<int, 0>{}, std::integral_constant<int, slot - 16>{}, Pc);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
            });
        });
        if constexpr (SM) opCV(X1{}, std::integral_constant<int, 7>{}, Pc);
        if constexpr (PV) {
            if (!V12_ABL_SEL) {
#if V12_SEL8
                v12_sel8(lA, lB, sel, Pv);
#else
                v12_sel4(lA, sel, Pv[0][0][0], Pv[0][0][1], Pv[0][1][0], Pv[0][1][1]);
                v12_sel4(lB, sel, Pv[1][0][0], Pv[1][0][1], Pv[1][1][0], Pv[1][1][1]);
#endif
            }
        }
        if constexpr (SM && !V12_SETTLE2) {
            mxA = v12_xor32_max(mxA);
            mxB = v12_xor32_max(mxB);
        }
    };

    // defer-max decision for the tile in S (rare path: drain, rescale O and
    // l, recompute S from the LDS copy of K in slot sk, redo exps and P; block
    // B's slices 8..15, still to come, then use the new m)
    // CAUSAL: block X's scores of tile t in place, key > row + Nk - Nq ->
    // -inf (element r of half tt is key 64t + 32tt + (r&3) + 8(r>>2) + 4h32
    // of row q0 + 32X + l32); the MFMA results are padded first
    auto mask_block = [&](auto x_tag, int t) __attribute__((always_inline)) {
        if constexpr (CAUSAL) {
            constexpr int X = decltype(x_tag)::value;
            asm volatile("s_nop 7\n\ts_nop 4" : "+v"(S[X][0]), "+v"(S[X][1]));
            // the lane id re-derived here (opaque asm): nothing lane-dependent
            // stays live through the loop for the mask
            int ln;
            asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
            const int base = (ln & 31) - 4 * (ln >> 5) + (q0 + 32 * X + Nk - Nq - KT * t);
            const float ninf = -INFINITY;
            v12_mask_half(S[X][0], base, ninf);
            v12_mask_half(S[X][1], base - 32, ninf);
        }
    };
    auto settle = [&](i32x4 (&Pc)[2][2][2], int sk, int t, bool msk) __attribute__((always_inline)) {
#if V12_SETTLE2
        // V12_SETTLE2: decided on each lane's HALF-row maxes (lanes l and
        // l^32 hold the two key halves of a row): fl(x*c) is non-decreasing
        // in x, so some half's max*c exceeds m + THR exactly when the full
        // row's does -- the same decision with no permlane merge, two
        // compares and one SGPR test; the merge runs on the rare path
        // mxA / mxB are scaled in place (fl(max * c) = max of fl(half * c)),
        // one temporary for the thresholds: the allocation has no room
        float tq;
        uint64_t hit;
        static_assert(THR == 0 || THR == 8 || THR == 64, "threshold literal");
#define V12_SETTLE_ASM(T)                                                                                      \
    asm volatile("v_mul_f32 %0, %0, %4\n\tv_mul_f32 %1, %1, %4\n\tv_add_f32 %2, " T ", %5\n\t"              \
                 "v_cmp_gt_f32_e64 %3, %0, %2\n\tv_add_f32 %2, " T ", %6\n\tv_cmp_gt_f32_e64 vcc, %1, %2\n\t" \
                 "s_or_b64 %3, %3, vcc"                                                                        \
                 : "+v"(mxA), "+v"(mxB), "=&v"(tq), "=&s"(hit)                                                  \
                 : "v"(c), "v"(mA), "v"(mB) : "vcc", "scc")
        if constexpr (THR == 64) V12_SETTLE_ASM("0x42800000");
        else if constexpr (THR == 8) V12_SETTLE_ASM("0x41000000");
        else V12_SETTLE_ASM("0");
#undef V12_SETTLE_ASM
        if (__builtin_expect(hit != 0, 0)) {
            mxA = v12_xor32_max(mxA);  // now the full rows' scaled maxes
            mxB = v12_xor32_max(mxB);
            const bool upA = mxA > mA + (float)THR, upB = mxB > mB + (float)THR;
            asm volatile("s_nop 7\n\ts_nop 7" : "+v"(lA), "+v"(lB));
            const float nA = upA ? mxA : mA, nB = upB ? mxB : mB;
#else
        const bool upA = mxA * c > mA + (float)THR, upB = mxB * c > mB + (float)THR;
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(upA || upB) != 0, 0)) {
            asm volatile("s_nop 7\n\ts_nop 7" : "+v"(lA), "+v"(lB));
            const float nA = upA ? mxA * c : mA, nB = upB ? mxB * c : mB;
#endif
            const float alA = __builtin_amdgcn_exp2f(mA - nA), alB = __builtin_amdgcn_exp2f(mB - nB);
            mA = nA;
            mB = nB;
            v12::o_scale(alA, alB);
            lA[0] *= alA;
            lB[0] *= alB;
            const char* kb = smem + sk * BUFB;
#pragma unroll
            for (int tt = 0; tt < 2; ++tt)
                sfor<8>([&](auto KK) {
                    const i32x4 kf = lds_read_b128(kb, (A0 ^ (KK << 5)) + tt * 8192);
                    v12::qk_v<0, KK>(S[0][tt], kf);
                    v12::qk_v<1, KK>(S[1][tt], kf);
                });
            v12_sfence(S);
            if (msk) {
                mask_block(X0{}, t);
                mask_block(X1{}, t);
            }
            expo_cvt_all(Pc);
            pfence(Pc);
        }
    };

    if (nt <= 0) return;  // host guarantees Nk >= 64
    // K/V source of the stream tile t+2 positions ahead of this block's tile
    // t: this block, the next block's tile 0 or 1 (persistent), or past the
    // last block a reload of tile nt-1 (keeps the vmcnt count constant)
    auto dma_src = [&](int t2, const uint16_t*& kt, const uint16_t*& vt) __attribute__((always_inline)) {
        if (__builtin_expect(t2 < nt, 1)) {
            kt = kp + (int64_t)t2 * KT * st.kn;
            vt = vp + (int64_t)t2 * KT * st.vn;
        } else if (has_next) {  // recomputed here: fewer scalars live through the block
            int b2, h2, r2;
            const uint16_t *q2, *k2, *v2;
            block_ptrs(L + (int)gridDim.x, b2, h2, r2, q2, k2, v2);
            kt = k2 + (int64_t)(t2 - nt) * KT * st.kn;
            vt = v2 + (int64_t)(t2 - nt) * KT * st.vn;
        } else {
            kt = kp + (int64_t)(nt - 1) * KT * st.kn;
            vt = vp + (int64_t)(nt - 1) * KT * st.vn;
        }
    };
    auto slot = [&](int t) __attribute__((always_inline)) { return (s0 + t) % NBUF; };

    // tile t: S(t) and P(t) in Pc = P(t&1); PV of tile t-1 from Pv.  LDS ring
    // of 5 slots, stream tile u in slot u % 5: the DMA of the stream tile two
    // ahead goes out during phase QA(t) into the slot of stream tile u-3
    // (= u+2-NBUF),
    // whose last reader (PV(u-3) in phase P(u-2)) every wave has passed at
    // barrier(u-1); the counted vmcnt(8) before barrier(u) retires tile u+1
    // and leaves u+2 in flight.  Across a block seam the stream continues
    // (the next block's tiles 0 and 1 are DMA'd by this block's last steps).
    // V12_SLOT_INC: the step carries slot(t-1) in `sm1` and steps it by one
    // (wrap at NBUF) instead of a modulo per use
    int sm1 = 0;
    auto inc_slot = [](int x) __attribute__((always_inline)) { return x == NBUF - 1 ? 0 : x + 1; };
    // causal: from the wave's tdiag on, the scores are masked in place right
    // after each block's QK^T chain (a uniform branch; compiled out of the
    // non-causal kernel)
    auto step = [&](int t, i32x4 (&Pc)[2][2][2], i32x4 (&Pv)[2][2][2]) __attribute__((always_inline)) {
        const bool msk = CAUSAL && t >= tdiag;
#if V12_SLOT_INC
        const int s_m1 = sm1, s_0 = inc_slot(s_m1), s_p1 = inc_slot(s_0), s_p2 = inc_slot(s_p1);
        sm1 = s_0;
#else
        const int s_m1 = slot(t - 1), s_0 = slot(t), s_p1 = slot(t + 1), s_p2 = slot(t + 2);
#endif
        stamp(6);
        lgkm<0>();  // K(t) fragments in AGPR
        stamp(0);
        {
            const uint16_t *kt, *vt;
            dma_src(t + 2, kt, vt);
            const uint32_t dbase = lds0 + (uint32_t)s_p2 * BUFB + (PPW * wave) * 1024;
            phaseQA(Pv, std::true_type{}, kt, vt, dbase);
            if (msk) mask_block(X0{}, t);
            phaseQB(Pv, Pc, std::true_type{}, s_m1);
            if (msk) mask_block(X1{}, t);
        }
        stamp(1);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // tile t+1 (issued one step ago)
        stamp(2);
        if (!V12_ABL_BAR) __syncthreads();
        stamp(3);
        asm volatile("s_nop 1" ::: "memory");  // P just written -> MFMA operands
        // K(t+1) fragments; past the last tile they read a stale slot (never
        // used) -- one instantiation, so no branch between phase QB's V^T reads
        // and their use here (at a branch hipcc may copy the not-yet-landed
        // fragment registers)
        phaseP(s_m1, Pv, Pc, s_p1, std::true_type{}, std::true_type{}, std::true_type{}, std::true_type{});
        stamp(4);
        if (!V12_ABL_SETTLE) settle(Pc, s_0, t, msk);
        stamp(5);
    };

    int nblk = 0;  // blocks walked
    for (;;) {
        ++nblk;
        has_next = L + (int)gridDim.x < nblocks;

        // ---- prologue: tiles 0 and 1 (and Q) landed, Q -> AGPR, O = 0, K(0)
        // fragments, S(0), the stream tile two ahead's DMA beside block A's
        // chains, softmax(0), K(1) fragments
        // Past the first block, tile 0 landed at the previous block's last
        // barrier: O = 0 and the K(0) reads go ahead of the wait for the Q
        // rows (issued under the previous epilogue) and the O stores.
        const uint32_t ks0 = (uint32_t)slot(0) * BUFB;
        if (nblk > 1) {
            v12::o_zero();
            sfor<16>([&](auto FF) { v12::kread<FF>(kaddr[FF % 8] + ks0); });
        }
        stamp(8);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        stamp(9);
        __syncthreads();
        if (nblk == 1) {
            v12::o_zero();
            sfor<16>([&](auto FF) { v12::kread<FF>(kaddr[FF % 8] + ks0); });
        }
        sfor<8>([&](auto KK) {
            v12::q_to_agpr<0, KK>(qa[KK]);
            v12::q_to_agpr<1, KK>(qb[KK]);
        });
        asm volatile("s_nop 2" ::: "memory");  // accvgpr writes -> MFMA operands
        mA = -1e30f;
        mB = -1e30f;
        lA = f32x4{0.f, 0.f, 0.f, 0.f};
        lB = f32x4{0.f, 0.f, 0.f, 0.f};
        // hipcc does not know the row-sum asm MFMAs read l as C: materialise
        // the zeros here, wait states after (VALU write -> MFMA source)
        asm volatile("s_nop 2" : "+v"(lA), "+v"(lB));
        lgkm<0>();
        stamp(10);
        {
            const uint16_t *kt, *vt;
            dma_src(2, kt, vt);
            const uint32_t dbase = lds0 + (uint32_t)slot(2) * BUFB + (PPW * wave) * 1024;
            phaseQA(P1, std::false_type{}, kt, vt, dbase);
            phaseQB(P1, P0, std::false_type{}, 0);
        }
        asm volatile("s_nop 7\n\ts_nop 4" : "+v"(S[0][0]), "+v"(S[0][1]), "+v"(S[1][0]), "+v"(S[1][1]));
        if (CAUSAL && 0 >= tdiag) {  // tile 0 holds the diagonal (first query block)
            mask_block(X0{}, 0);
            mask_block(X1{}, 0);
        }
        stamp(11);
        if (nt > 1)
            phaseP(0, P1, P1, slot(1), std::false_type{}, std::false_type{}, std::true_type{}, std::false_type{});
        {   // first tile: the max decides m before any exp
            mxA = -INFINITY;
            mxB = -INFINITY;
#pragma unroll
            for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                for (int r = 0; r < 16; r += 2) {
                    mxA = max3(mxA, S[0][tt][r], S[0][tt][r + 1]);
                    mxB = max3(mxB, S[1][tt][r], S[1][tt][r + 1]);
                }
            mxA = v12_xor32_max(mxA);
            mxB = v12_xor32_max(mxB);
            mA = mxA == -INFINITY ? -1e30f : mxA * c;
            mB = mxB == -INFINITY ? -1e30f : mxB * c;
            expo_cvt_all(P0);
            pfence(P0);
        }

        stamp(6);
        sm1 = s0;  // slot(0): tile t-1 of the first step
        int t = 1;
#if V12_UNROLL4
        for (; t + 3 < nt; t += 4) {
            step(t, P1, P0);
            step(t + 1, P0, P1);
            step(t + 2, P1, P0);
            step(t + 3, P0, P1);
        }
#endif
        for (; t + 1 < nt; t += 2) {
            step(t, P1, P0);
            step(t + 1, P0, P1);
        }
        if (t < nt) step(t, P1, P0);

        stamp(12);
        // the next block's Q rows, in flight under this block's epilogue
        // (past the last block a reload of this block's: unconditional, so
        // the old fragments are not kept live through the block)
        if (!V12_ABL_QLOAD) {
            int b2, h2, r2;
            const uint16_t *q2, *k2, *v2;
            block_ptrs(has_next ? L + (int)gridDim.x : L, b2, h2, r2, q2, k2, v2);
            load_q(q2, r2);
        }
        stamp(14);

        // ---- epilogue: block B's slices 8..15 and PV of the last tile, l, O
        // read-out and store.  The V^T addresses are made opaque here, or
        // hipcc precomputes the epilogue's slot addresses before the loop and
        // parks them in accumulator registers it thinks are free (the Q
        // fragments).
#pragma unroll
        for (int db = 0; db < 4; ++db) asm volatile("" : "+v"(valo[db]), "+v"(vahi[db]));
        if ((nt - 1) & 1) { tailB(P1); pfence(P1); }
        else { tailB(P0); pfence(P0); }
        stamp(15);
        if ((nt - 1) & 1)
            phaseP(slot(nt - 1), P1, P1, 0, std::true_type{}, std::false_type{}, std::false_type{}, std::false_type{});
        else
            phaseP(slot(nt - 1), P0, P0, 0, std::true_type{}, std::false_type{}, std::false_type{}, std::false_type{});
        stamp(16);
        asm volatile("s_nop 15\n\ts_nop 7" : "+v"(lA), "+v"(lB));
        const float invA = [&] { const float l = v12_xor32_sum(lA[0]); return l > 0.f ? 1.f / l : 0.f; }();
        const float invB = [&] { const float l = v12_xor32_sum(lB[0]); return l > 0.f ? 1.f / l : 0.f; }();
        auto store = [&](auto x_tag, float inv) __attribute__((always_inline)) {
            constexpr int X = decltype(x_tag)::value;
            const int qr = q0 + 32 * X + l32;
            sfor<4>([&](auto DB) {
                f32x16 a;
                v12::o_read<X, DB>(a);
                if (qr < Nq && (!V12_ABL_OSTORE || !has_next)) {
                    uint16_t* op = o + b * st.ob + hq * st.oh + (int64_t)qr * st.on;
#pragma unroll
                    for (int i = 0; i < 4; i += 2) {
                        const uint32_t ax = pack2<bf16_t>(a[4 * i] * inv, a[4 * i + 1] * inv);
                        const uint32_t ay = pack2<bf16_t>(a[4 * i + 2] * inv, a[4 * i + 3] * inv);
                        const uint32_t bx = pack2<bf16_t>(a[4 * i + 4] * inv, a[4 * i + 5] * inv);
                        const uint32_t by = pack2<bf16_t>(a[4 * i + 6] * inv, a[4 * i + 7] * inv);
                        const auto rx = __builtin_amdgcn_permlane32_swap(ax, bx, false, false);
                        const auto ry = __builtin_amdgcn_permlane32_swap(ay, by, false, false);
                        const int d = DB * 32 + 8 * i + 8 * h32;
                        *reinterpret_cast<i32x4*>(op + d) = i32x4{(int)rx[0], (int)ry[0], (int)rx[1], (int)ry[1]};
                    }
                }
            });
        };
        stamp(17);
        store(std::integral_constant<int, 0>{}, invA);
        stamp(18);
        store(std::integral_constant<int, 1>{}, invB);
        stamp(19);
        if (!has_next) break;
        s0 = (s0 + nt) % NBUF;
        L += (int)gridDim.x;
        block_ptrs(L, b, hq, q0, qp, kp, vp);
        if constexpr (CAUSAL) {
            nt = block_nt(q0);
            tdiag = (q0 + Nk - Nq + 1) / KT;
        }
    }
    // the last DMA (a reload of tile nt-1) lands before the LDS is released
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef PLI_FLASH_STAMPS
    if constexpr (STAMP == 1) {
        stamp(7);
        if (lane == 0) {
#pragma unroll
            for (int i = 0; i < 20; ++i) atomicAdd(&g_v12_stamps[i], st_sum[i]);
            atomicAdd(&g_v12_stamps[22], (unsigned long long)nt * (unsigned long long)nblk);
            atomicAdd(&g_v12_stamps[23], 1ull);
        }
    }
    if constexpr (STAMP == 2) {
        unsigned long long t1, r1;
        asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1), "=s"(r1)::"memory");
        if (lane == 0) {
            atomicAdd(&g_v12_stamps[0], t1 - clk_t0);
            atomicAdd(&g_v12_stamps[1], r1 - clk_r0);
            atomicAdd(&g_v12_stamps[22], (unsigned long long)nt * (unsigned long long)nblk);
            atomicAdd(&g_v12_stamps[23], 1ull);
        }
    }
#endif
}

}  // namespace

bool attn_v12_ok(int D, int is_bf16, int causal, int Nk) {
    return D == 128 && is_bf16 && !causal && Nk >= 64 && Nk % 64 == 0;
}

int launch_attn_v12(const void* q, const void* k, const void* v, void* o, int B, int H, int group, int Nq,
                    int Nk, const V7Strides& st, float scale, hipStream_t stream, bool persistent, float thr,
                    bool causal) {
    PLI_REQUIRE(thr == 0.f || thr == 64.f, "attn_fwd_v12: defer-max threshold %g not built", thr);
    PLI_REQUIRE(!causal || (thr == 64.f && Nq <= Nk), "attn_fwd_v12: causal needs Nq <= Nk (THR 64)");
    const int qblocks = cdiv(Nq, 256);
    const int64_t nb = (int64_t)B * H * qblocks;
    PLI_REQUIRE(nb < (1ll << 31), "pli_flash_attn_fwd: grid too large");
    const float c = scale * 1.4426950408889634f;
    // persistent: one workgroup per CU of the stream's device (the kernel
    // holds 160 KiB of LDS and the whole register file), a multiple of 8 so
    // each walks one XCD; the stream across block seams needs two tiles per
    // block.  Causal: only where causal_block's walk tiles the blocks exactly
    // (else one block per workgroup, heaviest first).
    int grid = (int)nb;
    if (persistent && Nk >= 128) {
        const int g = cu_count(stream) / 8 * 8;
        if (g >= 8 && nb > g) grid = g;
        if (causal && grid < nb) {
            const int64_t bh = nb / qblocks, w = g / 8;
            // every workgroup must walk whole pairs (whole multiples of the QB
            // query heights for the rotation: a walk shorter than QB sees a
            // run of light or heavy blocks, B2 H32 N8192 ran 813 vs 1098 TF/s
            // one block per workgroup)
#if V12_CAUSAL_PAIR
            const int hq = qblocks / 2;
            const bool rot = qblocks % 2 == 0 && w % hq == 0 && bh % 8 == 0 && (bh / 8) % (w / hq) == 0 &&
                             nb % g == 0 && (nb / g) % 2 == 0;
#else
            const bool rot = w % qblocks == 0 && bh % 8 == 0 && (bh / 8) % (w / qblocks) == 0 && nb % g == 0 &&
                             (nb / g) % qblocks == 0;
#endif
            if (!rot) grid = (int)nb;
        }
    }
    const dim3 gr((unsigned)grid), blk(256);
    const auto* qq = (const uint16_t*)q;
    const auto* kk = (const uint16_t*)k;
    const auto* vv = (const uint16_t*)v;
    auto* oo = (uint16_t*)o;
    if (causal)
        hipLaunchKernelGGL((attn_fwd_v12<0, 64, true>), gr, blk, 0, stream, qq, kk, vv, oo, H, group, Nq, Nk, st, c,
                           qblocks, (int)nb);
    else if (thr == 0.f)
        hipLaunchKernelGGL((attn_fwd_v12<0, 0>), gr, blk, 0, stream, qq, kk, vv, oo, H, group, Nq, Nk, st, c,
                           qblocks, (int)nb);
    else
        hipLaunchKernelGGL((attn_fwd_v12<0, 64>), gr, blk, 0, stream, qq, kk, vv, oo, H, group, Nq, Nk, st, c,
                           qblocks, (int)nb);
    return launch_status("attn_fwd_v12");
}

}  // namespace pli

#ifdef PLI_FLASH_STAMPS
// Diagnostic entry (tools/libpli_diag.so only): one stamped launch of
// attn_fwd_v12 on contiguous [B,H,N,128] bf16, the 24 stamp words to `out`
// (segments 0-19: tools/v12_stamps.py SEGS; 22 tiles, 23 waves;
// check, 6 prologue + loop overhead, 7 epilogue; 8 tiles, 9 waves).
extern "C" int pli_diag_v12_stamps(const void* q, const void* k, const void* v, void* o, int B, int H, int N,
                                   unsigned long long* out, int grid, int mode) {
    using namespace pli;
    const int64_t sn = 128, sh = (int64_t)N * 128, sb = (int64_t)H * N * 128;
    const V7Strides st{sb, sh, sn, sb, sh, sn, sb, sh, sn, sb, sh, sn};
    const int qblocks = cdiv(N, 256), nb = B * H * qblocks;
    const float c = (1.f / sqrtf(128.f)) * 1.4426950408889634f;
    unsigned long long zero[24] = {0};
    hipMemcpyToSymbol(HIP_SYMBOL(g_v12_stamps), zero, sizeof(zero));
    const dim3 gr(grid > 0 && grid < nb ? grid : nb);
    // mode 1: per-segment stamps; mode 2: entry / exit clock only (words 0, 1)
    if (mode == 2)
        hipLaunchKernelGGL((attn_fwd_v12<2, 64>), gr, dim3(256), 0, 0, (const uint16_t*)q, (const uint16_t*)k,
                           (const uint16_t*)v, (uint16_t*)o, H, 1, N, N, st, c, qblocks, nb);
    else
        hipLaunchKernelGGL((attn_fwd_v12<1, 64>), gr, dim3(256), 0, 0, (const uint16_t*)q, (const uint16_t*)k,
                           (const uint16_t*)v, (uint16_t*)o, H, 1, N, N, st, c, qblocks, nb);
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    hipMemcpyFromSymbol(out, HIP_SYMBOL(g_v12_stamps), 24 * sizeof(unsigned long long));
    return 0;
}
#endif
