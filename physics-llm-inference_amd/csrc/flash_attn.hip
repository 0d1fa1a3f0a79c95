// Fused attention forward for gfx950 (MI355X).
//
// Replaces the Python tile loop of ch06/flash_attention.py:14-74 (about 12
// torch launches per (q-block, k-block) pair, every intermediate through HBM)
// with ONE launch: Q stays in registers, K/V tiles stream through LDS, the
// online softmax runs in registers with fp32 statistics.
//
// MFMA kernel (bf16 / fp16, head_dim 64 or 128), one wave = 32 query rows:
//   S^T = K Q^T      v_mfma_f32_32x32x16  A = K tile (ds_read_b128, LDS),
//                                         B = Q fragment (registers)
//   -> lane l owns query row l&31; its 64 tile scores sit in 32 registers
//      split over the two half-waves, so the row max / sum are 31 VALU ops
//      plus one cross-half exchange (no LDS, no per-tile cross-lane sum: l is
//      kept per lane and combined once at the end).
//   O^T += V^T P^T   v_mfma_f32_32x32x16  A = V^T (ds_read_b64_tr_b16 from the
//                                         row-major V tile), B = P straight
//                                         from the S^T accumulator registers
//   -> O^T keeps the query row on the lane too, so the online-softmax rescale
//      and the final 1/l are lane-local.
// K and V share one XOR-swizzled LDS image layout that is conflict-free for
// both the row reads (b128) and the transposed reads (tr_b16); tiles are
// register-staged (global loads for tile t+1 issued before tile t's MFMAs,
// written to the other LDS buffer after them), one barrier per tile.
// Blocks are remapped so each XCD works through a contiguous range of heads:
// a head's K/V is then read from HBM once and re-read from that XCD's L2 by
// all of the head's query blocks.
//
// Generic kernel (fp32, or any head_dim <= 128, or unaligned operands):
// LDS-tiled VALU kernel with the same online recurrence, fp32 accumulate.
#include <cmath>
#include <type_traits>

#include "flash_w4.h"
#include "pli_common.h"

namespace pli {
namespace {

struct AttnStrides {
    int64_t qb, qh, qn, kb, kh, kn, vb, vh, vn, ob, oh, on;
};

// 32-bit LDS byte address of a __shared__ pointer (for M0)
__device__ __forceinline__ uint32_t lds_addr(const char* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

constexpr int KT = 64;  // keys per LDS tile
constexpr int QW = 32;  // query rows per wave

// Byte offset of 16-byte chunk `ch` of row `row` in a [KT][D] 16-bit tile.
// D=128 (256-B rows): chunk ^= ((row&3)<<2 | (row>>2)&3);  D=64 (128-B rows,
// two rows per 256-B bank row): chunk ^= g((row>>1)&7) with g(i) =
// ((i&1)<<2)|(i>>1).  Both are conflict-free for a b128 read of 16 distinct
// rows mod 16 and for a tr_b16 read of 4 aligned rows x 4 aligned chunks.
template <int D>
__device__ __forceinline__ int swz_off(int row, int ch) {
    if constexpr (D == 128) {
        const int f = ((row & 3) << 2) | ((row >> 2) & 3);
        return row * 256 + ((ch ^ f) << 4);
    } else {
        static_assert(D == 64, "MFMA attention supports head_dim 64 and 128");
        const int i = (row >> 1) & 7;
        const int g = ((i & 1) << 2) | (i >> 1);
        return row * 128 + ((ch ^ g) << 4);
    }
}

template <typename T, int D, int NW>
__global__ __launch_bounds__(NW * 64, 2) void attn_fwd_mfma(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
    const uint16_t* __restrict__ v, uint16_t* __restrict__ o, int H, int group,
    int Nq, int Nk, AttnStrides st, float c, int causal, int qblocks,
    int nblocks) {
    constexpr int NT = NW * 64;
    constexpr int TILE = KT * D * 2;  // bytes of one K (or V) tile
    constexpr int CPR = D / 8;        // 16-byte chunks per row
    constexpr int CPT = KT * CPR / NT;
    static_assert((KT * CPR) % NT == 0, "tile chunks must split evenly");
    __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h32 = lane >> 5, l32 = lane & 31;

    const int lb = xcd_remap(blockIdx.x, nblocks);
    const int bh = lb / qblocks, qblk = lb % qblocks;
    const int b = bh / H, hq = bh % H, hk = hq / group;
    const int qbase = qblk * (NW * QW);
    const int q0 = qbase + wave * QW;
    const int off_diag = Nk - Nq;  // causal: row i sees keys <= i + off_diag

    const uint16_t* qp = q + b * st.qb + hq * st.qh;
    const uint16_t* kp = k + b * st.kb + hk * st.kh;
    const uint16_t* vp = v + b * st.vb + hk * st.vh;

    // Q^T fragments (B operand): query row q0+l32, d = 16kk + 8h32 .. +7.
    i32x4 qf[D / 16];
    {
        const int qr = q0 + l32;
        const bool ok = qr < Nq;
        const uint16_t* src = qp + (int64_t)(ok ? qr : 0) * st.qn + 8 * h32;
#pragma unroll
        for (int kk = 0; kk < D / 16; ++kk) {
            const i32x4 x = *reinterpret_cast<const i32x4*>(src + 16 * kk);
            qf[kk] = ok ? x : i32x4{0, 0, 0, 0};
        }
    }

    int kv_end = Nk;
    if (causal) kv_end = min(Nk, qbase + NW * QW + off_diag);
    const int ntiles = kv_end > 0 ? cdiv(kv_end, KT) : 0;

    // register staging of one K tile + one V tile
    i32x4 kst[CPT], vst[CPT];
    auto load_tile = [&](int t) {
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
            const int cidx = tid + i * NT;
            const int row = cidx / CPR, ch = cidx % CPR;
            const int key = t * KT + row;
            const int kc = min(key, Nk - 1);  // always issue the load
            const i32x4 kx = *reinterpret_cast<const i32x4*>(kp + (int64_t)kc * st.kn + ch * 8);
            const i32x4 vx = *reinterpret_cast<const i32x4*>(vp + (int64_t)kc * st.vn + ch * 8);
            const bool ok = key < Nk;
            kst[i] = ok ? kx : i32x4{0, 0, 0, 0};
            vst[i] = ok ? vx : i32x4{0, 0, 0, 0};
        }
    };
    auto store_tile = [&](int buf) {
        char* kb = smem + buf * 2 * TILE;
        char* vb = kb + TILE;
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
            const int cidx = tid + i * NT;
            const int off = swz_off<D>(cidx / CPR, cidx % CPR);
            lds_write_b128(kb, off, kst[i]);
            lds_write_b128(vb, off, vst[i]);
        }
    };

    f32x16 oacc[D / 32];
#pragma unroll
    for (int d = 0; d < D / 32; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[d][r] = 0.f;
    float m_run = -1e30f;  // running max, already scaled by c (log2 domain)
    float l_run = 0.f;     // this lane's share of the running denominator

    // tr_b16 addressing: lane 4qq+pp of 16-lane group g reads row qq,
    // columns 4pp..4pp+3 of a 4x16 block.
    const int g = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;

    if (ntiles > 0) {
        load_tile(0);
        store_tile(0);
    }
    __syncthreads();

    for (int t = 0; t < ntiles; ++t) {
        const int buf = t & 1;
        if (t + 1 < ntiles) load_tile(t + 1);
        const char* kb = smem + buf * 2 * TILE;
        const char* vb = kb + TILE;

        // ---- S^T = K Q^T : s[tt][r] = score(key tt*32 + krow(r), query l32)
        f32x16 s[2];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
#pragma unroll
            for (int r = 0; r < 16; ++r) s[tt][r] = 0.f;
#pragma unroll
            for (int kk = 0; kk < D / 16; ++kk) {
                const i32x4 kf = lds_read_b128(kb, swz_off<D>(tt * 32 + l32, 2 * kk + h32));
                s[tt] = mfma32x32x16<T>(kf, qf[kk], s[tt]);
            }
        }

        // ---- masks: ragged last tile, causal diagonal (wave-uniform test)
        const int key0 = t * KT;
        const bool need_mask = (key0 + KT > Nk) || (causal && key0 + KT - 1 > q0 + off_diag);
        if (need_mask) {
            const int lim = causal ? q0 + l32 + off_diag : Nk;
#pragma unroll
            for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int key = key0 + tt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h32;
                    if (key >= Nk || key > lim) s[tt][r] = -INFINITY;
                }
        }

        // ---- online softmax, row = l32
        float mx = s[0][0];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
            for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[tt][r]);
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float m_new = fmaxf(m_run, mx * c);
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        m_run = m_new;
        float rs = 0.f;
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float p = __builtin_amdgcn_exp2f(fmaf(s[tt][r], c, -m_new));
                s[tt][r] = p;
                rs += p;
            }
        l_run = fmaf(l_run, alpha, rs);
#pragma unroll
        for (int d = 0; d < D / 32; ++d)
#pragma unroll
            for (int r = 0; r < 16; ++r) oacc[d][r] *= alpha;

        // P^T fragments: registers 8s2..8s2+7 of s[tt] are k-step s2 (keys
        // 16s2 + 8(j>>2) + 4h32 + (j&3) of the 32-key half tt).
        i32x4 pb[2][2];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const int r0 = 8 * s2;
                pb[tt][s2] = i32x4{(int)pack2<T>(s[tt][r0 + 0], s[tt][r0 + 1]),
                                   (int)pack2<T>(s[tt][r0 + 2], s[tt][r0 + 3]),
                                   (int)pack2<T>(s[tt][r0 + 4], s[tt][r0 + 5]),
                                   (int)pack2<T>(s[tt][r0 + 6], s[tt][r0 + 7])};
            }

        // ---- O^T += V^T P^T ; V^T fragment via two transposed reads
#pragma unroll
        for (int dblk = 0; dblk < D / 32; ++dblk) {
            const int ch = dblk * 4 + 2 * (g & 1) + (pp >> 1);
#pragma unroll
            for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    const int row = tt * 32 + 16 * s2 + 4 * h32 + qq;
                    const i32x2 lo = lds_read_tr16(vb, swz_off<D>(row, ch) + 8 * (pp & 1));
                    const i32x2 hi = lds_read_tr16(vb, swz_off<D>(row + 8, ch) + 8 * (pp & 1));
                    const i32x4 vf = {lo.x, lo.y, hi.x, hi.y};
                    oacc[dblk] = mfma32x32x16<T>(vf, pb[tt][s2], oacc[dblk]);
                }
        }

        if (t + 1 < ntiles) store_tile(buf ^ 1);
        __syncthreads();
    }

    // ---- epilogue: O = O^T / l, query row l32, d = dblk*32 + 8i + 4h32 + 0..3
    const float l = l_run + __shfl_xor(l_run, 32, 64);
    const float inv = l > 0.f ? 1.f / l : 0.f;
    const int qr = q0 + l32;
    if (qr < Nq) {
        uint16_t* op = o + b * st.ob + hq * st.oh + (int64_t)qr * st.on;
#pragma unroll
        for (int dblk = 0; dblk < D / 32; ++dblk)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int d = dblk * 32 + 8 * i + 4 * h32;
                const i32x2 w = {(int)pack2<T>(oacc[dblk][4 * i] * inv, oacc[dblk][4 * i + 1] * inv),
                                 (int)pack2<T>(oacc[dblk][4 * i + 2] * inv, oacc[dblk][4 * i + 3] * inv)};
                *reinterpret_cast<i32x2*>(op + d) = w;
            }
    }
}

// --------------------------------------------------------------------------
// attn_fwd_v2: attn_fwd_mfma's fragment mapping and register staging, with
// the per-tile overheads removed:
//  * padded LDS rows instead of an XOR swizzle -- K rows 2D+16 B, V rows
//    2D+64 B.  K's b128 reads of 16 consecutive rows land on 16 distinct
//    16-byte slots (stride = 17 slots mod 16); V's tr_b16 reads of 4 rows x
//    64 B land on 4 disjoint 16-bank quarters (stride = 80 dwords = 16 mod 64).
//    Every fragment address is then one per-lane base register + an
//    immediate offset: no per-read address arithmetic in the loop.
//  * global staging addresses are one per-lane base + scalar tile offset;
//    the clamp for rows past Nk only runs on a ragged last tile.
//  * the O rescale is skipped (exactly) when no row's max moved this tile.
// (A software-pipelined variant that issued QK^T(t+1) beside softmax(t) with
// LDS-DMA staging spilled at D=128 and ran 1.5-2.5x slower: every spill
// reload's vmcnt(0) also drained the in-flight DMA.  See DESIGN.md.)
template <int D, int KTL = KT> struct PadLayout {
    static constexpr int KS = 2 * D + 16;  // K row stride (bytes)
    static constexpr int VS = 2 * D + 64;  // V row stride (bytes)
    static constexpr int KSZ = KTL * KS, VSZ = KTL * VS, BUF = KSZ + VSZ;
};

// OPT bits (A/B levers on the v2 body, variants 16-20):
//  1: the xor-32 row-max exchange as v_permlane32_swap instead of ds_bpermute
//  2: static s_setprio 1 for the younger half of the workgroup (waves NW/2..)
//  4: defer-max: keep the running max unless a tile raises it by > 8 (log2
//     units), so P <= 2^8 and the O rescale almost never runs after tile 0
//  8: row sum over the bf16/f16-ROUNDED P (v_dot2c with {1,1}), so l
//     normalises exactly the weights P.V used.  Needed with 4: a dominant
//     weight is no longer exactly 1 and its rounding would otherwise go
//     uncorrected (measured 1.05e-2 on the spike test without it).
// 16: epilogue: pair the two half-waves' 8-byte pieces of a row with
//     v_permlane32_swap so each lane stores 16 B (8 dwordx4 instead of 16 dwordx2)
// 32 / 64: __builtin_amdgcn_iglp_opt(0) / (1) in the tile loop (the compiler's
//     MFMA + DS interleave strategies)
// 128: batched fragment reads (all K fragments of the tile, V^T one block
//     ahead) so LDS latency overlaps the MFMAs instead of pairing each read
//     with the MFMA that consumes it
constexpr int kOptPermlane = 1, kOptPrio = 2, kOptDefer = 4, kOptRoundedSum = 8, kOptWideStore = 16,
              kOptIglp0 = 32, kOptIglp1 = 64, kOptBatchReads = 128;
constexpr float kDeferThr = 8.f;

__device__ __forceinline__ float xor32_max(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xor32_sum(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

template <typename T, int D, int NW, bool LAZY, int OPT = 0, int KTL = KT>
__global__ __launch_bounds__(NW * 64, 2) void attn_fwd_v2(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
    const uint16_t* __restrict__ v, uint16_t* __restrict__ o, int H, int group,
    int Nq, int Nk, AttnStrides st, float c, int causal, int qblocks,
    int nblocks) {
    using L = PadLayout<D, KTL>;
    constexpr int NS = KTL / 32;        // 32-key sub-tiles per tile
    constexpr int NT = NW * 64;
    constexpr int CPR = D / 8;          // 16-byte chunks per row
    constexpr int RPI = NT / CPR;       // rows covered by one staging step
    constexpr int CPT = KTL / RPI;      // staging steps per tile
    static_assert(NT % CPR == 0 && KTL % RPI == 0, "staging must tile evenly");
    __shared__ __attribute__((aligned(16))) char smem[2 * L::BUF];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h32 = lane >> 5, l32 = lane & 31;
    const int lb = xcd_remap(blockIdx.x, nblocks);
    const int bh = lb / qblocks;
    // causal: a query block's work grows with its index; start each head's
    // heaviest blocks first so the grid drains on light ones
    const int qblk = causal ? qblocks - 1 - lb % qblocks : lb % qblocks;
    const int b = bh / H, hq = bh % H, hk = hq / group;
    const int qbase = qblk * (NW * QW);
    const int q0 = qbase + wave * QW;
    const int off_diag = Nk - Nq;

    const uint16_t* qp = q + b * st.qb + hq * st.qh;
    const uint16_t* kp = k + b * st.kb + hk * st.kh;
    const uint16_t* vp = v + b * st.vb + hk * st.vh;

    i32x4 qf[D / 16];
    {
        const int qr = q0 + l32;
        const bool ok = qr < Nq;
        const uint16_t* src = qp + (int64_t)(ok ? qr : 0) * st.qn + 8 * h32;
#pragma unroll
        for (int kk = 0; kk < D / 16; ++kk) {
            const i32x4 x = *reinterpret_cast<const i32x4*>(src + 16 * kk);
            qf[kk] = ok ? x : i32x4{0, 0, 0, 0};
        }
    }

    int kv_end = Nk;
    if (causal) kv_end = min(Nk, qbase + NW * QW + off_diag);
    const int nt = kv_end > 0 ? cdiv(kv_end, KTL) : 0;
    const int t_full = Nk / KTL;  // tiles [0, t_full) need no row clamp
    int t_mask = t_full;         // first tile this wave must mask
    if (causal) t_mask = min(t_mask, max(0, (q0 + off_diag + 1) / KTL));

    // staging: thread owns chunk `sch` of rows srow + i*RPI
    const int srow = tid / CPR, sch = tid % CPR;
    const uint16_t* kg = kp + (int64_t)srow * st.kn + sch * 8;
    const uint16_t* vg = vp + (int64_t)srow * st.vn + sch * 8;
    const int kw = srow * L::KS + sch * 16, vw = L::KSZ + srow * L::VS + sch * 16;
    i32x4 kst[CPT], vst[CPT];
    auto load_tile = [&](int t) {
        if (t < t_full) {
#pragma unroll
            for (int i = 0; i < CPT; ++i) {
                const int64_t r = (int64_t)t * KTL + i * RPI;
                kst[i] = *reinterpret_cast<const i32x4*>(kg + r * st.kn);
                vst[i] = *reinterpret_cast<const i32x4*>(vg + r * st.vn);
            }
        } else {
#pragma unroll
            for (int i = 0; i < CPT; ++i) {
                const int key = t * KTL + i * RPI + srow;
                const int64_t r = min(key, Nk - 1) - srow;
                const i32x4 kx = *reinterpret_cast<const i32x4*>(kg + r * st.kn);
                const i32x4 vx = *reinterpret_cast<const i32x4*>(vg + r * st.vn);
                kst[i] = key < Nk ? kx : i32x4{0, 0, 0, 0};
                vst[i] = key < Nk ? vx : i32x4{0, 0, 0, 0};
            }
        }
    };
    auto store_tile = [&](int buf) {
        char* base = smem + buf * L::BUF;
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
            lds_write_b128(base, kw + i * RPI * L::KS, kst[i]);
            lds_write_b128(base, vw + i * RPI * L::VS, vst[i]);
        }
    };

    // per-lane fragment bases (byte offsets inside one buffer)
    const int g = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;
    const int kr = l32 * L::KS + h32 * 16;
    const int vr = L::KSZ + (4 * h32 + qq) * L::VS + (2 * (g & 1) + (pp >> 1)) * 16 + 8 * (pp & 1);

    f32x16 oacc[D / 32];
#pragma unroll
    for (int d = 0; d < D / 32; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[d][r] = 0.f;
    float m_run = -1e30f, l_run = 0.f;

    if (nt > 0) {
        load_tile(0);
        store_tile(0);
    }
    __syncthreads();
    if constexpr ((OPT & kOptPrio) != 0) {
        if (wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
    }

    for (int t = 0; t < nt; ++t) {
        if constexpr ((OPT & kOptIglp0) != 0) __builtin_amdgcn_iglp_opt(0);
        if constexpr ((OPT & kOptIglp1) != 0) __builtin_amdgcn_iglp_opt(1);
        if (t + 1 < nt) load_tile(t + 1);
        const char* kb = smem + (t & 1) * L::BUF + kr;
        const char* vb = smem + (t & 1) * L::BUF + vr;

        f32x16 s[NS];
        if constexpr ((OPT & kOptBatchReads) != 0) {
            // every K fragment of the tile in flight before the first MFMA
            i32x4 kfr[NS][D / 16];
#pragma unroll
            for (int tt = 0; tt < NS; ++tt)
#pragma unroll
                for (int kk = 0; kk < D / 16; ++kk) kfr[tt][kk] = lds_read_b128(kb, tt * 32 * L::KS + kk * 32);
            __builtin_amdgcn_sched_barrier(0);  // keep the batch ahead of the MFMAs
#pragma unroll
            for (int tt = 0; tt < NS; ++tt) {
#pragma unroll
                for (int r = 0; r < 16; ++r) s[tt][r] = 0.f;
#pragma unroll
                for (int kk = 0; kk < D / 16; ++kk) s[tt] = mfma32x32x16<T>(kfr[tt][kk], qf[kk], s[tt]);
            }
        } else {
#pragma unroll
        for (int tt = 0; tt < NS; ++tt) {
#pragma unroll
            for (int r = 0; r < 16; ++r) s[tt][r] = 0.f;
#pragma unroll
            for (int kk = 0; kk < D / 16; ++kk) {
                const i32x4 kf = lds_read_b128(kb, tt * 32 * L::KS + kk * 32);
                s[tt] = mfma32x32x16<T>(kf, qf[kk], s[tt]);
            }
        }
        }

        if (t >= t_mask) {
            const int lim = causal ? q0 + l32 + off_diag : Nk;
#pragma unroll
            for (int tt = 0; tt < NS; ++tt)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int key = t * KTL + tt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h32;
                    if (key >= Nk || key > lim) s[tt][r] = -INFINITY;
                }
        }

        float mx, my;
        if constexpr (NS == 2) {
            mx = max3(s[0][0], s[1][0], s[0][1]);
            my = max3(s[1][1], s[0][2], s[1][2]);
#pragma unroll
            for (int r = 3; r < 15; r += 2) {
                mx = max3(mx, s[0][r], s[1][r]);
                my = max3(my, s[0][r + 1], s[1][r + 1]);
            }
            mx = max3(mx, my, max3(s[0][15], s[1][15], mx));
        } else {
            mx = max3(s[0][0], s[0][1], s[0][2]);
            my = max3(s[0][3], s[0][4], s[0][5]);
#pragma unroll
            for (int i = 6; i + 3 < NS * 16; i += 4) {
                mx = max3(mx, s[i / 16][i % 16], s[(i + 1) / 16][(i + 1) % 16]);
                my = max3(my, s[(i + 2) / 16][(i + 2) % 16], s[(i + 3) / 16][(i + 3) % 16]);
            }
            mx = max3(mx, my, max3(s[NS - 1][14], s[NS - 1][15], mx));
        }
        if constexpr ((OPT & kOptPermlane) != 0) mx = xor32_max(mx);
        else mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        float m_new = fmaxf(m_run, mx * c);
        if constexpr ((OPT & kOptDefer) != 0) m_new = mx * c > m_run + kDeferThr ? m_new : m_run;
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        m_run = m_new;
        float rs = 0.f;
#pragma unroll
        for (int tt = 0; tt < NS; ++tt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float p = __builtin_amdgcn_exp2f(fmaf(s[tt][r], c, -m_new));
                s[tt][r] = p;
                if constexpr ((OPT & kOptRoundedSum) == 0) rs += p;
            }
        if constexpr ((OPT & kOptRoundedSum) == 0) l_run = fmaf(l_run, alpha, rs);
        if (!LAZY || __ballot(alpha != 1.f)) {
#pragma unroll
            for (int d = 0; d < D / 32; ++d)
#pragma unroll
                for (int r = 0; r < 16; ++r) oacc[d][r] *= alpha;
        }

        i32x4 pb[NS][2];
#pragma unroll
        for (int tt = 0; tt < NS; ++tt)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const int r0 = 8 * s2;
                pb[tt][s2] = i32x4{(int)pack2<T>(s[tt][r0 + 0], s[tt][r0 + 1]),
                                   (int)pack2<T>(s[tt][r0 + 2], s[tt][r0 + 3]),
                                   (int)pack2<T>(s[tt][r0 + 4], s[tt][r0 + 5]),
                                   (int)pack2<T>(s[tt][r0 + 6], s[tt][r0 + 7])};
            }
        if constexpr ((OPT & kOptRoundedSum) != 0) {
            float r0 = 0.f, r1 = 0.f;
#pragma unroll
            for (int tt = 0; tt < NS; ++tt)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    r0 = add_pair<T>((uint32_t)pb[tt][s2][0], r0);
                    r1 = add_pair<T>((uint32_t)pb[tt][s2][1], r1);
                    r0 = add_pair<T>((uint32_t)pb[tt][s2][2], r0);
                    r1 = add_pair<T>((uint32_t)pb[tt][s2][3], r1);
                }
            l_run = fmaf(l_run, alpha, r0 + r1);
        }
        if constexpr ((OPT & kOptBatchReads) != 0) {
            // V^T fragments of one 32-column block read as a batch, the next
            // block's batch issued before this block's MFMAs
            i32x4 vf[2][NS][2];
            auto read_v = [&](int dblk, i32x4 (&dst)[NS][2]) {
#pragma unroll
                for (int tt = 0; tt < NS; ++tt)
#pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2) {
                        const int ro = (tt * 32 + 16 * s2) * L::VS + dblk * 64;
                        const i32x2 lo = lds_read_tr16(vb, ro);
                        const i32x2 hi = lds_read_tr16(vb, ro + 8 * L::VS);
                        dst[tt][s2] = i32x4{lo.x, lo.y, hi.x, hi.y};
                    }
            };
            read_v(0, vf[0]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int dblk = 0; dblk < D / 32; ++dblk) {
                if (dblk + 1 < D / 32) read_v(dblk + 1, vf[(dblk + 1) & 1]);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int tt = 0; tt < NS; ++tt)
#pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2)
                        oacc[dblk] = mfma32x32x16<T>(vf[dblk & 1][tt][s2], pb[tt][s2], oacc[dblk]);
            }
        } else {
#pragma unroll
        for (int dblk = 0; dblk < D / 32; ++dblk)
#pragma unroll
            for (int tt = 0; tt < NS; ++tt)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    const int ro = (tt * 32 + 16 * s2) * L::VS + dblk * 64;
                    const i32x2 lo = lds_read_tr16(vb, ro);
                    const i32x2 hi = lds_read_tr16(vb, ro + 8 * L::VS);
                    oacc[dblk] = mfma32x32x16<T>(i32x4{lo.x, lo.y, hi.x, hi.y}, pb[tt][s2], oacc[dblk]);
                }
        }

        if (t + 1 < nt) store_tile((t + 1) & 1);
        __syncthreads();
    }

    if constexpr ((OPT & kOptPrio) != 0) __builtin_amdgcn_s_setprio(0);
    float l;
    if constexpr ((OPT & kOptPermlane) != 0) l = xor32_sum(l_run);
    else l = l_run + __shfl_xor(l_run, 32, 64);
    const float inv = l > 0.f ? 1.f / l : 0.f;
    const int qr = q0 + l32;
    if (qr < Nq) {
        uint16_t* op = o + b * st.ob + hq * st.oh + (int64_t)qr * st.on;
        if constexpr ((OPT & kOptWideStore) != 0) {
            // group k = 4*dblk + i holds columns 8k+4*h32 .. +3 of row qr; after
            // swapping (k, k+1): lower lanes hold cols 8k..8k+7, upper 8k+8..8k+15
#pragma unroll
            for (int dblk = 0; dblk < D / 32; ++dblk)
#pragma unroll
                for (int i = 0; i < 4; i += 2) {
                    const f32x16& a = oacc[dblk];
                    uint32_t ax = pack2<T>(a[4 * i] * inv, a[4 * i + 1] * inv);
                    uint32_t ay = pack2<T>(a[4 * i + 2] * inv, a[4 * i + 3] * inv);
                    uint32_t bx = pack2<T>(a[4 * i + 4] * inv, a[4 * i + 5] * inv);
                    uint32_t by = pack2<T>(a[4 * i + 6] * inv, a[4 * i + 7] * inv);
                    const auto rx = __builtin_amdgcn_permlane32_swap(ax, bx, false, false);
                    const auto ry = __builtin_amdgcn_permlane32_swap(ay, by, false, false);
                    const int d = dblk * 32 + 8 * i + 8 * h32;
                    *reinterpret_cast<i32x4*>(op + d) =
                        i32x4{(int)rx[0], (int)ry[0], (int)rx[1], (int)ry[1]};
                }
        } else {
#pragma unroll
            for (int dblk = 0; dblk < D / 32; ++dblk)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int d = dblk * 32 + 8 * i + 4 * h32;
                    const i32x2 w = {(int)pack2<T>(oacc[dblk][4 * i] * inv, oacc[dblk][4 * i + 1] * inv),
                                     (int)pack2<T>(oacc[dblk][4 * i + 2] * inv, oacc[dblk][4 * i + 3] * inv)};
                    *reinterpret_cast<i32x2*>(op + d) = w;
                }
        }
    }
}

// --------------------------------------------------------------------------
// attn_fwd_pp: variant 21's body split into two barrier phases per tile,
//   X(t) = S = K.Q^T, mask, softmax -> P(t)      Y(t) = O rescale + P(t).V(t)
// with waves 4..7 one barrier behind waves 0..3 (one extra s_barrier at the
// start).  The two waves a SIMD holds (one from each half) then ping-pong:
// while one runs X (MFMA + the whole VALU softmax) the other runs Y (MFMA),
// instead of both entering QK^T, softmax and PV together after every
// barrier (in lockstep the softmax VALU of both waves serialises between
// the MFMA blocks).  Staging of tile t+1: the leading half stores its rows
// at the end of Y(t), the lagging half at the end of X(t) -- both after
// every read of tile t-1 and before the first read of t+1 (X(t+1) of the
// leading half); each thread then issues its loads for t+2.  The leading
// half ends with one extra barrier so both halves execute the same count.
template <typename T, int D>
__global__ __launch_bounds__(512, 2) void attn_fwd_pp(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
    const uint16_t* __restrict__ v, uint16_t* __restrict__ o, int H, int group,
    int Nq, int Nk, AttnStrides st, float c, int causal, int qblocks,
    int nblocks) {
    using L = PadLayout<D>;
    constexpr int NW = 8, NT = 512;
    constexpr int CPR = D / 8;
    constexpr int RPI = NT / CPR;
    constexpr int CPT = KT / RPI;
    static_assert(NT % CPR == 0 && KT % RPI == 0, "staging must tile evenly");
    __shared__ __attribute__((aligned(16))) char smem[2 * L::BUF];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const bool lag = wave >= NW / 2;
    const int h32 = lane >> 5, l32 = lane & 31;
    const int lb = xcd_remap(blockIdx.x, nblocks);
    const int bh = lb / qblocks;
    const int qblk = causal ? qblocks - 1 - lb % qblocks : lb % qblocks;
    const int b = bh / H, hq = bh % H, hk = hq / group;
    const int qbase = qblk * (NW * QW);
    const int q0 = qbase + wave * QW;
    const int off_diag = Nk - Nq;

    const uint16_t* qp = q + b * st.qb + hq * st.qh;
    const uint16_t* kp = k + b * st.kb + hk * st.kh;
    const uint16_t* vp = v + b * st.vb + hk * st.vh;

    i32x4 qf[D / 16];
    {
        const int qr = q0 + l32;
        const bool ok = qr < Nq;
        const uint16_t* src = qp + (int64_t)(ok ? qr : 0) * st.qn + 8 * h32;
#pragma unroll
        for (int kk = 0; kk < D / 16; ++kk) {
            const i32x4 x = *reinterpret_cast<const i32x4*>(src + 16 * kk);
            qf[kk] = ok ? x : i32x4{0, 0, 0, 0};
        }
    }

    int kv_end = Nk;
    if (causal) kv_end = min(Nk, qbase + NW * QW + off_diag);
    const int nt = kv_end > 0 ? cdiv(kv_end, KT) : 0;
    const int t_full = Nk / KT;
    int t_mask = t_full;
    if (causal) t_mask = min(t_mask, max(0, (q0 + off_diag + 1) / KT));

    const int srow = tid / CPR, sch = tid % CPR;
    const uint16_t* kg = kp + (int64_t)srow * st.kn + sch * 8;
    const uint16_t* vg = vp + (int64_t)srow * st.vn + sch * 8;
    const int kw = srow * L::KS + sch * 16, vw = L::KSZ + srow * L::VS + sch * 16;
    i32x4 kst[CPT], vst[CPT];
    auto load_tile = [&](int t) {
        if (t < t_full) {
#pragma unroll
            for (int i = 0; i < CPT; ++i) {
                const int64_t r = (int64_t)t * KT + i * RPI;
                kst[i] = *reinterpret_cast<const i32x4*>(kg + r * st.kn);
                vst[i] = *reinterpret_cast<const i32x4*>(vg + r * st.vn);
            }
        } else {
#pragma unroll
            for (int i = 0; i < CPT; ++i) {
                const int key = t * KT + i * RPI + srow;
                const int64_t r = min(key, Nk - 1) - srow;
                const i32x4 kx = *reinterpret_cast<const i32x4*>(kg + r * st.kn);
                const i32x4 vx = *reinterpret_cast<const i32x4*>(vg + r * st.vn);
                kst[i] = key < Nk ? kx : i32x4{0, 0, 0, 0};
                vst[i] = key < Nk ? vx : i32x4{0, 0, 0, 0};
            }
        }
    };
    auto store_tile = [&](int buf) {
        char* base = smem + buf * L::BUF;
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
            lds_write_b128(base, kw + i * RPI * L::KS, kst[i]);
            lds_write_b128(base, vw + i * RPI * L::VS, vst[i]);
        }
    };

    const int g = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;
    const int kr = l32 * L::KS + h32 * 16;
    const int vr = L::KSZ + (4 * h32 + qq) * L::VS + (2 * (g & 1) + (pp >> 1)) * 16 + 8 * (pp & 1);

    f32x16 oacc[D / 32];
#pragma unroll
    for (int d = 0; d < D / 32; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[d][r] = 0.f;
    float m_run = -1e30f, l_run = 0.f;

    if (nt > 0) {
        load_tile(0);
        store_tile(0);
    }
    __syncthreads();
    if (nt > 1) load_tile(1);
    if (lag) __builtin_amdgcn_s_barrier();  // the lagging half runs one phase behind

    for (int t = 0; t < nt; ++t) {
        const char* kb = smem + (t & 1) * L::BUF + kr;
        const char* vb = smem + (t & 1) * L::BUF + vr;
        // ------------------------------------------------------------ X(t)
        f32x16 s[2];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
#pragma unroll
            for (int r = 0; r < 16; ++r) s[tt][r] = 0.f;
#pragma unroll
            for (int kk = 0; kk < D / 16; ++kk) {
                const i32x4 kf = lds_read_b128(kb, tt * 32 * L::KS + kk * 32);
                s[tt] = mfma32x32x16<T>(kf, qf[kk], s[tt]);
            }
        }
        if (t >= t_mask) {
            const int lim = causal ? q0 + l32 + off_diag : Nk;
#pragma unroll
            for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int key = t * KT + tt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h32;
                    if (key >= Nk || key > lim) s[tt][r] = -INFINITY;
                }
        }
        float mx = max3(s[0][0], s[1][0], s[0][1]);
        float my = max3(s[1][1], s[0][2], s[1][2]);
#pragma unroll
        for (int r = 3; r < 15; r += 2) {
            mx = max3(mx, s[0][r], s[1][r]);
            my = max3(my, s[0][r + 1], s[1][r + 1]);
        }
        mx = xor32_max(max3(mx, my, max3(s[0][15], s[1][15], mx)));
        float m_new = fmaxf(m_run, mx * c);
        m_new = mx * c > m_run + kDeferThr ? m_new : m_run;
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        m_run = m_new;
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
            for (int r = 0; r < 16; ++r) s[tt][r] = __builtin_amdgcn_exp2f(fmaf(s[tt][r], c, -m_new));
        i32x4 pb[2][2];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const int r0 = 8 * s2;
                pb[tt][s2] = i32x4{(int)pack2<T>(s[tt][r0 + 0], s[tt][r0 + 1]),
                                   (int)pack2<T>(s[tt][r0 + 2], s[tt][r0 + 3]),
                                   (int)pack2<T>(s[tt][r0 + 4], s[tt][r0 + 5]),
                                   (int)pack2<T>(s[tt][r0 + 6], s[tt][r0 + 7])};
            }
        {
            float r0 = 0.f, r1 = 0.f;
#pragma unroll
            for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    r0 = add_pair<T>((uint32_t)pb[tt][s2][0], r0);
                    r1 = add_pair<T>((uint32_t)pb[tt][s2][1], r1);
                    r0 = add_pair<T>((uint32_t)pb[tt][s2][2], r0);
                    r1 = add_pair<T>((uint32_t)pb[tt][s2][3], r1);
                }
            l_run = fmaf(l_run, alpha, r0 + r1);
        }
        if (lag && t + 1 < nt) {
            store_tile((t + 1) & 1);
            if (t + 2 < nt) load_tile(t + 2);
        }
        __syncthreads();
        // ------------------------------------------------------------ Y(t)
        if (__ballot(alpha != 1.f)) {
#pragma unroll
            for (int d = 0; d < D / 32; ++d)
#pragma unroll
                for (int r = 0; r < 16; ++r) oacc[d][r] *= alpha;
        }
#pragma unroll
        for (int dblk = 0; dblk < D / 32; ++dblk)
#pragma unroll
            for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    const int ro = (tt * 32 + 16 * s2) * L::VS + dblk * 64;
                    const i32x2 lo = lds_read_tr16(vb, ro);
                    const i32x2 hi = lds_read_tr16(vb, ro + 8 * L::VS);
                    oacc[dblk] = mfma32x32x16<T>(i32x4{lo.x, lo.y, hi.x, hi.y}, pb[tt][s2], oacc[dblk]);
                }
        if (!lag && t + 1 < nt) {
            store_tile((t + 1) & 1);
            if (t + 2 < nt) load_tile(t + 2);
        }
        __syncthreads();
    }
    if (!lag) __builtin_amdgcn_s_barrier();  // match the lagging half's extra barrier

    const float l = xor32_sum(l_run);
    const float inv = l > 0.f ? 1.f / l : 0.f;
    const int qr = q0 + l32;
    if (qr < Nq) {
        uint16_t* op = o + b * st.ob + hq * st.oh + (int64_t)qr * st.on;
#pragma unroll
        for (int dblk = 0; dblk < D / 32; ++dblk)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int d = dblk * 32 + 8 * i + 4 * h32;
                const i32x2 w = {(int)pack2<T>(oacc[dblk][4 * i] * inv, oacc[dblk][4 * i + 1] * inv),
                                 (int)pack2<T>(oacc[dblk][4 * i + 2] * inv, oacc[dblk][4 * i + 3] * inv)};
                *reinterpret_cast<i32x2*>(op + d) = w;
            }
    }
}

// --------------------------------------------------------------------------
// attn_fwd_v2b: v2 with the softmax restructured for the scheduler.
//  * one instance of the tile body per mask mode (template), so an unmasked
//    tile is a single scheduling region (QK^T MFMAs .. PV MFMAs);
//  * the 32 scores are exponentiated, packed and fed to PV 8 at a time
//    (keys of one P fragment), so the exps of block i+1 issue in the gaps of
//    block i's 4 PV MFMAs instead of all 32 exps preceding all 16 MFMAs;
//  * the row max and row sum run as 4 independent chains (the serial
//    32-long v_add chain exposed ~8 cycles of latency per add);
//  * eager rescale (no branch inside the region); optional s_setprio(1)
//    around the MFMA clusters (PRIO).
template <typename T, int D, bool PRIO>
__global__ __launch_bounds__(512, 2) void attn_fwd_v2b(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
    const uint16_t* __restrict__ v, uint16_t* __restrict__ o, int H, int group,
    int Nq, int Nk, AttnStrides st, float c, int causal, int qblocks,
    int nblocks) {
    using L = PadLayout<D>;
    constexpr int NW = 8, NT = 512;
    constexpr int CPR = D / 8;
    constexpr int RPI = NT / CPR;
    constexpr int CPT = KT / RPI;
    static_assert(NT % CPR == 0 && KT % RPI == 0, "staging must tile evenly");
    __shared__ __attribute__((aligned(16))) char smem[2 * L::BUF];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h32 = lane >> 5, l32 = lane & 31;
    const int lb = xcd_remap(blockIdx.x, nblocks);
    const int bh = lb / qblocks, qblk = lb % qblocks;
    const int b = bh / H, hq = bh % H, hk = hq / group;
    const int qbase = qblk * (NW * QW);
    const int q0 = qbase + wave * QW;
    const int off_diag = Nk - Nq;

    const uint16_t* qp = q + b * st.qb + hq * st.qh;
    const uint16_t* kp = k + b * st.kb + hk * st.kh;
    const uint16_t* vp = v + b * st.vb + hk * st.vh;

    i32x4 qf[D / 16];
    {
        const int qr = q0 + l32;
        const bool ok = qr < Nq;
        const uint16_t* src = qp + (int64_t)(ok ? qr : 0) * st.qn + 8 * h32;
#pragma unroll
        for (int kk = 0; kk < D / 16; ++kk) {
            const i32x4 x = *reinterpret_cast<const i32x4*>(src + 16 * kk);
            qf[kk] = ok ? x : i32x4{0, 0, 0, 0};
        }
    }

    int kv_end = Nk;
    if (causal) kv_end = min(Nk, qbase + NW * QW + off_diag);
    const int nt = kv_end > 0 ? cdiv(kv_end, KT) : 0;
    const int t_full = Nk / KT;
    int t_mask = t_full;
    if (causal) t_mask = min(t_mask, max(0, (q0 + off_diag + 1) / KT));

    const int srow = tid / CPR, sch = tid % CPR;
    const uint16_t* kg = kp + (int64_t)srow * st.kn + sch * 8;
    const uint16_t* vg = vp + (int64_t)srow * st.vn + sch * 8;
    const int kw = srow * L::KS + sch * 16, vw = L::KSZ + srow * L::VS + sch * 16;
    i32x4 kst[CPT], vst[CPT];
    auto load_tile = [&](int t) {
        if (t < t_full) {
#pragma unroll
            for (int i = 0; i < CPT; ++i) {
                const int64_t r = (int64_t)t * KT + i * RPI;
                kst[i] = *reinterpret_cast<const i32x4*>(kg + r * st.kn);
                vst[i] = *reinterpret_cast<const i32x4*>(vg + r * st.vn);
            }
        } else {
#pragma unroll
            for (int i = 0; i < CPT; ++i) {
                const int key = t * KT + i * RPI + srow;
                const int64_t r = min(key, Nk - 1) - srow;
                const i32x4 kx = *reinterpret_cast<const i32x4*>(kg + r * st.kn);
                const i32x4 vx = *reinterpret_cast<const i32x4*>(vg + r * st.vn);
                kst[i] = key < Nk ? kx : i32x4{0, 0, 0, 0};
                vst[i] = key < Nk ? vx : i32x4{0, 0, 0, 0};
            }
        }
    };
    auto store_tile = [&](int buf) {
        char* base = smem + buf * L::BUF;
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
            lds_write_b128(base, kw + i * RPI * L::KS, kst[i]);
            lds_write_b128(base, vw + i * RPI * L::VS, vst[i]);
        }
    };

    const int g = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;
    const int kr = l32 * L::KS + h32 * 16;
    const int vr = L::KSZ + (4 * h32 + qq) * L::VS + (2 * (g & 1) + (pp >> 1)) * 16 + 8 * (pp & 1);

    f32x16 oacc[D / 32];
#pragma unroll
    for (int d = 0; d < D / 32; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[d][r] = 0.f;
    float m_run = -1e30f, l_run = 0.f;

    auto body = [&](auto mask_tag, int t) {
        constexpr bool MASK = decltype(mask_tag)::value;
        if (t + 1 < nt) load_tile(t + 1);
        const char* kb = smem + (t & 1) * L::BUF + kr;
        const char* vb = smem + (t & 1) * L::BUF + vr;

        f32x16 s[2];
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
#pragma unroll
            for (int r = 0; r < 16; ++r) s[tt][r] = 0.f;
#pragma unroll
            for (int kk = 0; kk < D / 16; ++kk)
                s[tt] = mfma32x32x16<T>(lds_read_b128(kb, tt * 32 * L::KS + kk * 32), qf[kk], s[tt]);
        }
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
        if constexpr (MASK) {
            const int lim = causal ? q0 + l32 + off_diag : Nk;
#pragma unroll
            for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int key = t * KT + tt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h32;
                    if (key >= Nk || key > lim) s[tt][r] = -INFINITY;
                }
        }
        float m4[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) m4[j] = max3(s[0][4 * j], s[1][4 * j], s[0][4 * j + 1]);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            m4[j] = max3(m4[j], s[1][4 * j + 1], s[0][4 * j + 2]);
            m4[j] = max3(m4[j], s[1][4 * j + 2], s[0][4 * j + 3]);
            m4[j] = fmaxf(m4[j], s[1][4 * j + 3]);
        }
        float mx = max3(m4[0], m4[1], max3(m4[2], m4[3], m4[0]));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float m_new = fmaxf(m_run, mx * c);
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        m_run = m_new;
#pragma unroll
        for (int d = 0; d < D / 32; ++d)
#pragma unroll
            for (int r = 0; r < 16; ++r) oacc[d][r] *= alpha;
        float rs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                float p[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    p[j] = __builtin_amdgcn_exp2f(fmaf(s[tt][8 * s2 + j], c, -m_new));
                    rs[j & 3] += p[j];
                }
                const i32x4 pb = {(int)pack2<T>(p[0], p[1]), (int)pack2<T>(p[2], p[3]),
                                  (int)pack2<T>(p[4], p[5]), (int)pack2<T>(p[6], p[7])};
                if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
                for (int dblk = 0; dblk < D / 32; ++dblk) {
                    const int ro = (tt * 32 + 16 * s2) * L::VS + dblk * 64;
                    const i32x2 lo = lds_read_tr16(vb, ro);
                    const i32x2 hi = lds_read_tr16(vb, ro + 8 * L::VS);
                    oacc[dblk] = mfma32x32x16<T>(i32x4{lo.x, lo.y, hi.x, hi.y}, pb, oacc[dblk]);
                }
                if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
            }
        l_run = fmaf(l_run, alpha, (rs[0] + rs[1]) + (rs[2] + rs[3]));
        if (t + 1 < nt) store_tile((t + 1) & 1);
        __syncthreads();
    };

    if (nt > 0) {
        load_tile(0);
        store_tile(0);
    }
    __syncthreads();
    for (int t = 0; t < nt; ++t) {
        if (t < t_mask)
            body(std::false_type{}, t);
        else
            body(std::true_type{}, t);
    }

    const float l = l_run + __shfl_xor(l_run, 32, 64);
    const float inv = l > 0.f ? 1.f / l : 0.f;
    const int qr = q0 + l32;
    if (qr < Nq) {
        uint16_t* op = o + b * st.ob + hq * st.oh + (int64_t)qr * st.on;
#pragma unroll
        for (int dblk = 0; dblk < D / 32; ++dblk)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int d = dblk * 32 + 8 * i + 4 * h32;
                const i32x2 w = {(int)pack2<T>(oacc[dblk][4 * i] * inv, oacc[dblk][4 * i + 1] * inv),
                                 (int)pack2<T>(oacc[dblk][4 * i + 2] * inv, oacc[dblk][4 * i + 3] * inv)};
                *reinterpret_cast<i32x2*>(op + d) = w;
            }
    }
}

// --------------------------------------------------------------------------
// attn_fwd_v4: intra-wave software pipeline on the v2b body.  Iteration t
// holds S(t) from the previous iteration and issues QK^T(t+1) in the same
// scheduling region as softmax(t), so the 16 QK MFMAs of the next tile run
// under this tile's ~150 softmax VALU instructions; PV(t) follows.  K runs one
// tile ahead of V (iteration t reads K[t+1], V[t]; stages K[t+2], V[t+1]),
// register-staged into 2+2 LDS buffers, one barrier per tile.  S(t)/S(t+1)
// live in two named register sets (loop unrolled by 2: no runtime-indexed
// register arrays).
template <typename T, int D, int SGB>
__global__ __launch_bounds__(512, 2) void attn_fwd_v4(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
    const uint16_t* __restrict__ v, uint16_t* __restrict__ o, int H, int group,
    int Nq, int Nk, AttnStrides st, float c, int causal, int qblocks,
    int nblocks) {
    using L = PadLayout<D>;
    constexpr int NW = 8, NT = 512;
    constexpr int CPR = D / 8;
    constexpr int RPI = NT / CPR;
    constexpr int CPT = KT / RPI;
    static_assert(NT % CPR == 0 && KT % RPI == 0, "staging must tile evenly");
    __shared__ __attribute__((aligned(16))) char smem[2 * L::BUF];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h32 = lane >> 5, l32 = lane & 31;
    const int lb = xcd_remap(blockIdx.x, nblocks);
    const int bh = lb / qblocks, qblk = lb % qblocks;
    const int b = bh / H, hq = bh % H, hk = hq / group;
    const int qbase = qblk * (NW * QW);
    const int q0 = qbase + wave * QW;
    const int off_diag = Nk - Nq;

    const uint16_t* qp = q + b * st.qb + hq * st.qh;
    const uint16_t* kp = k + b * st.kb + hk * st.kh;
    const uint16_t* vp = v + b * st.vb + hk * st.vh;

    i32x4 qf[D / 16];
    {
        const int qr = q0 + l32;
        const bool ok = qr < Nq;
        const uint16_t* src = qp + (int64_t)(ok ? qr : 0) * st.qn + 8 * h32;
#pragma unroll
        for (int kk = 0; kk < D / 16; ++kk) {
            const i32x4 x = *reinterpret_cast<const i32x4*>(src + 16 * kk);
            qf[kk] = ok ? x : i32x4{0, 0, 0, 0};
        }
    }

    int kv_end = Nk;
    if (causal) kv_end = min(Nk, qbase + NW * QW + off_diag);
    const int nt = kv_end > 0 ? cdiv(kv_end, KT) : 0;
    const int t_full = Nk / KT;
    int t_mask = t_full;
    if (causal) t_mask = min(t_mask, max(0, (q0 + off_diag + 1) / KT));

    const int srow = tid / CPR, sch = tid % CPR;
    const uint16_t* kg = kp + (int64_t)srow * st.kn + sch * 8;
    const uint16_t* vg = vp + (int64_t)srow * st.vn + sch * 8;
    const int kw = srow * L::KS + sch * 16, vw = L::KSZ + srow * L::VS + sch * 16;
    auto load_rows = [&](i32x4 (&dst)[CPT], const uint16_t* gp, int64_t ld, int t) {
        if (t < t_full) {
#pragma unroll
            for (int i = 0; i < CPT; ++i)
                dst[i] = *reinterpret_cast<const i32x4*>(gp + ((int64_t)t * KT + i * RPI) * ld);
        } else {
#pragma unroll
            for (int i = 0; i < CPT; ++i) {
                const int key = t * KT + i * RPI + srow;
                const i32x4 x = *reinterpret_cast<const i32x4*>(gp + (int64_t)(min(key, Nk - 1) - srow) * ld);
                dst[i] = key < Nk ? x : i32x4{0, 0, 0, 0};
            }
        }
    };
    auto store_rows = [&](char* base, int off0, int stride, const i32x4 (&src)[CPT]) {
#pragma unroll
        for (int i = 0; i < CPT; ++i) lds_write_b128(base, off0 + i * RPI * stride, src[i]);
    };

    const int g = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;
    const int kr = l32 * L::KS + h32 * 16;
    const int vr = L::KSZ + (4 * h32 + qq) * L::VS + (2 * (g & 1) + (pp >> 1)) * 16 + 8 * (pp & 1);

    f32x16 oacc[D / 32];
#pragma unroll
    for (int d = 0; d < D / 32; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[d][r] = 0.f;
    float m_run = -1e30f, l_run = 0.f;

    auto qk = [&](int buf, f32x16 (&s)[2]) {
        const char* kb = smem + buf * L::BUF + kr;
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
#pragma unroll
            for (int r = 0; r < 16; ++r) s[tt][r] = 0.f;
#pragma unroll
            for (int kk = 0; kk < D / 16; ++kk)
                s[tt] = mfma32x32x16<T>(lds_read_b128(kb, tt * 32 * L::KS + kk * 32), qf[kk], s[tt]);
        }
    };

    i32x4 kst[CPT], vst[CPT];
    auto body = [&](auto mask_tag, f32x16 (&cur)[2], f32x16 (&nxt)[2], int t) {
        constexpr bool MASK = decltype(mask_tag)::value;
        if (t + 2 < nt) load_rows(kst, kg, st.kn, t + 2);
        if (t + 1 < nt) load_rows(vst, vg, st.vn, t + 1);

        // QK^T of tile t+1 (K[t+1] is resident; garbage and unused when t+1 == nt)
        qk((t + 1) & 1, nxt);

        if constexpr (MASK) {
            const int lim = causal ? q0 + l32 + off_diag : Nk;
#pragma unroll
            for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int key = t * KT + tt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h32;
                    if (key >= Nk || key > lim) cur[tt][r] = -INFINITY;
                }
        }
        float m4[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) m4[j] = max3(cur[0][4 * j], cur[1][4 * j], cur[0][4 * j + 1]);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            m4[j] = max3(m4[j], cur[1][4 * j + 1], cur[0][4 * j + 2]);
            m4[j] = max3(m4[j], cur[1][4 * j + 2], cur[0][4 * j + 3]);
            m4[j] = fmaxf(m4[j], cur[1][4 * j + 3]);
        }
        float mx = max3(m4[0], m4[1], max3(m4[2], m4[3], m4[0]));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float m_new = fmaxf(m_run, mx * c);
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        m_run = m_new;
        float rs[4] = {0.f, 0.f, 0.f, 0.f};
        i32x4 pb[2][2];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                float p[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    p[j] = __builtin_amdgcn_exp2f(fmaf(cur[tt][8 * s2 + j], c, -m_new));
                    rs[j & 3] += p[j];
                }
                pb[tt][s2] = i32x4{(int)pack2<T>(p[0], p[1]), (int)pack2<T>(p[2], p[3]),
                                   (int)pack2<T>(p[4], p[5]), (int)pack2<T>(p[6], p[7])};
            }
        l_run = fmaf(l_run, alpha, (rs[0] + rs[1]) + (rs[2] + rs[3]));
#pragma unroll
        for (int d = 0; d < D / 32; ++d)
#pragma unroll
            for (int r = 0; r < 16; ++r) oacc[d][r] *= alpha;

        const char* vb = smem + (t & 1) * L::BUF + vr;
#pragma unroll
        for (int dblk = 0; dblk < D / 32; ++dblk)
#pragma unroll
            for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    const int ro = (tt * 32 + 16 * s2) * L::VS + dblk * 64;
                    const i32x2 lo = lds_read_tr16(vb, ro);
                    const i32x2 hi = lds_read_tr16(vb, ro + 8 * L::VS);
                    oacc[dblk] = mfma32x32x16<T>(i32x4{lo.x, lo.y, hi.x, hi.y}, pb[tt][s2], oacc[dblk]);
                }

        if constexpr (SGB == 2) {
            // as SGB==1 but with the LDS fragment reads issued 3 MFMAs ahead
            __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                if (i < 13) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x402, 9, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
#pragma unroll
            for (int i = 0; i < 4 * (D / 32); ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                if (i < 4 * (D / 32) - 3) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x402, 2, 0);
            }
        }
        if constexpr (SGB == 1) {
            // Scheduling recipe for this region (LLVM SchedGroupMask bits:
            // VALU 0x2, MFMA 0x8, DS_READ 0x100, TRANS 0x400): QK^T(t+1)'s 16
            // MFMAs each followed by ~9 softmax VALU/TRANS ops, then PV's 16
            // MFMAs each behind its two transposed V reads.
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x402, 9, 0);
            }
#pragma unroll
            for (int i = 0; i < 4 * (D / 32); ++i) {
                __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x402, 2, 0);
            }
        }

        if (t + 2 < nt) store_rows(smem + (t & 1) * L::BUF, kw, L::KS, kst);
        if (t + 1 < nt) store_rows(smem + ((t + 1) & 1) * L::BUF, vw, L::VS, vst);
        __syncthreads();
    };

    f32x16 sA[2], sB[2];
    if (nt > 0) {
        load_rows(kst, kg, st.kn, 0);
        load_rows(vst, vg, st.vn, 0);
        store_rows(smem, kw, L::KS, kst);
        store_rows(smem, vw, L::VS, vst);
        if (nt > 1) {
            load_rows(kst, kg, st.kn, 1);
            store_rows(smem + L::BUF, kw, L::KS, kst);
        }
    }
    __syncthreads();
    if (nt > 0) qk(0, sA);
    for (int t = 0; t < nt;) {
        if (t < t_mask) body(std::false_type{}, sA, sB, t);
        else body(std::true_type{}, sA, sB, t);
        if (++t >= nt) break;
        if (t < t_mask) body(std::false_type{}, sB, sA, t);
        else body(std::true_type{}, sB, sA, t);
        ++t;
    }

    const float l = l_run + __shfl_xor(l_run, 32, 64);
    const float inv = l > 0.f ? 1.f / l : 0.f;
    const int qr = q0 + l32;
    if (qr < Nq) {
        uint16_t* op = o + b * st.ob + hq * st.oh + (int64_t)qr * st.on;
#pragma unroll
        for (int dblk = 0; dblk < D / 32; ++dblk)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int d = dblk * 32 + 8 * i + 4 * h32;
                const i32x2 w = {(int)pack2<T>(oacc[dblk][4 * i] * inv, oacc[dblk][4 * i + 1] * inv),
                                 (int)pack2<T>(oacc[dblk][4 * i + 2] * inv, oacc[dblk][4 * i + 3] * inv)};
                *reinterpret_cast<i32x2*>(op + d) = w;
            }
    }
}

// --------------------------------------------------------------------------
// attn_fwd_v5: 64 query rows per wave (two 32-row blocks), 4 waves = 256 rows
// per workgroup, ONE wave per SIMD with the 512-register budget.
//  * every K fragment read from LDS feeds two QK^T MFMAs and every V^T
//    fragment two PV MFMAs: half v2's LDS read traffic per MFMA;
//  * software pipeline across tiles inside the wave: the loop body is one
//    scheduling region holding QK^T(t+1) for both row blocks (32 MFMAs),
//    softmax(t) for both blocks (VALU), the O rescale and PV(t) (32 MFMAs),
//    so the softmax VALU fills the QK^T MFMA gaps of the same wave (there is
//    no partner wave on the SIMD to hide it);
//  * K runs one tile ahead of V (iteration t reads K[t+1], V[t]; stages
//    K[t+2], V[t+1] through registers into the padded 2+2 buffer ring).
template <typename T, int D, int SGB, bool DMA>
__global__ __launch_bounds__(256, 1) void attn_fwd_v5(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
    const uint16_t* __restrict__ v, uint16_t* __restrict__ o, int H, int group,
    int Nq, int Nk, AttnStrides st, float c, int causal, int qblocks,
    int nblocks) {
    using L = PadLayout<D>;
    constexpr int NW = 4, NT = 256;
    constexpr int CPR = D / 8;
    constexpr int RPI = NT / CPR;
    constexpr int CPT = KT / RPI;
    static_assert(NT % CPR == 0 && KT % RPI == 0, "staging must tile evenly");
    __shared__ __attribute__((aligned(16))) char smem[2 * L::BUF];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h32 = lane >> 5, l32 = lane & 31;
    const int lb = xcd_remap(blockIdx.x, nblocks);
    const int bh = lb / qblocks, qblk = lb % qblocks;
    const int b = bh / H, hq = bh % H, hk = hq / group;
    const int qbase = qblk * (NW * 2 * QW);
    const int qw0 = qbase + wave * 2 * QW;  // first row of this wave's 64
    const int off_diag = Nk - Nq;

    const uint16_t* qp = q + b * st.qb + hq * st.qh;
    const uint16_t* kp = k + b * st.kb + hk * st.kh;
    const uint16_t* vp = v + b * st.vb + hk * st.vh;

    i32x4 qf0[D / 16], qf1[D / 16];
    {
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
            const int qr = qw0 + rb * QW + l32;
            const bool ok = qr < Nq;
            const uint16_t* src = qp + (int64_t)(ok ? qr : 0) * st.qn + 8 * h32;
#pragma unroll
            for (int kk = 0; kk < D / 16; ++kk) {
                const i32x4 x = *reinterpret_cast<const i32x4*>(src + 16 * kk);
                (rb ? qf1 : qf0)[kk] = ok ? x : i32x4{0, 0, 0, 0};
            }
        }
    }

    int kv_end = Nk;
    if (causal) kv_end = min(Nk, qbase + NW * 2 * QW + off_diag);
    const int nt = kv_end > 0 ? cdiv(kv_end, KT) : 0;
    const int t_full = Nk / KT;
    int t_mask = t_full;
    if (causal) t_mask = min(t_mask, max(0, (qw0 + off_diag + 1) / KT));

    const int srow = tid / CPR, sch = tid % CPR;
    const uint16_t* kg = kp + (int64_t)srow * st.kn + sch * 8;
    const uint16_t* vg = vp + (int64_t)srow * st.vn + sch * 8;
    const int kw = srow * L::KS + sch * 16, vw = L::KSZ + srow * L::VS + sch * 16;
    auto load_rows = [&](i32x4 (&dst)[CPT], const uint16_t* gp, int64_t ld, int t) {
        if (t < t_full) {
#pragma unroll
            for (int i = 0; i < CPT; ++i)
                dst[i] = *reinterpret_cast<const i32x4*>(gp + ((int64_t)t * KT + i * RPI) * ld);
        } else {
#pragma unroll
            for (int i = 0; i < CPT; ++i) {
                const int key = t * KT + i * RPI + srow;
                const i32x4 x = *reinterpret_cast<const i32x4*>(gp + (int64_t)(min(key, Nk - 1) - srow) * ld);
                dst[i] = key < Nk ? x : i32x4{0, 0, 0, 0};
            }
        }
    };
    auto store_rows = [&](char* base, int off0, int stride, const i32x4 (&src)[CPT]) {
#pragma unroll
        for (int i = 0; i < CPT; ++i) lds_write_b128(base, off0 + i * RPI * stride, src[i]);
    };
    // DMA staging (global_load_lds_dwordx4): the padded tile is filled as
    // consecutive 1 KiB pieces; each lane derives its (row, chunk) from its
    // linear LDS position, lanes landing on a row's pad load a dummy chunk.
    // Rows past Nk are clamped to Nk-1 (finite; masked to -inf / weight 0).
    auto dma_tile = [&](char* dst, const uint16_t* base, int64_t ld, int stride, int bytes, int t) {
        for (int piece = wave; piece * 1024 < bytes; piece += NW) {
            const int pos = piece * 1024 + lane * 16;
            const int row = pos / stride, off = pos - row * stride;
            const int ch = off < 2 * D ? off >> 4 : 0;
            const int key = min(t * KT + row, Nk - 1);
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void*)(base + (int64_t)key * ld + ch * 8),
                (__attribute__((address_space(3))) void*)(dst + piece * 1024), 16, 0, 0);
        }
    };

    const int g = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;
    const int kr = l32 * L::KS + h32 * 16;
    const int vr = L::KSZ + (4 * h32 + qq) * L::VS + (2 * (g & 1) + (pp >> 1)) * 16 + 8 * (pp & 1);

    f32x16 o0[D / 32], o1[D / 32];
#pragma unroll
    for (int d = 0; d < D / 32; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) o0[d][r] = o1[d][r] = 0.f;
    float m0 = -1e30f, m1 = -1e30f, l0 = 0.f, l1 = 0.f;

    // S^T for both row blocks from one pass over K: each K fragment -> 2 MFMAs
    auto qk2 = [&](int buf, f32x16 (&s0)[2], f32x16 (&s1)[2]) {
        const char* kb = smem + buf * L::BUF + kr;
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
#pragma unroll
            for (int r = 0; r < 16; ++r) s0[tt][r] = s1[tt][r] = 0.f;
#pragma unroll
            for (int kk = 0; kk < D / 16; ++kk) {
                const i32x4 kf = lds_read_b128(kb, tt * 32 * L::KS + kk * 32);
                s0[tt] = mfma32x32x16<T>(kf, qf0[kk], s0[tt]);
                s1[tt] = mfma32x32x16<T>(kf, qf1[kk], s1[tt]);
            }
        }
    };
    auto mask = [&](f32x16 (&s)[2], int row0, int t) {
        const int lim = causal ? row0 + l32 + off_diag : Nk;
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int key = t * KT + tt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h32;
                if (key >= Nk || key > lim) s[tt][r] = -INFINITY;
            }
    };
    // online softmax of one 32-row block: returns alpha, fills pb, updates m/l
    auto softmax = [&](f32x16 (&s)[2], float& m_run, float& l_run, i32x4 (&pb)[2][2]) {
        float m4[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) m4[j] = max3(s[0][4 * j], s[1][4 * j], s[0][4 * j + 1]);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            m4[j] = max3(m4[j], s[1][4 * j + 1], s[0][4 * j + 2]);
            m4[j] = max3(m4[j], s[1][4 * j + 2], s[0][4 * j + 3]);
            m4[j] = fmaxf(m4[j], s[1][4 * j + 3]);
        }
        float mx = max3(m4[0], m4[1], max3(m4[2], m4[3], m4[0]));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float m_new = fmaxf(m_run, mx * c);
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        m_run = m_new;
        float rs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                float p[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    p[j] = __builtin_amdgcn_exp2f(fmaf(s[tt][8 * s2 + j], c, -m_new));
                    rs[j & 3] += p[j];
                }
                pb[tt][s2] = i32x4{(int)pack2<T>(p[0], p[1]), (int)pack2<T>(p[2], p[3]),
                                   (int)pack2<T>(p[4], p[5]), (int)pack2<T>(p[6], p[7])};
            }
        l_run = fmaf(l_run, alpha, (rs[0] + rs[1]) + (rs[2] + rs[3]));
        return alpha;
    };

    i32x4 kst[CPT], vst[CPT];
    auto body = [&](auto mask_tag, f32x16 (&c0)[2], f32x16 (&c1)[2], f32x16 (&n0)[2],
                    f32x16 (&n1)[2], int t) {
        constexpr bool MASK = decltype(mask_tag)::value;
        if constexpr (DMA) {
            if (t + 2 < nt) dma_tile(smem + (t & 1) * L::BUF, kp, st.kn, L::KS, L::KSZ, t + 2);
            if (t + 1 < nt) dma_tile(smem + ((t + 1) & 1) * L::BUF + L::KSZ, vp, st.vn, L::VS, L::VSZ, t + 1);
        } else {
            if (t + 2 < nt) load_rows(kst, kg, st.kn, t + 2);
            if (t + 1 < nt) load_rows(vst, vg, st.vn, t + 1);
        }

        qk2((t + 1) & 1, n0, n1);  // QK^T(t+1), unused when t+1 == nt
        if constexpr (MASK) {
            mask(c0, qw0, t);
            mask(c1, qw0 + QW, t);
        }
        i32x4 pb0[2][2], pb1[2][2];
        const float a0 = softmax(c0, m0, l0, pb0);
        const float a1 = softmax(c1, m1, l1, pb1);
#pragma unroll
        for (int d = 0; d < D / 32; ++d)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                o0[d][r] *= a0;
                o1[d][r] *= a1;
            }
        const char* vb = smem + (t & 1) * L::BUF + vr;
#pragma unroll
        for (int dblk = 0; dblk < D / 32; ++dblk)
#pragma unroll
            for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    const int ro = (tt * 32 + 16 * s2) * L::VS + dblk * 64;
                    const i32x2 lo = lds_read_tr16(vb, ro);
                    const i32x2 hi = lds_read_tr16(vb, ro + 8 * L::VS);
                    const i32x4 vf = {lo.x, lo.y, hi.x, hi.y};
                    o0[dblk] = mfma32x32x16<T>(vf, pb0[tt][s2], o0[dblk]);
                    o1[dblk] = mfma32x32x16<T>(vf, pb1[tt][s2], o1[dblk]);
                }
        if constexpr (SGB == 1) {
            // QK^T phase: K reads 4 ahead, ~8 softmax VALU/TRANS per MFMA gap;
            // PV phase: one tr read + 2 VALU per MFMA.
            __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
            for (int i = 0; i < 32; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                if ((i & 1) && i < 24) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x402, 8, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
            for (int i = 0; i < 32; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x402, 2, 0);
            }
        }
        if constexpr (!DMA) {
            if (t + 2 < nt) store_rows(smem + (t & 1) * L::BUF, kw, L::KS, kst);
            if (t + 1 < nt) store_rows(smem + ((t + 1) & 1) * L::BUF, vw, L::VS, vst);
        }
        __syncthreads();  // (DMA: vmcnt(0) first -- the prefetched tiles have landed)
    };

    f32x16 sA0[2], sA1[2], sB0[2], sB1[2];
    if (nt > 0) {
        load_rows(kst, kg, st.kn, 0);
        load_rows(vst, vg, st.vn, 0);
        store_rows(smem, kw, L::KS, kst);
        store_rows(smem, vw, L::VS, vst);
        if (nt > 1) {
            load_rows(kst, kg, st.kn, 1);
            store_rows(smem + L::BUF, kw, L::KS, kst);
        }
    }
    __syncthreads();
    if (nt > 0) qk2(0, sA0, sA1);
    for (int t = 0; t < nt;) {
        if (t < t_mask) body(std::false_type{}, sA0, sA1, sB0, sB1, t);
        else body(std::true_type{}, sA0, sA1, sB0, sB1, t);
        if (++t >= nt) break;
        if (t < t_mask) body(std::false_type{}, sB0, sB1, sA0, sA1, t);
        else body(std::true_type{}, sB0, sB1, sA0, sA1, t);
        ++t;
    }

#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
        const float lr = rb ? l1 : l0;
        const float l = lr + __shfl_xor(lr, 32, 64);
        const float inv = l > 0.f ? 1.f / l : 0.f;
        const int qr = qw0 + rb * QW + l32;
        if (qr < Nq) {
            uint16_t* op = o + b * st.ob + hq * st.oh + (int64_t)qr * st.on;
#pragma unroll
            for (int dblk = 0; dblk < D / 32; ++dblk)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const f32x16& acc = rb ? o1[dblk] : o0[dblk];
                    const int d = dblk * 32 + 8 * i + 4 * h32;
                    const i32x2 w = {(int)pack2<T>(acc[4 * i] * inv, acc[4 * i + 1] * inv),
                                     (int)pack2<T>(acc[4 * i + 2] * inv, acc[4 * i + 3] * inv)};
                    *reinterpret_cast<i32x2*>(op + d) = w;
                }
        }
    }
}

// --------------------------------------------------------------------------
// attn_fwd_v6: v2's structure on v_mfma_f32_16x16x32 (the shape MI355X holds
// a higher clock on under load).  Each wave owns 32 query rows as two 16-row
// blocks, so every K and V^T fragment read from LDS feeds two MFMAs.
//   S^T[16 keys][16 q] = K[16 keys, 32 d] . Q^T : lane l holds query row l&15
//      of its block and keys 4(l>>4)+r (r = 0..3) of each 16-key block;
//   P^T fragment of a 32-key k-step s = the S registers of key blocks 2s and
//      2s+1 (k order permuted: j<4 -> key 32s+4g+j, j>=4 -> 32s+16+4g+j-4),
//      V^T fragment = two ds_read_b64_tr_b16 of the same permuted rows.
// V rows are padded to 2D+32 B so the 8 rows x 32 B of a half-wave's
// transposed read cover all 64 banks.
template <int D> struct PadLayout16 {
    static constexpr int KS = 2 * D + 16;
    static constexpr int VS = 2 * D + 32;
    static constexpr int KSZ = KT * KS, VSZ = KT * VS, BUF = KSZ + VSZ;
};

template <typename T, int D>
__global__ __launch_bounds__(512, 2) void attn_fwd_v6(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
    const uint16_t* __restrict__ v, uint16_t* __restrict__ o, int H, int group,
    int Nq, int Nk, AttnStrides st, float c, int causal, int qblocks,
    int nblocks) {
    using L = PadLayout16<D>;
    constexpr int NW = 8, NT = 512;
    constexpr int CPR = D / 8;
    constexpr int RPI = NT / CPR;
    constexpr int CPT = KT / RPI;
    constexpr int KSTEPS = D / 32;  // 32-d k-steps of QK^T
    constexpr int DB = D / 16;      // 16-d output blocks
    static_assert(NT % CPR == 0 && KT % RPI == 0, "staging must tile evenly");
    __shared__ __attribute__((aligned(16))) char smem[2 * L::BUF];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int l16 = lane & 15, g = lane >> 4;
    const int lb = xcd_remap(blockIdx.x, nblocks);
    const int bh = lb / qblocks;
    const int qblk = causal ? qblocks - 1 - lb % qblocks : lb % qblocks;
    const int b = bh / H, hq = bh % H, hk = hq / group;
    const int qbase = qblk * (NW * QW);
    const int q0 = qbase + wave * QW;
    const int off_diag = Nk - Nq;

    const uint16_t* qp = q + b * st.qb + hq * st.qh;
    const uint16_t* kp = k + b * st.kb + hk * st.kh;
    const uint16_t* vp = v + b * st.vb + hk * st.vh;

    // Q^T fragments: block qb, k-step ks: Q[q0+16qb+l16][32ks+8g .. +7]
    i32x4 qf[2][KSTEPS];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
        const int qr = q0 + 16 * qb + l16;
        const bool ok = qr < Nq;
        const uint16_t* src = qp + (int64_t)(ok ? qr : 0) * st.qn + 8 * g;
#pragma unroll
        for (int ks = 0; ks < KSTEPS; ++ks) {
            const i32x4 x = *reinterpret_cast<const i32x4*>(src + 32 * ks);
            qf[qb][ks] = ok ? x : i32x4{0, 0, 0, 0};
        }
    }

    int kv_end = Nk;
    if (causal) kv_end = min(Nk, qbase + NW * QW + off_diag);
    const int nt = kv_end > 0 ? cdiv(kv_end, KT) : 0;
    const int t_full = Nk / KT;
    int t_mask = t_full;
    if (causal) t_mask = min(t_mask, max(0, (q0 + off_diag + 1) / KT));

    const int srow = tid / CPR, sch = tid % CPR;
    const uint16_t* kg = kp + (int64_t)srow * st.kn + sch * 8;
    const uint16_t* vg = vp + (int64_t)srow * st.vn + sch * 8;
    const int kw = srow * L::KS + sch * 16, vw = L::KSZ + srow * L::VS + sch * 16;
    i32x4 kst[CPT], vst[CPT];
    auto load_tile = [&](int t) {
        if (t < t_full) {
#pragma unroll
            for (int i = 0; i < CPT; ++i) {
                const int64_t r = (int64_t)t * KT + i * RPI;
                kst[i] = *reinterpret_cast<const i32x4*>(kg + r * st.kn);
                vst[i] = *reinterpret_cast<const i32x4*>(vg + r * st.vn);
            }
        } else {
#pragma unroll
            for (int i = 0; i < CPT; ++i) {
                const int key = t * KT + i * RPI + srow;
                const int64_t r = min(key, Nk - 1) - srow;
                const i32x4 kx = *reinterpret_cast<const i32x4*>(kg + r * st.kn);
                const i32x4 vx = *reinterpret_cast<const i32x4*>(vg + r * st.vn);
                kst[i] = key < Nk ? kx : i32x4{0, 0, 0, 0};
                vst[i] = key < Nk ? vx : i32x4{0, 0, 0, 0};
            }
        }
    };
    auto store_tile = [&](int buf) {
        char* base = smem + buf * L::BUF;
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
            lds_write_b128(base, kw + i * RPI * L::KS, kst[i]);
            lds_write_b128(base, vw + i * RPI * L::VS, vst[i]);
        }
    };

    const int qq = l16 >> 2, pp = lane & 3;
    const int kr = l16 * L::KS + g * 16;                                  // K: key l16, chunk g
    const int vr = L::KSZ + (4 * g + qq) * L::VS + 8 * pp;                 // V: key 4g+qq, col 4pp

    f32x4 oacc[2][DB];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
        for (int d = 0; d < DB; ++d) oacc[qb][d] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m_run[2] = {-1e30f, -1e30f}, l_run[2] = {0.f, 0.f};

    if (nt > 0) {
        load_tile(0);
        store_tile(0);
    }
    __syncthreads();

    for (int t = 0; t < nt; ++t) {
        if (t + 1 < nt) load_tile(t + 1);
        const char* kb = smem + (t & 1) * L::BUF + kr;
        const char* vb = smem + (t & 1) * L::BUF + vr;

        f32x4 s[2][4];  // [q block][16-key block]
#pragma unroll
        for (int qb = 0; qb < 2; ++qb)
#pragma unroll
            for (int kb2 = 0; kb2 < 4; ++kb2) s[qb][kb2] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kb2 = 0; kb2 < 4; ++kb2)
#pragma unroll
            for (int ks = 0; ks < KSTEPS; ++ks) {
                const i32x4 kf = lds_read_b128(kb, kb2 * 16 * L::KS + ks * 64);
                s[0][kb2] = mfma16x16x32<T>(kf, qf[0][ks], s[0][kb2]);
                s[1][kb2] = mfma16x16x32<T>(kf, qf[1][ks], s[1][kb2]);
            }

        if (t >= t_mask) {
#pragma unroll
            for (int qb = 0; qb < 2; ++qb) {
                const int lim = causal ? q0 + 16 * qb + l16 + off_diag : Nk;
#pragma unroll
                for (int kb2 = 0; kb2 < 4; ++kb2)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int key = t * KT + 16 * kb2 + 4 * g + r;
                        if (key >= Nk || key > lim) s[qb][kb2][r] = -INFINITY;
                    }
            }
        }

        i32x4 pb[2][2];
        float alpha[2];
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
            float mx = max3(s[qb][0][0], s[qb][0][1], s[qb][0][2]);
            float my = max3(s[qb][0][3], s[qb][1][0], s[qb][1][1]);
            mx = max3(mx, s[qb][1][2], s[qb][1][3]);
            my = max3(my, s[qb][2][0], s[qb][2][1]);
            mx = max3(mx, s[qb][2][2], s[qb][2][3]);
            my = max3(my, s[qb][3][0], s[qb][3][1]);
            mx = max3(mx, s[qb][3][2], s[qb][3][3]);
            mx = fmaxf(mx, my);
            mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
            mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
            const float m_new = fmaxf(m_run[qb], mx * c);
            alpha[qb] = __builtin_amdgcn_exp2f(m_run[qb] - m_new);
            m_run[qb] = m_new;
            float rs0 = 0.f, rs1 = 0.f;
#pragma unroll
            for (int kb2 = 0; kb2 < 4; ++kb2)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float pv = __builtin_amdgcn_exp2f(fmaf(s[qb][kb2][r], c, -m_new));
                    s[qb][kb2][r] = pv;
                    if (r & 1) rs1 += pv; else rs0 += pv;
                }
            l_run[qb] = fmaf(l_run[qb], alpha[qb], rs0 + rs1);
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2)
                pb[qb][s2] = i32x4{(int)pack2<T>(s[qb][2 * s2][0], s[qb][2 * s2][1]),
                                   (int)pack2<T>(s[qb][2 * s2][2], s[qb][2 * s2][3]),
                                   (int)pack2<T>(s[qb][2 * s2 + 1][0], s[qb][2 * s2 + 1][1]),
                                   (int)pack2<T>(s[qb][2 * s2 + 1][2], s[qb][2 * s2 + 1][3])};
#pragma unroll
            for (int d = 0; d < DB; ++d) oacc[qb][d] *= alpha[qb];
        }

#pragma unroll
        for (int d = 0; d < DB; ++d)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const int ro = 32 * s2 * L::VS + d * 32;
                const i32x2 lo = lds_read_tr16(vb, ro);
                const i32x2 hi = lds_read_tr16(vb, ro + 16 * L::VS);
                const i32x4 vf = {lo.x, lo.y, hi.x, hi.y};
                oacc[0][d] = mfma16x16x32<T>(vf, pb[0][s2], oacc[0][d]);
                oacc[1][d] = mfma16x16x32<T>(vf, pb[1][s2], oacc[1][d]);
            }

        if (t + 1 < nt) store_tile((t + 1) & 1);
        __syncthreads();
    }

#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
        float l = l_run[qb] + __shfl_xor(l_run[qb], 16, 64);
        l += __shfl_xor(l, 32, 64);
        const float inv = l > 0.f ? 1.f / l : 0.f;
        const int qr = q0 + 16 * qb + l16;
        if (qr < Nq) {
            uint16_t* op = o + b * st.ob + hq * st.oh + (int64_t)qr * st.on;
#pragma unroll
            for (int d = 0; d < DB; ++d) {
                const f32x4 a = oacc[qb][d];
                *reinterpret_cast<i32x2*>(op + d * 16 + 4 * g) =
                    i32x2{(int)pack2<T>(a[0] * inv, a[1] * inv), (int)pack2<T>(a[2] * inv, a[3] * inv)};
            }
        }
    }
}

// --------------------------------------------------------------------------
// attn_fwd_v3: v2 with the two waves of each SIMD staggered.  A workgroup's
// waves w and w+4 share a SIMD; in v2 both run QK^T-MFMA, softmax-VALU,
// PV-MFMA in lockstep between barriers, so the SIMD alternates between a
// saturated matrix pipe and a saturated VALU.  Here waves 0-3 ("A") run
//     QK^T(t) | softmax(t) | PV(t)
// and waves 4-7 ("B") run the rotated body
//     softmax(t) | PV(t) | QK^T(t+1)
// inside the same barrier interval: B's softmax VALU overlaps A's QK^T MFMAs
// and A's softmax overlaps B's PV, so only the last third is MFMA vs MFMA.
// B needs K[t+1] during interval t, so K runs in a 3-buffer ring
// (K[t], K[t+1] read, K[t+2] being staged) and V in 2 buffers.
template <typename T, int D, bool QLDS>
__global__ __launch_bounds__(512, 2) void attn_fwd_v3(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
    const uint16_t* __restrict__ v, uint16_t* __restrict__ o, int H, int group,
    int Nq, int Nk, AttnStrides st, float c, int causal, int qblocks,
    int nblocks) {
    using L = PadLayout<D>;
    constexpr int NW = 8, NT = 512;
    constexpr int CPR = D / 8;
    constexpr int RPI = NT / CPR;
    constexpr int CPT = KT / RPI;
    static_assert(NT % CPR == 0 && KT % RPI == 0, "staging must tile evenly");
    constexpr int QSZ = QLDS ? NW * QW * L::KS : 0;  // Q tile, K-style padded rows
    __shared__ __attribute__((aligned(16))) char smem[3 * L::KSZ + 2 * L::VSZ + QSZ];
    char* const vbase = smem + 3 * L::KSZ;
    char* const qbase_lds = vbase + 2 * L::VSZ;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h32 = lane >> 5, l32 = lane & 31;
    const bool grpB = __builtin_amdgcn_readfirstlane(wave) >= 4;
    const int lb = xcd_remap(blockIdx.x, nblocks);
    const int bh = lb / qblocks, qblk = lb % qblocks;
    const int b = bh / H, hq = bh % H, hk = hq / group;
    const int qbase = qblk * (NW * QW);
    const int q0 = qbase + wave * QW;
    const int off_diag = Nk - Nq;

    const uint16_t* qp = q + b * st.qb + hq * st.qh;
    const uint16_t* kp = k + b * st.kb + hk * st.kh;
    const uint16_t* vp = v + b * st.vb + hk * st.vh;

    // Q^T fragments: in registers, or (QLDS) in a padded LDS tile re-read per
    // tile (frees 32 VGPRs at D=128).  Lane: row q0+l32, d = 16kk + 8h32 .. +7.
    i32x4 qf[QLDS ? 1 : D / 16];
    {
        const int qr = q0 + l32;
        const bool ok = qr < Nq;
        const uint16_t* src = qp + (int64_t)(ok ? qr : 0) * st.qn + 8 * h32;
#pragma unroll
        for (int kk = 0; kk < D / 16; ++kk) {
            const i32x4 x = *reinterpret_cast<const i32x4*>(src + 16 * kk);
            if constexpr (QLDS)
                lds_write_b128(qbase_lds, (wave * QW + l32) * L::KS + (2 * kk + h32) * 16,
                               ok ? x : i32x4{0, 0, 0, 0});
            else
                qf[kk] = ok ? x : i32x4{0, 0, 0, 0};
        }
    }
    const char* qfr = qbase_lds + (wave * QW + l32) * L::KS + h32 * 16;

    int kv_end = Nk;
    if (causal) kv_end = min(Nk, qbase + NW * QW + off_diag);
    const int nt = kv_end > 0 ? cdiv(kv_end, KT) : 0;
    const int t_full = Nk / KT;
    int t_mask = t_full;
    if (causal) t_mask = min(t_mask, max(0, (q0 + off_diag + 1) / KT));

    const int srow = tid / CPR, sch = tid % CPR;
    const uint16_t* kg = kp + (int64_t)srow * st.kn + sch * 8;
    const uint16_t* vg = vp + (int64_t)srow * st.vn + sch * 8;
    const int kw = srow * L::KS + sch * 16, vw = srow * L::VS + sch * 16;
    auto load_rows = [&](i32x4 (&dst)[CPT], const uint16_t* g, int64_t ld, int t) {
        if (t < t_full) {
#pragma unroll
            for (int i = 0; i < CPT; ++i)
                dst[i] = *reinterpret_cast<const i32x4*>(g + ((int64_t)t * KT + i * RPI) * ld);
        } else {
#pragma unroll
            for (int i = 0; i < CPT; ++i) {
                const int key = t * KT + i * RPI + srow;
                const i32x4 x = *reinterpret_cast<const i32x4*>(g + (int64_t)(min(key, Nk - 1) - srow) * ld);
                dst[i] = key < Nk ? x : i32x4{0, 0, 0, 0};
            }
        }
    };
    auto store_k = [&](int buf, const i32x4 (&src)[CPT]) {
#pragma unroll
        for (int i = 0; i < CPT; ++i) lds_write_b128(smem + buf * L::KSZ, kw + i * RPI * L::KS, src[i]);
    };
    auto store_v = [&](int buf, const i32x4 (&src)[CPT]) {
#pragma unroll
        for (int i = 0; i < CPT; ++i) lds_write_b128(vbase + buf * L::VSZ, vw + i * RPI * L::VS, src[i]);
    };

    const int g = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;
    const int kr = l32 * L::KS + h32 * 16;
    const int vr = (4 * h32 + qq) * L::VS + (2 * (g & 1) + (pp >> 1)) * 16 + 8 * (pp & 1);

    f32x16 oacc[D / 32];
#pragma unroll
    for (int d = 0; d < D / 32; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[d][r] = 0.f;
    float m_run = -1e30f, l_run = 0.f;
    f32x16 s[2];

    auto qk = [&](int kbuf) {
        const char* kb = smem + kbuf * L::KSZ + kr;
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
#pragma unroll
            for (int r = 0; r < 16; ++r) s[tt][r] = 0.f;
#pragma unroll
            for (int kk = 0; kk < D / 16; ++kk) {
                const i32x4 qv = QLDS ? lds_read_b128(qfr, kk * 32) : qf[QLDS ? 0 : kk];
                s[tt] = mfma32x32x16<T>(lds_read_b128(kb, tt * 32 * L::KS + kk * 32), qv, s[tt]);
            }
        }
    };
    auto softmax_pv = [&](int t, int vbuf) {
        if (t >= t_mask) {
            const int lim = causal ? q0 + l32 + off_diag : Nk;
#pragma unroll
            for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int key = t * KT + tt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h32;
                    if (key >= Nk || key > lim) s[tt][r] = -INFINITY;
                }
        }
        float mx = max3(s[0][0], s[1][0], s[0][1]);
        float my = max3(s[1][1], s[0][2], s[1][2]);
#pragma unroll
        for (int r = 3; r < 15; r += 2) {
            mx = max3(mx, s[0][r], s[1][r]);
            my = max3(my, s[0][r + 1], s[1][r + 1]);
        }
        mx = max3(mx, my, max3(s[0][15], s[1][15], mx));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float m_new = fmaxf(m_run, mx * c);
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        m_run = m_new;
        float rs = 0.f;
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float p = __builtin_amdgcn_exp2f(fmaf(s[tt][r], c, -m_new));
                s[tt][r] = p;
                rs += p;
            }
        l_run = fmaf(l_run, alpha, rs);
#pragma unroll
        for (int d = 0; d < D / 32; ++d)
#pragma unroll
            for (int r = 0; r < 16; ++r) oacc[d][r] *= alpha;
        i32x4 pb[2][2];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const int r0 = 8 * s2;
                pb[tt][s2] = i32x4{(int)pack2<T>(s[tt][r0 + 0], s[tt][r0 + 1]),
                                   (int)pack2<T>(s[tt][r0 + 2], s[tt][r0 + 3]),
                                   (int)pack2<T>(s[tt][r0 + 4], s[tt][r0 + 5]),
                                   (int)pack2<T>(s[tt][r0 + 6], s[tt][r0 + 7])};
            }
        const char* vb = vbase + vbuf * L::VSZ + vr;
#pragma unroll
        for (int dblk = 0; dblk < D / 32; ++dblk)
#pragma unroll
            for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    const int ro = (tt * 32 + 16 * s2) * L::VS + dblk * 64;
                    const i32x2 lo = lds_read_tr16(vb, ro);
                    const i32x2 hi = lds_read_tr16(vb, ro + 8 * L::VS);
                    oacc[dblk] = mfma32x32x16<T>(i32x4{lo.x, lo.y, hi.x, hi.y}, pb[tt][s2], oacc[dblk]);
                }
    };

    i32x4 kst[CPT], vst[CPT];
    if (nt > 0) {
        load_rows(kst, kg, st.kn, 0);
        load_rows(vst, vg, st.vn, 0);
        store_k(0, kst);
        store_v(0, vst);
        if (nt > 1) {
            load_rows(kst, kg, st.kn, 1);
            store_k(1, kst);
        }
    }
    __syncthreads();
    if (grpB && nt > 0) qk(0);

    int kc = 0;  // K ring slot of tile t
    for (int t = 0; t < nt; ++t) {
        const int kn1 = kc == 2 ? 0 : kc + 1, kn2 = kn1 == 2 ? 0 : kn1 + 1;
        if (t + 1 < nt) load_rows(vst, vg, st.vn, t + 1);
        if (t + 2 < nt) load_rows(kst, kg, st.kn, t + 2);
        if (!grpB) {
            qk(kc);
            softmax_pv(t, t & 1);
        } else {
            softmax_pv(t, t & 1);
            // keep QK^T(t+1)'s fragment reads below the PV MFMAs: hoisting
            // them above doubles the live fragment registers and spills
            __builtin_amdgcn_sched_barrier(0);
            if (t + 1 < nt) qk(kn1);
        }
        if (t + 1 < nt) store_v((t + 1) & 1, vst);
        if (t + 2 < nt) store_k(kn2, kst);
        __syncthreads();
        kc = kn1;
    }

    const float l = l_run + __shfl_xor(l_run, 32, 64);
    const float inv = l > 0.f ? 1.f / l : 0.f;
    const int qr = q0 + l32;
    if (qr < Nq) {
        uint16_t* op = o + b * st.ob + hq * st.oh + (int64_t)qr * st.on;
#pragma unroll
        for (int dblk = 0; dblk < D / 32; ++dblk)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int d = dblk * 32 + 8 * i + 4 * h32;
                const i32x2 w = {(int)pack2<T>(oacc[dblk][4 * i] * inv, oacc[dblk][4 * i + 1] * inv),
                                 (int)pack2<T>(oacc[dblk][4 * i + 2] * inv, oacc[dblk][4 * i + 3] * inv)};
                *reinterpret_cast<i32x2*>(op + d) = w;
            }
    }
}

// --------------------------------------------------------------------------
// Generic kernel: 256 threads own 32 query rows (8 threads per row, each
// thread owns columns sub + 8u of the score tile and d = sub + 8u of O).
constexpr int GQ = 32, GK = 64, GDMAX = 128;

template <typename T>
__global__ __launch_bounds__(256) void attn_fwd_generic(
    const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v,
    T* __restrict__ o, int H, int group, int Nq, int Nk, int D, AttnStrides st,
    float scale, int causal, int qblocks) {
    extern __shared__ __attribute__((aligned(16))) float gsm[];
    const int ldq = D + 1;
    float* Qs = gsm;                 // [GQ][D+1]
    float* Ks = Qs + GQ * ldq;       // [GK][D+1]
    float* Vs = Ks + GK * ldq;       // [GK][D]
    float* Ps = Vs + GK * D;         // [GQ][GK+1]

    const int tid = threadIdx.x, row = tid >> 3, sub = tid & 7;
    const int bh = blockIdx.x / qblocks, qblk = blockIdx.x % qblocks;
    const int b = bh / H, hq = bh % H, hk = hq / group;
    const int q0 = qblk * GQ;
    const int off_diag = Nk - Nq;
    const T* qp = q + b * st.qb + hq * st.qh;
    const T* kp = k + b * st.kb + hk * st.kh;
    const T* vp = v + b * st.vb + hk * st.vh;

    for (int i = tid; i < GQ * D; i += 256) {
        const int r = i / D, d = i % D;
        Qs[r * ldq + d] = (q0 + r < Nq) ? elem<T>::to_f32(qp[(int64_t)(q0 + r) * st.qn + d]) : 0.f;
    }

    float acc[GDMAX / 8];
#pragma unroll
    for (int u = 0; u < GDMAX / 8; ++u) acc[u] = 0.f;
    float m_run = -INFINITY, l_run = 0.f;
    const int qi = q0 + row;
    const int lim = causal ? qi + off_diag : Nk - 1;
    int kv_end = Nk;
    if (causal) kv_end = min(Nk, q0 + GQ + off_diag);

    for (int k0 = 0; k0 < kv_end; k0 += GK) {
        __syncthreads();
        for (int i = tid; i < GK * D; i += 256) {
            const int r = i / D, d = i % D;
            const bool ok = k0 + r < Nk;
            Ks[r * ldq + d] = ok ? elem<T>::to_f32(kp[(int64_t)(k0 + r) * st.kn + d]) : 0.f;
            Vs[r * D + d] = ok ? elem<T>::to_f32(vp[(int64_t)(k0 + r) * st.vn + d]) : 0.f;
        }
        __syncthreads();
        float sc[GK / 8];
        float mx = -INFINITY;
#pragma unroll
        for (int u = 0; u < GK / 8; ++u) {
            const int j = sub + 8 * u;
            float dot = 0.f;
            for (int d = 0; d < D; ++d) dot = fmaf(Qs[row * ldq + d], Ks[j * ldq + d], dot);
            const int key = k0 + j;
            dot = (key < Nk && key <= lim) ? dot * scale : -INFINITY;
            sc[u] = dot;
            mx = fmaxf(mx, dot);
        }
#pragma unroll
        for (int o2 = 1; o2 < 8; o2 <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o2, 64));
        const float m_new = fmaxf(m_run, mx);
        const float alpha = (m_new == -INFINITY) ? 1.f : expf(m_run - m_new);
        float rs = 0.f;
#pragma unroll
        for (int u = 0; u < GK / 8; ++u) {
            const float p = (m_new == -INFINITY) ? 0.f : expf(sc[u] - m_new);
            Ps[row * (GK + 1) + sub + 8 * u] = p;
            rs += p;
        }
#pragma unroll
        for (int o2 = 1; o2 < 8; o2 <<= 1) rs += __shfl_xor(rs, o2, 64);
        l_run = l_run * alpha + rs;
        m_run = m_new;
        __syncthreads();
#pragma unroll
        for (int u = 0; u < GDMAX / 8; ++u) {
            const int d = sub + 8 * u;
            if (d < D) {
                float a = acc[u] * alpha;
                for (int j = 0; j < GK; ++j) a = fmaf(Ps[row * (GK + 1) + j], Vs[j * D + d], a);
                acc[u] = a;
            }
        }
    }
    if (qi < Nq) {
        const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
        T* op = o + b * st.ob + hq * st.oh + (int64_t)qi * st.on;
#pragma unroll
        for (int u = 0; u < GDMAX / 8; ++u) {
            const int d = sub + 8 * u;
            if (d < D) op[d] = elem<T>::from_f32(acc[u] * inv);
        }
    }
}

// --------------------------------------------------------------------------
// attn_fwd_seg: segmented 8-wave structure (D = 128).  Each 64-key tile is
// four barrier-separated segments per wave,
//   S1 load:    K(t) fragments LDS -> registers (16 ds_read_b128) + LDS-DMA of K(t+2)
//   S2 compute: S(t) = K(t) Q^T (16 MFMAs, registers only)
//   S3 load:    V(t-1)^T fragments -> the same registers (32 ds_read_b64_tr_b16)
//               + LDS-DMA of V(t+1)
//   S4 compute: O += P(t-1) V(t-1) (16 MFMAs) beside softmax(t): mask, row
//               max, deferred running max, exp2, bf16 pack -> P(t), rounded
//               row sum (P double-buffered in registers, S(t) lives S2-S4)
// and waves 4-7 run one segment behind waves 0-3, so the two waves of every
// SIMD pair a compute segment with a load segment.  K and V tiles arrive by
// LDS-DMA (global_load_lds, 1 KiB lane-linear pieces, two per wave per tile)
// into 3-deep rings of XOR-swizzled [64][256 B] images (chunk ^= (row&3)<<2 |
// (row>>2)&3, applied on the DMA source address): a buffer is restaged >= 4
// segments after its last read, and the counted vmcnt(4) at the end of S2
// (retires K(t+1)) and S4 (retires V(t)) precedes, for both halves, the
// barrier before the first read.  Softmax as variant 21 (defer-max, rounded
// row sum, permlane row max).  SGB: sched_group_barrier interleave of the
// compute segments.
template <typename T, int SGB>
__global__ __launch_bounds__(512, 2) void attn_fwd_seg(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
    const uint16_t* __restrict__ v, uint16_t* __restrict__ o, int H, int group,
    int Nq, int Nk, AttnStrides st, float c, int causal, int qblocks,
    int nblocks) {
    constexpr int D = 128, NW = 8, TB = KT * 256;  // one 16 KiB tile image
    __shared__ __attribute__((aligned(1024))) char smem[6 * TB];  // K ring 0-2, V ring 3-5

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // scalar: DMA destinations in SGPRs
    const int h32 = lane >> 5, l32 = lane & 31;
    const int lag = wave >> 2;  // 1: the half that runs one segment behind
    const int lb = xcd_remap(blockIdx.x, nblocks);
    const int bh = lb / qblocks;
    const int qblk = causal ? qblocks - 1 - lb % qblocks : lb % qblocks;
    const int b = bh / H, hq = bh % H, hk = hq / group;
    const int qbase = qblk * (NW * QW);
    const int q0 = qbase + wave * QW;
    const int off_diag = Nk - Nq;

    const uint16_t* qp = q + b * st.qb + hq * st.qh;
    const uint16_t* kp = k + b * st.kb + hk * st.kh;
    const uint16_t* vp = v + b * st.vb + hk * st.vh;

    int kv_end = Nk;
    if (causal) kv_end = min(Nk, qbase + NW * QW + off_diag);
    const int nt = kv_end > 0 ? cdiv(kv_end, KT) : 0;
    int t_mask = Nk / KT;
    if (causal) t_mask = min(t_mask, max(0, (q0 + off_diag + 1) / KT));

    // LDS-DMA plan: piece 2*wave+i of a tile image = rows 4*piece .. +3;
    // lane -> row 4*piece + (lane>>4), physical chunk lane&15 = logical chunk
    // (lane&15) ^ f(row)
    auto fsw = [](int row) { return ((row & 3) << 2) | ((row >> 2) & 3); };
    // per-lane element offsets of the two pieces inside a tile (32-bit: the
    // tile's own offset t*KT*stride is scalar)
    int drow[2], koff[2], voff[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        drow[i] = 4 * (2 * wave + i) + (lane >> 4);
        const int ch = (lane & 15) ^ fsw(drow[i]);
        koff[i] = drow[i] * (int)st.kn + 8 * ch;
        voff[i] = drow[i] * (int)st.vn + 8 * ch;
    }
    auto dma = [&](const uint16_t* base, int64_t sn, const int (&off)[2], int t, char* img) {
        const uint16_t* tb = base + (int64_t)t * KT * sn;
        const bool ragged = t * KT + KT > Nk;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            int o = off[i];
            if (ragged && t * KT + drow[i] >= Nk)  // rows past Nk re-read row Nk-1 (masked / P = 0)
                o += (Nk - 1 - t * KT - drow[i]) * (int)sn;
            // inline asm: hipcc's waitcnt pass does not see it, so it does not
            // drain it with vmcnt(0) before the (alias-unknown) tr_b16 reads;
            // the counted vmcnt(4) waits below order every use
            const uint32_t m0v = lds_addr(img + (2 * wave + i) * 1024);
            asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
                         :: "s"(m0v), "v"(tb + o) : "memory", "m0");
        }
    };
    auto kimg = [&](int t) { return smem + (t % 3) * TB; };
    auto vimg = [&](int t) { return smem + (3 + t % 3) * TB; };

    // fragment addresses (see the derivation in DESIGN.md §3.1):
    //   K: row tt*32 + l32, chunk 2kk + h32  -> (A0 ^ (kk << 5)) + tt * 8192
    //   V^T: rows tt*32 + 16*s2 + 4*h32 + qq (+8), chunk 4*dblk + c0
    //        -> (B0 ^ (dblk << 6) [^ 32]) + (tt*32 + 16*s2) * 256 [+ 2048]
    const int g = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;
    int A0 = l32 * 256 + ((h32 ^ fsw(l32)) << 4);
    const int c0 = 2 * (g & 1) + (pp >> 1);
    int B0 = (4 * h32 + qq) * 256 + ((c0 ^ ((qq << 2) | h32)) << 4) + 8 * (pp & 1);

    i32x4 qf[D / 16];
    {
        const int qr = q0 + l32;
        const bool ok = qr < Nq;
        const uint16_t* src = qp + (int64_t)(ok ? qr : 0) * st.qn + 8 * h32;
#pragma unroll
        for (int kk = 0; kk < D / 16; ++kk) {
            const i32x4 x = *reinterpret_cast<const i32x4*>(src + 16 * kk);
            qf[kk] = ok ? x : i32x4{0, 0, 0, 0};
        }
    }

    f32x16 oacc[D / 32];
#pragma unroll
    for (int d = 0; d < D / 32; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[d][r] = 0.f;
    float m_run = -1e30f, l_run = 0.f, alpha_p = 1.f;

    // prologue: K(0), K(1), V(0); K(0) retired before the first barrier
    if (nt > 0) {
        dma(kp, st.kn, koff, 0, kimg(0));
        if (nt > 1) dma(kp, st.kn, koff, 1, kimg(1));
        dma(vp, st.vn, voff, 0, vimg(0));
    }
    if (nt > 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    auto seg_barrier = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    seg_barrier();
    if (lag) seg_barrier();

    i32x4 fr[16];  // K(t) fragments [tt*8 + kk] in S1-S2, V^T fragments in S3-S4
    f32x16 sc[2];  // S(t), S2 -> S4
    // HC: tile t exists (S1 K reads, S2 QK^T, S4 softmax(t));
    // HP: tile t-1 exists (S3 V reads, S4 PV(t-1) with pkp = P(t-1));
    // pkc receives P(t)
    auto iter = [&](auto HC_, auto HP_, int t, i32x4 (&pkc)[2][2], i32x4 (&pkp)[2][2]) {
        constexpr bool HC = decltype(HC_)::value, HP = decltype(HP_)::value;
        // opaque per iteration: the compiler recomputes the few VALU of
        // address math instead of keeping dozens of hoisted addresses live
        asm volatile("" : "+v"(A0), "+v"(B0), "+v"(koff[0]), "+v"(koff[1]), "+v"(voff[0]), "+v"(voff[1]),
                     "+v"(drow[0]), "+v"(drow[1]));
        // ---- S1: K(t) fragments; DMA K(t+2)
        if constexpr (HC) {
            const int ab = (int)(kimg(t) - smem) + A0;  // image base is 16 KiB aligned
#pragma unroll
            for (int kk = 0; kk < 8; ++kk) {
                const int a = ab ^ (kk << 5);
                fr[kk] = lds_read_b128(smem, a);
                fr[8 + kk] = lds_read_b128(smem, a + 8192);
            }
        }
        if (t + 2 < nt) dma(kp, st.kn, koff, t + 2, kimg(t + 2));
        seg_barrier();
        // ---- S2: S(t) = K Q^T (registers only)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (HC) {
#pragma unroll
            for (int tt = 0; tt < 2; ++tt) {
#pragma unroll
                for (int r = 0; r < 16; ++r) sc[tt][r] = 0.f;
#pragma unroll
                for (int kk = 0; kk < 8; ++kk) sc[tt] = mfma32x32x16<T>(fr[tt * 8 + kk], qf[kk], sc[tt]);
            }
            asm volatile("" : "+v"(sc[0]), "+v"(sc[1]));  // keep QK^T in S2
        }
        if (t + 2 < nt) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // K(t+1) landed
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        seg_barrier();
        // ---- S3: V(t-1)^T fragments; DMA V(t+1)
        if constexpr (HP) {
            const int bb = (int)(vimg(t - 1) - smem) + B0;
#pragma unroll
            for (int dblk = 0; dblk < 4; ++dblk) {
                const int alo = bb ^ (dblk << 6), ahi = (alo ^ 32) + 2048;
#pragma unroll
                for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2) {
                        const int ro = (tt * 32 + 16 * s2) * 256;
                        const i32x2 lo = lds_read_tr16(smem, alo + ro);
                        const i32x2 hi = lds_read_tr16(smem, ahi + ro);
                        fr[dblk * 4 + tt * 2 + s2] = i32x4{lo.x, lo.y, hi.x, hi.y};
                    }
            }
        }
        if (t + 1 < nt) dma(vp, st.vn, voff, t + 1, vimg(t + 1));
        seg_barrier();
        // ---- S4: O += P(t-1) V(t-1)  ||  softmax(t) -> P(t)
        if (HP && __ballot(alpha_p != 1.f)) {
#pragma unroll
            for (int d = 0; d < D / 32; ++d)
#pragma unroll
                for (int r = 0; r < 16; ++r) oacc[d][r] *= alpha_p;
        }
        if (HC && t >= t_mask) {
            // key t*KT + 4*h32 + kr(tt, r) is valid iff kr <= thr (one per-lane
            // threshold against constants: nothing per register to hoist)
            const int last = causal ? min(q0 + l32 + off_diag, Nk - 1) : Nk - 1;
            const int thr = last - t * KT - 4 * h32;
#pragma unroll
            for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    if (tt * 32 + (r & 3) + 8 * (r >> 2) > thr) sc[tt][r] = -INFINITY;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (HP) {
#pragma unroll
            for (int dblk = 0; dblk < 4; ++dblk)
#pragma unroll
                for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2)
                        oacc[dblk] = mfma32x32x16<T>(fr[dblk * 4 + tt * 2 + s2], pkp[tt][s2], oacc[dblk]);
        }
        if constexpr (HC) {
            float mx = max3(sc[0][0], sc[1][0], sc[0][1]);
            float my = max3(sc[1][1], sc[0][2], sc[1][2]);
#pragma unroll
            for (int r = 3; r < 15; r += 2) {
                mx = max3(mx, sc[0][r], sc[1][r]);
                my = max3(my, sc[0][r + 1], sc[1][r + 1]);
            }
            mx = max3(mx, my, max3(sc[0][15], sc[1][15], mx));
            mx = xor32_max(mx);
            float m_new = fmaxf(m_run, mx * c);
            m_new = mx * c > m_run + kDeferThr ? m_new : m_run;
            const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
            m_run = m_new;
#pragma unroll
            for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                for (int r = 0; r < 16; ++r) sc[tt][r] = __builtin_amdgcn_exp2f(fmaf(sc[tt][r], c, -m_new));
#pragma unroll
            for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    const int r0 = 8 * s2;
                    pkc[tt][s2] = i32x4{(int)pack2<T>(sc[tt][r0 + 0], sc[tt][r0 + 1]),
                                        (int)pack2<T>(sc[tt][r0 + 2], sc[tt][r0 + 3]),
                                        (int)pack2<T>(sc[tt][r0 + 4], sc[tt][r0 + 5]),
                                        (int)pack2<T>(sc[tt][r0 + 6], sc[tt][r0 + 7])};
                }
            float r0 = 0.f, r1 = 0.f;
#pragma unroll
            for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    r0 = add_pair<T>((uint32_t)pkc[tt][s2][0], r0);
                    r1 = add_pair<T>((uint32_t)pkc[tt][s2][1], r1);
                    r0 = add_pair<T>((uint32_t)pkc[tt][s2][2], r0);
                    r1 = add_pair<T>((uint32_t)pkc[tt][s2][3], r1);
                }
            l_run = fmaf(l_run, alpha, r0 + r1);
            alpha_p = alpha;  // O rescale before PV(t), in the next S4
            // pin: without it the softmax sinks past the barriers to its use in
            // the next tile's S4 (sched_barrier does not stop IR-level sinking)
            asm volatile("" : "+v"(pkc[0][0]), "+v"(pkc[0][1]), "+v"(pkc[1][0]), "+v"(pkc[1][1]),
                         "+v"(l_run), "+v"(alpha_p), "+v"(m_run));
        }
        if constexpr (SGB != 0 && HC && HP) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);  // MFMA
                __builtin_amdgcn_sched_group_barrier(0x002, 8, 1);  // VALU
            }
        }
        if (t + 2 < nt) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // V(t) landed
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        seg_barrier();
    };

    // tiles 0 .. nt-1 plus one drain step (t = nt: PV of the last tile);
    // even t packs P(t) into pa, odd t into pb
    const std::true_type Y{};
    const std::false_type N{};
    i32x4 pa[2][2], pb[2][2];
    if (nt > 0) {
        iter(Y, N, 0, pa, pb);
        int t = 1;
        for (; t + 1 < nt; t += 2) {
            iter(Y, Y, t, pb, pa);
            iter(Y, Y, t + 1, pa, pb);
        }
        if (t < nt) {
            iter(Y, Y, t, pb, pa);
            iter(N, Y, t + 1, pa, pb);
        } else {
            iter(N, Y, t, pb, pa);
        }
    }
    if (!lag) seg_barrier();  // equal barrier counts for both halves

    const float l = xor32_sum(l_run);
    const float inv = l > 0.f ? 1.f / l : 0.f;
    const int qr = q0 + l32;
    if (qr < Nq) {
        uint16_t* op = o + b * st.ob + hq * st.oh + (int64_t)qr * st.on;
#pragma unroll
        for (int dblk = 0; dblk < D / 32; ++dblk)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int d = dblk * 32 + 8 * i + 4 * h32;
                const i32x2 w = {(int)pack2<T>(oacc[dblk][4 * i] * inv, oacc[dblk][4 * i + 1] * inv),
                                 (int)pack2<T>(oacc[dblk][4 * i + 2] * inv, oacc[dblk][4 * i + 3] * inv)};
                *reinterpret_cast<i32x2*>(op + d) = w;
            }
    }
}

// Kernel variants behind the same ABI (A/B-able via pli_flash_attn_fwd_variant):
//   0: attn_fwd_mfma (XOR-swizzled LDS), 4 waves
//   1: attn_fwd_v2, 4 waves, lazy rescale    2: attn_fwd_v2, 8 waves, lazy rescale
//   3: attn_fwd_v2, 4 waves, eager rescale
//   4: attn_fwd_v3, 8 waves, staggered (waves 4-7 run a rotated body)
//   5: attn_fwd_v3 with Q in LDS
//   6: attn_fwd_v2b (block-wise softmax/PV)   7: attn_fwd_v2b + s_setprio
//   8: attn_fwd_v4 (intra-wave pipeline: QK^T(t+1) beside softmax(t))
//   9: attn_fwd_v4 + sched_group_barrier interleave  10: same, reads 3 ahead
//  11: attn_fwd_v5 (64 rows/wave, 1 wave/SIMD)  12: v5 + sched_group_barrier
//  13: v5 with LDS-DMA staging                  14: v5 + DMA + sched_group_barrier
//  15: attn_fwd_v6 (v2 structure on 16x16x32 MFMA, 8 waves)
//  16-20: v2 NW8 with OPT levers 1 (permlane max), 2 (younger-half prio),
//         4 (defer-max), 7 (all), 5 (permlane + defer)
//  21-23: v2 NW8 OPT 13 (permlane + defer + rounded sum), 12 (defer + rounded
//         sum), 9 (permlane + rounded sum)
//  24: variant 21 + epilogue stores widened to dwordx4 (OPT 16)
//  (16 waves x 32 rows was tried: needs <= 128 VGPRs and spills 296 B/lane)
//  25: variant 21 with 128-key tiles (one barrier per 128 keys; 148 KiB LDS)
//  27: attn_fwd_pp -- variant 21 split in two phases, waves 4-7 one phase
//      behind (ping-pong of the two waves on each SIMD)
//  28: variant 21 + iglp_opt(0)      29: variant 21 + batched fragment reads
//  30: attn_fwd_seg (four barrier-separated load / compute segments per tile,
//      waves 4-7 one segment behind, LDS-DMA into 3-deep rings; D=128, else 21)
//  31: attn_fwd_seg + sched_group_barrier interleave of the compute segments
//  40-42: attn_fwd_w4 (flash_w4.hip: 4 waves x 64 rows, one wave per SIMD,
//      two-slot software pipeline; LDS reads 3 / 2 / 4 MFMAs ahead); D=64 -> 21
//  43-45: attn_fwd_w4p (two phases of 32 MFMAs per tile, each K / V fragment
//      feeding both row blocks; fragments 2 / 3 / 4 ahead; ragged Nk -> w4)
//  46: attn_fwd_w4p fragments 3 ahead + s_memtime stamps (diagnostic; cycle
//      anatomy in DESIGN.md 3.1, tools/w4_stamps.py)
// default: v2 NW8 + permlane row max + defer-max (THR 8, log2) + rounded-P row sum
// (1057 TF vs 983 for plain v2 at B8 H32 S4096 D128; spike + variant parity green)
constexpr int kDefaultVariant = 21;

template <typename T, int D>
int launch_mfma(const void* q, const void* k, const void* v, void* o, int B, int H,
                int group, int Nq, int Nk, const AttnStrides& st, float scale,
                int causal, hipStream_t stream, int variant) {
    // v5 (11-14): 4 waves x 64 rows; 24: 16 waves x 32 rows
    const int nw = (variant == 2 || variant >= 4) ? 8 : 4;
    const int qblocks = cdiv(Nq, nw * QW);
    const int64_t nb = (int64_t)B * H * qblocks;
    PLI_REQUIRE(nb < (1ll << 31), "pli_flash_attn_fwd: grid too large");
    const float c = scale * 1.4426950408889634f;  // fold log2(e) into the scale
    const auto* qq = (const uint16_t*)q;
    const auto* kk = (const uint16_t*)k;
    const auto* vv = (const uint16_t*)v;
    auto* oo = (uint16_t*)o;
    const dim3 grid((unsigned)nb), block(nw * 64);
#define PLI_ATTN_LAUNCH(KERNEL) \
    hipLaunchKernelGGL(KERNEL, grid, block, 0, stream, qq, kk, vv, oo, H, group, Nq, Nk, st, c, \
                       causal, qblocks, (int)nb)
    switch (variant) {
        case 0: PLI_ATTN_LAUNCH((attn_fwd_mfma<T, D, 4>)); break;
        case 1: PLI_ATTN_LAUNCH((attn_fwd_v2<T, D, 4, true>)); break;
        case 2: PLI_ATTN_LAUNCH((attn_fwd_v2<T, D, 8, true>)); break;
        case 3: PLI_ATTN_LAUNCH((attn_fwd_v2<T, D, 4, false>)); break;
        case 4: PLI_ATTN_LAUNCH((attn_fwd_v3<T, D, false>)); break;
        case 5: PLI_ATTN_LAUNCH((attn_fwd_v3<T, D, true>)); break;
        case 6: PLI_ATTN_LAUNCH((attn_fwd_v2b<T, D, false>)); break;
        case 7: PLI_ATTN_LAUNCH((attn_fwd_v2b<T, D, true>)); break;
        case 8: PLI_ATTN_LAUNCH((attn_fwd_v4<T, D, 0>)); break;
        case 9: PLI_ATTN_LAUNCH((attn_fwd_v4<T, D, 1>)); break;
        case 10: PLI_ATTN_LAUNCH((attn_fwd_v4<T, D, 2>)); break;
#define PLI_ATTN_V5(SGB, DMA)                                                                    \
    hipLaunchKernelGGL((attn_fwd_v5<T, D, SGB, DMA>), grid, dim3(256), 0, stream, qq, kk, vv, oo, \
                       H, group, Nq, Nk, st, c, causal, qblocks, (int)nb)
        case 11: PLI_ATTN_V5(0, false); break;
        case 12: PLI_ATTN_V5(1, false); break;
        case 13: PLI_ATTN_V5(0, true); break;
        case 16: PLI_ATTN_LAUNCH((attn_fwd_v2<T, D, 8, true, 1>)); break;
        case 17: PLI_ATTN_LAUNCH((attn_fwd_v2<T, D, 8, true, 2>)); break;
        case 18: PLI_ATTN_LAUNCH((attn_fwd_v2<T, D, 8, true, 4>)); break;
        case 19: PLI_ATTN_LAUNCH((attn_fwd_v2<T, D, 8, true, 7>)); break;
        case 20: PLI_ATTN_LAUNCH((attn_fwd_v2<T, D, 8, true, 5>)); break;
        case 21: PLI_ATTN_LAUNCH((attn_fwd_v2<T, D, 8, true, 13>)); break;
        case 22: PLI_ATTN_LAUNCH((attn_fwd_v2<T, D, 8, true, 12>)); break;
        case 23: PLI_ATTN_LAUNCH((attn_fwd_v2<T, D, 8, true, 9>)); break;
        case 24: PLI_ATTN_LAUNCH((attn_fwd_v2<T, D, 8, true, 29>)); break;
        case 25: PLI_ATTN_LAUNCH((attn_fwd_v2<T, D, 8, true, 13, 128>)); break;
        case 27: PLI_ATTN_LAUNCH((attn_fwd_pp<T, D>)); break;
        case 28: PLI_ATTN_LAUNCH((attn_fwd_v2<T, D, 8, true, 13 | 32>)); break;
        case 29: PLI_ATTN_LAUNCH((attn_fwd_v2<T, D, 8, true, 13 | 128>)); break;
        case 30:
        case 31:
            if constexpr (D == 128) {
                if (variant == 30) PLI_ATTN_LAUNCH((attn_fwd_seg<T, 0>));
                else PLI_ATTN_LAUNCH((attn_fwd_seg<T, 1>));
            } else {
                PLI_ATTN_LAUNCH((attn_fwd_v2<T, D, 8, true, 13>));
            }
            break;
        case 40:
        case 41:
        case 42:
        case 43:
        case 44:
        case 45:
        case 46:
            if constexpr (D == 128) {
                const W4Strides w4{st.qb, st.qh, st.qn, st.kb, st.kh, st.kn,
                                   st.vb, st.vh, st.vn, st.ob, st.oh, st.on};
                return launch_attn_w4(q, k, v, o, B, H, group, Nq, Nk, w4, scale, causal,
                                      std::is_same<T, bf16_t>::value ? 1 : 0, stream, variant - 40);
            } else {
                PLI_ATTN_LAUNCH((attn_fwd_v2<T, D, 8, true, 13>));
            }
            break;
        case 15: hipLaunchKernelGGL((attn_fwd_v6<T, D>), grid, dim3(512), 0, stream, qq, kk, vv, oo,
                                    H, group, Nq, Nk, st, c, causal, qblocks, (int)nb); break;
        case 14: PLI_ATTN_V5(1, true); break;
#undef PLI_ATTN_V5
        default:
            set_error("pli_flash_attn_fwd: unknown variant %d", variant);
            return PLI_EINVAL;
    }
#undef PLI_ATTN_LAUNCH
    return launch_status("attn_fwd");
}

template <typename T>
int launch_generic(const void* q, const void* k, const void* v, void* o, int B, int H,
                   int group, int Nq, int Nk, int D, const AttnStrides& st, float scale,
                   int causal, hipStream_t stream) {
    const int qblocks = cdiv(Nq, GQ);
    const int64_t nb = (int64_t)B * H * qblocks;
    PLI_REQUIRE(nb < (1ll << 31), "pli_flash_attn_fwd: grid too large");
    const size_t lds = sizeof(float) * ((size_t)GQ * (D + 1) + (size_t)GK * (D + 1) +
                                        (size_t)GK * D + (size_t)GQ * (GK + 1));
    hipLaunchKernelGGL((attn_fwd_generic<T>), dim3((unsigned)nb), dim3(256), lds, stream,
                       (const T*)q, (const T*)k, (const T*)v, (T*)o, H, group, Nq, Nk, D, st,
                       scale, causal, qblocks);
    return launch_status("attn_fwd_generic");
}


}  // namespace
}  // namespace pli

// Not in pli.h: same contract as pli_flash_attn_fwd plus an explicit kernel
// variant (tuning / A-B runs); variant < 0 selects the default.
extern "C" int pli_flash_attn_fwd_variant(const void* q, const void* k, const void* v, void* o,
                                          int batch, int heads, int kv_heads, int n_q, int n_kv,
                                          int head_dim, const int64_t* strides, float scale,
                                          int causal, int dtype, void* stream, int variant) {
    using namespace pli;
    clear_error();
    PLI_REQUIRE(q && k && v && o && strides, "pli_flash_attn_fwd: null pointer");
    PLI_REQUIRE(batch >= 0 && heads > 0 && kv_heads > 0 && n_q >= 0 && n_kv >= 0 && head_dim > 0,
                "pli_flash_attn_fwd: bad shape B=%d H=%d Hkv=%d Nq=%d Nk=%d D=%d", batch, heads,
                kv_heads, n_q, n_kv, head_dim);
    PLI_REQUIRE(heads % kv_heads == 0, "pli_flash_attn_fwd: heads %d not a multiple of kv_heads %d",
                heads, kv_heads);
    PLI_REQUIRE(dtype == PLI_F32 || dtype == PLI_F16 || dtype == PLI_BF16,
                "pli_flash_attn_fwd: bad dtype %d", dtype);
    PLI_REQUIRE(std::isfinite(scale), "pli_flash_attn_fwd: non-finite scale");
    if (batch == 0 || n_q == 0) return PLI_OK;
    const AttnStrides st{strides[0], strides[1], strides[2], strides[3], strides[4], strides[5],
                         strides[6], strides[7], strides[8], strides[9], strides[10], strides[11]};
    const int group = heads / kv_heads;
    hipStream_t s = (hipStream_t)stream;
    // n_kv == 0 (softmax over no keys) goes to the generic kernel, which
    // defines the output as zeros.
    bool vec = (dtype == PLI_BF16 || dtype == PLI_F16) && (head_dim == 64 || head_dim == 128) &&
               aligned16(q) && aligned16(k) && aligned16(v) && aligned16(o) && n_kv > 0;
    for (int i = 0; i < 12; ++i) {
        const bool inner = (i % 3) == 2;
        vec = vec && (strides[i] % 8 == 0) && (!inner || strides[i] >= head_dim);
    }
    if (vec) {
        if (variant < 0) variant = kDefaultVariant;
        if (dtype == PLI_BF16)
            return head_dim == 128 ? launch_mfma<bf16_t, 128>(q, k, v, o, batch, heads, group, n_q, n_kv, st, scale, causal, s, variant)
                                   : launch_mfma<bf16_t, 64>(q, k, v, o, batch, heads, group, n_q, n_kv, st, scale, causal, s, variant);
        return head_dim == 128 ? launch_mfma<f16_t, 128>(q, k, v, o, batch, heads, group, n_q, n_kv, st, scale, causal, s, variant)
                               : launch_mfma<f16_t, 64>(q, k, v, o, batch, heads, group, n_q, n_kv, st, scale, causal, s, variant);
    }
    if (head_dim > GDMAX) {
        set_error("pli_flash_attn_fwd: head_dim %d > %d unsupported on the generic path", head_dim,
                  GDMAX);
        return PLI_EUNSUPPORTED;
    }
    switch (dtype) {
        case PLI_F32:
            return launch_generic<float>(q, k, v, o, batch, heads, group, n_q, n_kv, head_dim, st, scale, causal, s);
        case PLI_F16:
            return launch_generic<f16_t>(q, k, v, o, batch, heads, group, n_q, n_kv, head_dim, st, scale, causal, s);
        default:
            return launch_generic<bf16_t>(q, k, v, o, batch, heads, group, n_q, n_kv, head_dim, st, scale, causal, s);
    }
}

extern "C" int pli_flash_attn_fwd(const void* q, const void* k, const void* v, void* o,
                                  int batch, int heads, int kv_heads, int n_q, int n_kv,
                                  int head_dim, const int64_t* strides, float scale,
                                  int causal, int dtype, void* stream) {
    return pli_flash_attn_fwd_variant(q, k, v, o, batch, heads, kv_heads, n_q, n_kv, head_dim,
                                      strides, scale, causal, dtype, stream, -1);
}
