// Fused attention forward for gfx950 (MI355X).
//
// Replaces the Python tile loop of ch06/flash_attention.py:14-74 (about 12
// torch launches per (q-block, k-block) pair, every intermediate through HBM)
// with ONE launch: Q stays in registers, K/V tiles stream through LDS, the
// online softmax runs in registers with fp32 statistics.
//
// MFMA kernels (bf16 / fp16, head_dim 64 or 128), one wave = 32 query rows:
//   S^T = K Q^T      v_mfma_f32_32x32x16  A = K tile (ds_read_b128, LDS),
//                                         B = Q fragment (registers)
//   -> lane l owns query row l&31; its 64 tile scores sit in 32 registers
//      split over the two half-waves, so the row max is lane-local plus one
//      cross-half exchange (no LDS, no per-tile cross-lane sum).
//   O^T += V^T P^T   v_mfma_f32_32x32x16  A = V^T (ds_read_b64_tr_b16 from the
//                                         row-major V tile), B = P straight
//                                         from the S^T accumulator registers
//   -> O^T keeps the query row on the lane too, so the online-softmax rescale
//      and the final 1/l are lane-local.
// attn_fwd_v7 (flash_v7.hip, the default) and attn_fwd_v2 (below, the
// previous default, kept as the A/B baseline) share that mapping; v7 moves
// the score scaling into the MFMA and the row sum onto the matrix core.
// Blocks are remapped so each XCD works through a contiguous range of heads:
// a head's K/V is then read from HBM once and re-read from that XCD's L2 by
// all of the head's query blocks.
//
// Generic kernel (fp32, or any head_dim <= 128, or unaligned operands):
// LDS-tiled VALU kernel with the same online recurrence, fp32 accumulate.
#include <cmath>
#include <type_traits>

#include "flash_v7.h"
#include "pli_common.h"

namespace pli {
namespace {

struct AttnStrides {
    int64_t qb, qh, qn, kb, kh, kn, vb, vh, vn, ob, oh, on;
};

constexpr int KT = 64;  // keys per LDS tile
constexpr int QW = 32;  // query rows per wave

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

// Kernel variants behind the same ABI (pli_flash_attn_fwd_variant, tuning /
// A-B runs; every one is parity-tested, the default at the full bench size):
//  21: attn_fwd_v2, 8 waves, permlane row max + defer-max (THR 8, log2) +
//      rounded-P row sum by v_dot2c (the round-1 default, kept as baseline)
//  50: attn_fwd_v7 (flash_v7.hip): Q prescaled by scale*log2(e) (bf16-rounded)
//      with -m as the first QK^T MFMA's C operand, speculative exp2, row sum
//      on the matrix core; register-staged K/V, one tile ahead
//  51: attn_fwd_v7 with exact scaling (p = exp2(fma(s, c, -m)))
//  54: attn_fwd_v10: v7's body, K/V by LDS-DMA two tiles ahead into a 3-deep
//      ring of XOR-swizzled images (D = 128; other head dims take v7), prescaled
//  55: attn_fwd_v10 with exact scaling -- the DEFAULT (D = 128; D = 64 -> 51)
//  60: attn_fwd_v10 exact with 4-wave workgroups (128 rows), two per CU, a
//      2-slot ring one tile ahead -- the CAUSAL default (D = 128; D = 64 -> 51)
// The round-1 experiments (XOR-swizzled v1, staggered v3, pipelined v4/v5,
// 16x16x32 v6, ping-pong, segmented, one-wave-per-SIMD w4/w4p) and the
// round-2 ones that lost (in-wave pipelined v8, one-wave-per-SIMD v9, a
// two-barrier stagger with s_setprio, a half-tile lag on a 4-deep ring, the
// 4-wave one-wave-per-SIMD software-pipelined v11: 719-760 TF, static
// s_setprio 1 on waves 4-7: 1088 vs 1088 TF, the DMA pieces issued between
// the PV MFMAs: 1035 vs 1061 TF, two 64-key tiles per barrier on a 4-slot
// ring: 1054 vs 1054 TF, causal 850 vs 844) are
// not in the library; their measurements are in DESIGN.md 3.1.
//  70: attn_fwd_v12 (flash_v12.hip): 4 waves x 64 rows, one wave per SIMD,
//      O / Q / K fragments in literally named accumulator registers, a
//      hand-placed stream (one exp per MFMA gap), 5-slot LDS ring; bitwise
//      equal to 55 (bf16, D = 128, non-causal, Nk % 64 == 0; else 55)
//  71: attn_fwd_v12 persistent (one workgroup per CU walking its XCD's
//      blocks, the K/V stream and the next block's Q across block seams) --
//      the DEFAULT where 70 applies (1181 vs 1082 TF/s for 55)
//  73 / 74: attn_fwd_v12 causal (bottom-right, Nq <= Nk), one block per
//      workgroup heaviest first / persistent with the pair walk
//  72: variant 71 with the defer-max threshold at 0 (a rescale whenever a
//      tile raises a row's max): tests only, the threshold sweep of
//      cdna_hip_programming.md rule 26 (72 and 71 agree to rounding)
//  80: attn_fwd_v13 (flash_v13.hip): 4 waves x 64 rows, one wave per SIMD,
//      v_mfma_f32_16x16x32_bf16 (the shape the chip clocks higher under load),
//      one generated instruction stream (tools/gen_flash_v13.py), persistent;
//      defer-max on P itself (D = 128 / 64, non-causal, Nk % 64 == 0 and Nk
//      >= 128, or any Nk > 64 on the ragged bodies attn_fwd_v13r / v13hr --
//      round 5; else 71); fp16 inputs run the same program on the f16 MFMA
//      (attn_fwd_v13h / v13hc, since round 5; before: 71 -> 55 / 60)
//  81: variant 80 with one block per workgroup
//  82: variant 80 with mu = max * c (P = 1 at the max, so every row's l >= 1
//      and the rare path runs at every tile): tests only
//  83 / 84: attn_fwd_v13c causal (bottom-right, Nq <= Nk; any diagonal
//      offset -- virtual rows -- and ragged Nk -- attn_fwd_v13rc -- since
//      round 5): 83 persistent (the pair walk where it tiles the grid), 84 one
//      block per workgroup heaviest first; 85 = 83 with mu = max * c
// default since round 4: attn_fwd_v13 (80), 1388 vs 1242 TF/s for v12 (71)
// at B8 S4096 H32 D128 in the same process (profiles/r04/flash/ab.log); where
// v13 does not apply (D not 64 / 128, Nk <= 64) it routes to 71 / 74.
// Since round 6 the default is 88: attn_fwd_pp64 / pp64h (86) for head dim 64
// non-causal where its blocks fill the chip (two waves per SIMD in ping-pong;
// bitwise v13's D = 64 result, 1259 vs 1104 TF/s at B8 H32 S4096 D64 in the
// same process, profiles/r06/pp64/), v13 (80) for everything else
constexpr int kDefaultVariant = 88;
// v13's mu = row max * c + PLI_V13_MUOFF (log2 units): P <= 2^-MUOFF right
// after a max is taken and a tile takes the rescale path once some row's sum l
// reaches 1 (since round 5; a row max grown by about MUOFF - log2 Nk -- the P
// >= 2 bit test of round 4 fired at MUOFF + 1).  62 (since round 4; was 7, the THR 8 of v10 /
// v12): P stays a normal bf16 / fp32 down to 2^-126, so only scores 64+ log2
// units under the row max flush to 0 (weight < 2^-64), and the rescale path
// all but vanishes where the scaled scores spread wide -- B8 H32 S4096, N(0,1)
// inputs, TF/s 7 -> 62: scale 1.0 590 -> 1368 (causal 452 -> 1172), 0.25
// 1150 -> 1386 (891 -> 1167), 1/sqrt(128) 1377 -> 1390 (1166 -> 1167)
// (profiles/r04/scale/ab_muoff.jsonl)
#ifndef PLI_V13_MUOFF
#define PLI_V13_MUOFF 62.f
#endif
// Range of V this offset supports (bf16 v13; the v12 / v7 / v10 bf16 bodies'
// threshold 64 mirrors it): P is about 2^-62 at a row's max, so P * V stays a
// normal fp32 down to |V| ~ 2^-64 and products below flush gradually
// (subnormal fp32 keeps 2^-149 absolute); on the other side P <= 1 (v13's
// clamp) and O <= l max|V|, so any finite bf16 V is safe.  Exercised at |V|
// scaled by 2^-60 and 2^50 against f64 (tests/test_gpu_flash_v13.py
// test_v13_v_range, variants 80 / 83 / 71 / 55).
// fp16 (attn_fwd_v13h / v13hc, since round 5): fp16 P is normal down to 2^-14
// and zero below 2^-24, so the offset stays small -- P <= 2^-4 when a max is
// taken, the rescale path once a row max grows by 5 (some P >= 2, the bit-14
// test), scores 20+ log2 units under the running estimate flush to 0 (weight
// < 2^-20 of the row's largest: at most Nk * 2^-20 of the sum in total)
//
// Round 6: that flush is what limits fp16 at long context.  On an
// attention-sink row (one dominant key, the rest d log2 units under it) the
// weights just above 2^-(24 - offset) are quantised to a few subnormal steps
// and those below it dropped, so the worst-case error grows with Nk * 2^offset:
// a numpy model of the packing gives, offset 4 / 3 / 2 / 1 (torch's fp16 SDPA
// in brackets), Nk 4096 2.9e-3 / 1.5e-3 / 7.5e-4 / 1.9e-4 (9.3e-4), 8192
// 9.6e-3 / 2.5e-3 / 1.5e-3 / 3.4e-4 (1.3e-3), 16384 1.1e-2 / 5.9e-3 / 3.2e-3 /
// 6.9e-4 (1.5e-3), 32768 2.6e-2 / 1.1e-2 / 5.6e-3 / 1.5e-3 (1.5e-3), 65536
// 4.6e-2 / 2.7e-2 / 1.1e-2 / 3.1e-3 (2.7e-3).  So the offset
// falls by one per doubling of Nk past 4096 (floor 1): the worst case stays
// at ~3e-3, within ~2x of torch's, and the bench's Nk 4096 keeps offset 4.
// A smaller offset takes the rescale path more often (B8 S4096: 4 / 2 / 0 at
// 1308 / 1138 / 662 TF/s; B1 S32768: 1393 / 1324 / 1035).
#ifndef PLI_V13_MUOFF_F16
#define PLI_V13_MUOFF_F16 4.f
#endif
static float v13_muoff_f16(int Nk) {
    float m = PLI_V13_MUOFF_F16;
    for (int64_t n = 4096; n < Nk && m > 1.f; n *= 2) m -= 1.f;
    return m;
}
// causal: attn_fwd_v12 causal (74; one block per workgroup where the
// persistent pair walk does not tile the shape), 60 where v12 does not apply
// (fp16, D != 128, Nq > Nk, Nk % 64): B8 S4096 H32 D128 bf16 1002 (74, the
// first rotation walk) vs 945 (60) TF/s, B2 S8192 1098 vs 1013, B32 S2048 867
// vs 830 (profiles/r03/flash/ab_causal.log); the pair walk: 1049 at B8 S4096,
// 1154 at B2 S8192, 1223 at B1 H64 S16384 (ab_causal_pair.log)
// causal default since round 4: attn_fwd_v13c (83), 1210 vs 1058 TF/s for
// 74 (profiles/r04/flash/ab_causal.log); since round 5 83 takes any diagonal
// offset, ragged Nk, fp16 and D 64 too; Nk <= 64 -> 74 where v12 applies (bf16,
// D 128, Nk = 64), else 60 (so also other D and Nq > Nk)
constexpr int kDefaultCausalVariant = 83;

template <typename T, int D>
int launch_mfma(const void* q, const void* k, const void* v, void* o, int B, int H,
                int group, int Nq, int Nk, const AttnStrides& st, float scale,
                int causal, hipStream_t stream, int variant) {
    // the MFMA bodies' defer-max sets m from the raw score max times c =
    // scale*log2(e): only for c > 0 is that the row's largest scaled score
    // (c <= 0 would make exp2(s*c - m) >= 1 and overflow); zero or negative
    // scales never get here (the generic kernel's max is of the scaled scores).
    // Only the prescaled variants 50 / 54 multiply Q by c in the 16-bit input
    // type (so c > 1 could overflow fp16 Q): they alone need c <= 1; v13, v12
    // and the exact 51 / 55 / 60 apply c by fma in fp32 (any c > 0).
    const float c_log2 = scale * 1.4426950408889634f;
    const bool c_ok = c_log2 > 0.f && c_log2 <= 1.f;
    // the exact bodies (v12 70-74, v7 / v10 51 / 55 / 60) apply c by fma to
    // the fp32 scores: any c > 0; only the prescaled ones (50 / 54) need c <= 1
    const bool c_pos = c_log2 > 0.f;
    // 86: attn_fwd_pp64 / pp64h (causal: pp64c / pp64hc) where it applies
    // (head dim 64, bf16 / fp16, Nk % 64 == 0; causal with Nq and Nk - Nq
    // multiples of 64; tools/v14/pp64.py), else the default v13 form; 87: the
    // same with the rescale path at every tile (muoff 0 / -1, tests)
    // 88 (the default since round 6): 86 where its 512-row blocks fill the
    // chip (B H ceil(Nq / 512) >= the CU count), else 80 -- below that v13's
    // 256-row blocks spread the same work over twice as many CUs (B2 H8 S512:
    // 61 vs 85 TF/s on pp64, profiles/r06/pp64/)
    // (causal stays on v13c: pp64c -- the causal pp64 forms, one block per
    // workgroup heaviest first -- measured 725 vs 946 TF/s bf16, 802 vs 941
    // fp16 at B8 H32 S4096 D64, profiles/r06/pp64/ab9_causal_*.jsonl)
    if (variant == 88) {
        const bool fill = (int64_t)B * H * cdiv(Nq, 512) >= cu_count(stream);
        variant = causal ? 83 : fill ? 86 : 80;
    }
    if (variant == 86 || variant == 87) {
        const bool bf = std::is_same<T, bf16_t>::value;
        const V7Strides s7{st.qb, st.qh, st.qn, st.kb, st.kh, st.kn, st.vb, st.vh, st.vn, st.ob, st.oh, st.on};
        if (attn_pp64_ok(D, !bf, causal != 0, Nq, Nk) && attn_v13_ok(D, bf ? 1 : 0, causal, Nq, Nk, s7) &&
            c_log2 > 0.f && H < (1 << 16))
            return launch_attn_v13(q, k, v, o, B, H, group, Nq, Nk, s7, scale, stream, true,
                                   variant == 87 ? (bf ? 0.f : -1.f) : bf ? PLI_V13_MUOFF : v13_muoff_f16(Nk),
                                   nullptr, causal != 0, !bf, D, true);
        variant = causal ? (variant == 87 ? 85 : 83) : variant == 87 ? 82 : 80;
    }
    if (variant >= 80 && variant <= 85) {
        const bool bf = std::is_same<T, bf16_t>::value;
        const bool cv = variant >= 83;  // the causal forms
        const V7Strides s7{st.qb, st.qh, st.qn, st.kb, st.kh, st.kn, st.vb, st.vh, st.vn, st.ob, st.oh, st.on};
        // v13 scales in fp32 (s * c - mu by v_fma): any c > 0 (scale = 1 etc.)
        // the rare-path sweep (82 / 85): bf16's l check trips at every tile with
        // mu = max * c (P = 1 at the max), fp16's P-bit check with mu = max * c - 1
        const float sweep = bf ? 0.f : -1.f;
        if (cv == (causal != 0) && attn_v13_ok(D, bf ? 1 : 0, causal, Nq, Nk, s7) && c_log2 > 0.f && H < (1 << 16))
            return launch_attn_v13(q, k, v, o, B, H, group, Nq, Nk, s7, scale, stream, variant != 81 && variant != 84,
                                   (variant == 82 || variant == 85) ? sweep : bf ? PLI_V13_MUOFF : v13_muoff_f16(Nk),
                                   nullptr, causal != 0, !bf, D);
        variant = causal ? 74 : 71;
    }
    if (variant == 70 || variant == 71 || variant == 72) {
        const bool bf = std::is_same<T, bf16_t>::value;
        if (attn_v12_ok(D, bf ? 1 : 0, causal, Nk) && c_pos) {
            const V7Strides s7{st.qb, st.qh, st.qn, st.kb, st.kh, st.kn,
                               st.vb, st.vh, st.vn, st.ob, st.oh, st.on};
            return launch_attn_v12(q, k, v, o, B, H, group, Nq, Nk, s7, scale, stream, variant != 70,
                                   variant == 72 ? 0.f : 64.f);
        }
        variant = causal ? 60 : 55;
    }
    if (variant == 73 || variant == 74) {
        const bool bf = std::is_same<T, bf16_t>::value;
        if (causal && attn_v12_ok(D, bf ? 1 : 0, 0, Nk) && Nq <= Nk && c_pos) {
            const V7Strides s7{st.qb, st.qh, st.qn, st.kb, st.kh, st.kn,
                               st.vb, st.vh, st.vn, st.ob, st.oh, st.on};
            return launch_attn_v12(q, k, v, o, B, H, group, Nq, Nk, s7, scale, stream, variant == 74, 64.f, true);
        }
        variant = causal ? 60 : 55;
    }
    if (variant == 50 || variant == 51 || variant == 54 || variant == 55 || variant == 60) {
        if (variant == 50 || variant == 54 ? c_ok : c_pos) {
            const V7Strides s7{st.qb, st.qh, st.qn, st.kb, st.kh, st.kn,
                               st.vb, st.vh, st.vn, st.ob, st.oh, st.on};
            return launch_attn_v7(q, k, v, o, B, H, group, Nq, Nk, D, s7, scale, causal,
                                  std::is_same<T, bf16_t>::value ? 1 : 0, stream, variant - 50);
        }
        variant = 21;
    }
    constexpr int nw = 8;
    const int qblocks = cdiv(Nq, nw * QW);
    const int64_t nb = (int64_t)B * H * qblocks;
    PLI_REQUIRE(nb < (1ll << 31), "pli_flash_attn_fwd: grid too large");
    const float c = scale * 1.4426950408889634f;  // fold log2(e) into the scale
    const auto* qq = (const uint16_t*)q;
    const auto* kk = (const uint16_t*)k;
    const auto* vv = (const uint16_t*)v;
    auto* oo = (uint16_t*)o;
    const dim3 grid((unsigned)nb), block(nw * 64);
    switch (variant) {
        case 21:
            hipLaunchKernelGGL((attn_fwd_v2<T, D, 8, true, 13>), grid, block, 0, stream, qq, kk, vv, oo, H,
                               group, Nq, Nk, st, c, causal, qblocks, (int)nb);
            break;
        default:
            set_error("pli_flash_attn_fwd: unknown variant %d", variant);
            return PLI_EINVAL;
    }
    return launch_status("attn_fwd_v2");
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

// Same contract as pli_flash_attn_fwd plus an explicit kernel variant
// (include/pli.h tuning section); variant < 0 selects the default.
extern "C" int pli_flash_attn_fwd_variant(const void* q, const void* k, const void* v, void* o,
                                          int batch, int heads, int kv_heads, int n_q, int n_kv,
                                          int head_dim, const int64_t* strides, float scale,
                                          int causal, int dtype, void* stream, int variant) {
    using namespace pli;
    clear_error();
    PLI_REQUIRE(batch >= 0 && heads > 0 && kv_heads > 0 && n_q >= 0 && n_kv >= 0 && head_dim > 0,
                "pli_flash_attn_fwd: bad shape B=%d H=%d Hkv=%d Nq=%d Nk=%d D=%d", batch, heads,
                kv_heads, n_q, n_kv, head_dim);
    PLI_REQUIRE(heads % kv_heads == 0, "pli_flash_attn_fwd: heads %d not a multiple of kv_heads %d",
                heads, kv_heads);
    PLI_REQUIRE(dtype == PLI_F32 || dtype == PLI_F16 || dtype == PLI_BF16,
                "pli_flash_attn_fwd: bad dtype %d", dtype);
    PLI_REQUIRE(std::isfinite(scale), "pli_flash_attn_fwd: non-finite scale");
    // empty operands may be NULL (pli.h): no output rows -> nothing to do; no
    // keys -> O = 0 (the generic kernel reads no K / V)
    if (batch == 0 || n_q == 0) return PLI_OK;
    PLI_REQUIRE(q && o && strides && (n_kv == 0 || (k && v)), "pli_flash_attn_fwd: null pointer");
    const AttnStrides st{strides[0], strides[1], strides[2], strides[3], strides[4], strides[5],
                         strides[6], strides[7], strides[8], strides[9], strides[10], strides[11]};
    const int group = heads / kv_heads;
    hipStream_t s = (hipStream_t)stream;
    // n_kv == 0 (softmax over no keys) goes to the generic kernel, which
    // defines the output as zeros.
    bool vec = (dtype == PLI_BF16 || dtype == PLI_F16) && (head_dim == 64 || head_dim == 128) &&
               aligned16(q) && aligned16(k) && aligned16(v) && aligned16(o) && n_kv > 0 &&
               scale > 0.f;  // the MFMA kernels' running max assumes a positive scale (launch_mfma)
    for (int i = 0; i < 12; ++i) {
        const bool inner = (i % 3) == 2;
        vec = vec && (strides[i] % 8 == 0) && (!inner || strides[i] >= head_dim);
    }
    if (vec) {
        if (variant < 0) variant = causal ? kDefaultCausalVariant : kDefaultVariant;
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
