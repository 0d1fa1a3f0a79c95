// attn_fwd_v7: flash-attention forward with a lean softmax (gfx950, D 64/128).
//
// Same tile structure as attn_fwd_v2 (flash_attn.hip; reference
// ch06/flash_attention.py:14-74): 8 waves x 32 query rows, 64-key K/V tiles
// register-staged into padded LDS images, S^T = K Q^T and O^T += V^T P^T on
// v_mfma_f32_32x32x16 with the query row on the lane.  What changes is the
// VALU work per score, which is what held v2 at ~40 % of the MFMA roof (it is
// issue-bound: ~5.8 VALU per MFMA):
//
//  * Q is prescaled once by c = scale * log2(e) (rounded to the 16-bit input
//    type), and the first MFMA of every S chain takes its C operand from a
//    register block holding -m (the running row max, log2 units).  The MFMA
//    then leaves S' = S*c - m and p = exp2(S') needs no fma: 1 VALU per score
//    instead of 2.
//  * The exp is speculative: it does not wait for the row max.  The max (16
//    v_max3 + one permlane) only decides whether the tile raised it by more
//    than 8 (defer-max); in that rare case the wave recomputes the tile's S
//    from LDS with the new -m block, redoes the exps and rescales O and l.
//  * The row sum l is taken by the matrix core: one v_mfma_f32_16x16x32 per
//    16-key step with a 0/1 selector as A and the packed bf16 P fragment as B
//    sums exactly the rounded P the PV product uses (the v2 default used 16
//    v_dot2c per tile for that), for 1/16 more matrix time and no VALU.
//
// Per 64-key tile and lane that leaves 32 v_exp + 16 v_cvt_pk + 16 v_max3
// (was + 32 v_fma + 16 v_dot2c).
#include <cmath>
#include <type_traits>

#include "flash_v7.h"
#include "pli_common.h"

namespace pli {
namespace {

typedef __attribute__((ext_vector_type(2))) float f32x2;

constexpr int V7_KT = 64;       // keys per tile
constexpr int V7_QW = 32;       // query rows per wave
constexpr int V7_NW = 8;        // waves per workgroup
// defer-max threshold (log2 units): P <= 2^THR.  bf16 64 since round 4 (8
// before; a normal bf16 / fp32 value, the rescale path all but vanishes where
// the scaled scores spread wide -- as v12 / v13); fp16 8 (its P stops at 2^15)
template <typename T> constexpr float v7_thr() { return std::is_same<T, bf16_t>::value ? 64.f : 8.f; }

template <int D> struct V7Layout {
    static constexpr int KS = 2 * D + 16;  // K row stride (bytes): b128 reads conflict-free
    static constexpr int VS = 2 * D + 64;  // V row stride (bytes): tr_b16 reads conflict-free
    static constexpr int KSZ = V7_KT * KS, VSZ = V7_KT * VS, BUF = KSZ + VSZ;
};

template <typename T> struct V7Ones;
template <> struct V7Ones<bf16_t> { static constexpr int pair = 0x3F803F80; };
template <> struct V7Ones<f16_t> { static constexpr int pair = 0x3C003C00; };

// both 16-bit halves of a word, scaled by c and re-rounded to T
template <typename T> __device__ __forceinline__ int v7_scale_pair(int w, float c);
template <> __device__ __forceinline__ int v7_scale_pair<bf16_t>(int w, float c) {
    const float lo = __uint_as_float((uint32_t)w << 16), hi = __uint_as_float((uint32_t)w & 0xffff0000u);
    return (int)pack2<bf16_t>(lo * c, hi * c);
}
template <> __device__ __forceinline__ int v7_scale_pair<f16_t>(int w, float c) {
    const float lo = (float)__builtin_bit_cast(_Float16, (uint16_t)((uint32_t)w & 0xffffu));
    const float hi = (float)__builtin_bit_cast(_Float16, (uint16_t)((uint32_t)w >> 16));
    return (int)pack2<f16_t>(lo * c, hi * c);
}

__device__ __forceinline__ float v7_xor32_max(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float v7_xor32_sum(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// PRE = 1: Q prescaled by c (rounded to the 16-bit input type) and -m as the
//          C operand of the first QK^T MFMA: p = exp2(acc), no fma per score;
//          the Q rounding costs score precision (2^-9 relative in bf16).
// PRE = 0: exact scaling, S accumulates from 0 and p = exp2(fma(s, c, -m)).
#ifdef PLI_FLASH_STAMPS
// diagnostic build only (tools/build_diag.sh -> tools/libpli_diag.so, never
// the product library): per-segment s_memtime sums over all waves
__device__ unsigned long long g_v7_stamps[16];
#endif

template <typename T, int D, int PRE, bool STAMP = false>
__global__ __launch_bounds__(512, 2) void attn_fwd_v7(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
    const uint16_t* __restrict__ v, uint16_t* __restrict__ o, int H, int group,
    int Nq, int Nk, V7Strides st, float c, int causal, int qblocks, int nblocks) {
    using L = V7Layout<D>;
    constexpr int NT = V7_NW * 64;
    constexpr int CPR = D / 8;     // 16-byte chunks per row
    constexpr int RPI = NT / CPR;  // rows covered by one staging step
    constexpr int CPT = V7_KT / RPI;
    static_assert(NT % CPR == 0 && V7_KT % RPI == 0, "staging must tile evenly");
    __shared__ __attribute__((aligned(16))) char smem[2 * L::BUF];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h32 = lane >> 5, l32 = lane & 31;
    // STAMP: segment cycle sums (see the .s: each stamp is fenced by
    // sched_barriers, so the diagnostic build's schedule differs -- read shares)
    unsigned long long st_sum[8] = {0, 0, 0, 0, 0, 0, 0, 0}, st_last = 0;
    auto stamp = [&](int seg) __attribute__((always_inline)) {
        if constexpr (STAMP) {
            unsigned long long now;
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(now)::"memory");
            __builtin_amdgcn_sched_barrier(0);
            if (seg >= 0) st_sum[seg] += now - st_last;
            st_last = now;
        }
    };
    const int lb = xcd_remap(blockIdx.x, nblocks);
    const int bh = lb / qblocks;
    // causal: heaviest query blocks of a head first, so the grid drains on light ones
    const int qblk = causal ? qblocks - 1 - lb % qblocks : lb % qblocks;
    const int b = bh / H, hq = bh % H, hk = hq / group;
    const int qbase = qblk * (V7_NW * V7_QW);
    const int q0 = qbase + wave * V7_QW;
    const int off_diag = Nk - Nq;  // causal (bottom-right): row i sees keys <= i + off_diag

    const uint16_t* qp = q + b * st.qb + hq * st.qh;
    const uint16_t* kp = k + b * st.kb + hk * st.kh;
    const uint16_t* vp = v + b * st.vb + hk * st.vh;

    // Q^T fragments (B operand): query row q0 + l32, d = 16kk + 8h32 .. +7
    i32x4 qf[D / 16];
    {
        const int qr = q0 + l32;
        // rows past Nq read row 0 (finite scores, never stored): no select,
        // which hipcc otherwise re-materialises inside the K loop (32 v_cndmask
        // per tile)
        const uint16_t* src = qp + (int64_t)(qr < Nq ? qr : 0) * st.qn + 8 * h32;
#pragma unroll
        for (int kk = 0; kk < D / 16; ++kk) qf[kk] = *reinterpret_cast<const i32x4*>(src + 16 * kk);
        if constexpr (PRE != 0) {
#pragma unroll
            for (int kk = 0; kk < D / 16; ++kk)
#pragma unroll
                for (int j = 0; j < 4; ++j) qf[kk][j] = v7_scale_pair<T>(qf[kk][j], c);
        }
    }

    int kv_end = Nk;
    if (causal) kv_end = min(Nk, qbase + V7_NW * V7_QW + off_diag);
    const int nt = kv_end > 0 ? cdiv(kv_end, V7_KT) : 0;
    const int t_full = Nk / V7_KT;  // tiles [0, t_full) need no row clamp
    int t_mask = t_full;            // first tile this wave must mask
    if (causal) t_mask = min(t_mask, max(0, (q0 + off_diag + 1) / V7_KT));

    // staging: thread owns chunk `sch` of rows srow + i*RPI
    const int srow = tid / CPR, sch = tid % CPR;
    const uint16_t* kg = kp + (int64_t)srow * st.kn + sch * 8;
    const uint16_t* vg = vp + (int64_t)srow * st.vn + sch * 8;
    const int kw = srow * L::KS + sch * 16, vw = L::KSZ + srow * L::VS + sch * 16;
    i32x4 kst[CPT], vst[CPT];
    auto load_tile = [&](int t) __attribute__((always_inline)) {
        if (t < t_full) {
#pragma unroll
            for (int i = 0; i < CPT; ++i) {
                const int64_t r = (int64_t)t * V7_KT + i * RPI;
                kst[i] = *reinterpret_cast<const i32x4*>(kg + r * st.kn);
                vst[i] = *reinterpret_cast<const i32x4*>(vg + r * st.vn);
            }
        } else {
#pragma unroll
            for (int i = 0; i < CPT; ++i) {
                const int key = t * V7_KT + i * RPI + srow;
                const int64_t r = min(key, Nk - 1) - srow;
                const i32x4 kx = *reinterpret_cast<const i32x4*>(kg + r * st.kn);
                const i32x4 vx = *reinterpret_cast<const i32x4*>(vg + r * st.vn);
                kst[i] = key < Nk ? kx : i32x4{0, 0, 0, 0};
                vst[i] = key < Nk ? vx : i32x4{0, 0, 0, 0};
            }
        }
    };
    auto store_tile = [&](int buf) __attribute__((always_inline)) {
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

    // Row-sum selector (A of v_mfma_f32_16x16x32): lane l supplies row l&15,
    // k' = 8(l>>4)..+7.  Read as that MFMA's B, the P^T fragment of a 32x32x16
    // k-step puts query n's keys in k' groups 0 and 2 and query n+16's in 1 and
    // 3 (n = l&15), so row 0 = ones on groups {0,2}, row 4 = ones on {1,3}
    // leaves query l's sum in register 0 of lane l (l < 32) and zeros in lanes
    // 32..63.
    const bool sel_on = (i16 == 0 && (g & 1) == 0) || (i16 == 4 && (g & 1) == 1);
    const int one = sel_on ? V7Ones<T>::pair : 0;
    const i32x4 sel = {one, one, one, one};

    f32x16 oacc[D / 32];
#pragma unroll
    for (int d = 0; d < D / 32; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[d][r] = 0.f;
    f32x16 negm;  // PRE: -m_run in every register, C of the first QK^T MFMA
#pragma unroll
    for (int r = 0; r < 16; ++r) negm[r] = 0.f;
    // running max, log2 units (PRE: the offset already inside S')
    float m_run = PRE != 0 ? 0.f : -1e30f;
    f32x4 lsum = {0.f, 0.f, 0.f, 0.f};

    // X(t): S = K(t) Q^T, mask, row max, (speculative) exps, pack -> pb
    i32x4 pb[2][2];
    auto X = [&](int t, auto first_tag) __attribute__((always_inline)) {
        constexpr bool FIRST = decltype(first_tag)::value;
        const char* kb = smem + (t & 1) * L::BUF + kr;

        // s[tt][r] = S(key 32tt + 8(r>>2) + 4h32 + (r&3), query l32)  (PRE: S*c - m)
        f32x16 s[2];
        auto qk = [&]() __attribute__((always_inline)) {
#pragma unroll
            for (int tt = 0; tt < 2; ++tt) {
                if constexpr (PRE != 0) {
                    s[tt] = mfma32x32x16<T>(lds_read_b128(kb, tt * 32 * L::KS), qf[0], negm);
                } else {
                    f32x16 z;
#pragma unroll
                    for (int r = 0; r < 16; ++r) z[r] = 0.f;
                    s[tt] = mfma32x32x16<T>(lds_read_b128(kb, tt * 32 * L::KS), qf[0], z);
                }
#pragma unroll
                for (int kk = 1; kk < D / 16; ++kk)
                    s[tt] = mfma32x32x16<T>(lds_read_b128(kb, tt * 32 * L::KS + kk * 32), qf[kk], s[tt]);
            }
            if (t >= t_mask) {
                const int lim = causal ? q0 + l32 + off_diag : Nk;
#pragma unroll
                for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int key = t * V7_KT + tt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h32;
                        if (key >= Nk || key > lim) s[tt][r] = -INFINITY;
                    }
            }
        };
        auto expo = [&]() __attribute__((always_inline)) {
#pragma unroll
            for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    s[tt][r] = __builtin_amdgcn_exp2f(PRE != 0 ? s[tt][r] : fmaf(s[tt][r], c, -m_run));
        };
        stamp(0);
        qk();

        // row max: two v_max3 chains (-fno-honor-nans: no canonicalising
        // v_max_f32 in front of the MFMA results) + one cross-half swap
        float mx = fmaxf(s[0][0], s[1][0]), my = fmaxf(s[0][1], s[1][1]);
#pragma unroll
        for (int r = 2; r < 16; r += 2) {
            mx = fmaxf(fmaxf(mx, s[0][r]), s[1][r]);
            my = fmaxf(fmaxf(my, s[0][r + 1]), s[1][r + 1]);
        }
        mx = v7_xor32_max(fmaxf(mx, my));
        if constexpr (STAMP) asm volatile("" ::"v"(mx));
        stamp(1);

        if constexpr (FIRST) {
            // the first tile sets the running max (O and l are still zero)
            if constexpr (PRE != 0) {
                const float delta = mx == -INFINITY ? 0.f : mx;
                m_run = delta;
#pragma unroll
                for (int r = 0; r < 16; ++r) negm[r] = -m_run;
#pragma unroll
                for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) s[tt][r] -= delta;
            } else {
                m_run = mx == -INFINITY ? -1e30f : mx * c;
            }
            expo();
        } else {
            // speculative exps against the running max, kept ahead of the
            // branch (hipcc would otherwise sink them into both arms, behind
            // the max chain)
            expo();
            asm volatile("" : "+v"(s[0]), "+v"(s[1]));
            stamp(2);
            const bool up = PRE != 0 ? mx > v7_thr<T>() : mx * c > m_run + v7_thr<T>();
            if (__ballot(up)) {
                // rare: some row's max rose by more than the threshold.  K(t)
                // is still in LDS: recompute S and redo the exps.  (O holds
                // every earlier tile's PV: its rescale is exact here.)
                float alpha;
                if constexpr (PRE != 0) {
                    const float delta = up ? mx : 0.f;
                    m_run += delta;
#pragma unroll
                    for (int r = 0; r < 16; ++r) negm[r] = -m_run;
                    alpha = __builtin_amdgcn_exp2f(-delta);
                } else {
                    const float m_new = up ? mx * c : m_run;
                    alpha = __builtin_amdgcn_exp2f(m_run - m_new);
                    m_run = m_new;
                }
                qk();
                expo();
#pragma unroll
                for (int d = 0; d < D / 32; ++d)
#pragma unroll
                    for (int r = 0; r < 16; ++r) oacc[d][r] *= alpha;
                lsum[0] *= alpha;
            }
        }

        // P^T fragments: registers 8s2..8s2+7 of s[tt] are k-step s2
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
        if constexpr (STAMP) asm volatile("" ::"v"(pb[0][0]), "v"(pb[0][1]), "v"(pb[1][0]), "v"(pb[1][1]));
        stamp(3);
    };
    // Y(t): l += rowsum(P) (selector MFMA), O^T += V(t)^T P^T
    auto Y = [&](int t) __attribute__((always_inline)) {
        const char* vb = smem + (t & 1) * L::BUF + vr;
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) lsum = mfma16x16x32<T>(sel, pb[tt][s2], lsum);
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
        stamp(4);
    };

    // one barrier per tile; tile t+1 register-staged under tile t
    if (nt > 0) {
        load_tile(0);
        store_tile(0);
    }
    __syncthreads();
    auto tile = [&](int t, auto first_tag) __attribute__((always_inline)) {
        stamp(-1);
        if (t + 1 < nt) load_tile(t + 1);
        X(t, first_tag);
        Y(t);
        if (t + 1 < nt) store_tile((t + 1) & 1);
        stamp(5);
        __syncthreads();
        stamp(6);
    };
    if (nt > 0) tile(0, std::true_type{});
    for (int t = 1; t < nt; ++t) tile(t, std::false_type{});

#ifdef PLI_FLASH_STAMPS
    if constexpr (STAMP) {
        if (lane == 0) {
#pragma unroll
            for (int i = 0; i < 7; ++i) atomicAdd(&g_v7_stamps[i], st_sum[i]);
            atomicAdd(&g_v7_stamps[8], (unsigned long long)nt);
            atomicAdd(&g_v7_stamps[9], 1ull);
        }
    }
#endif
    // ---- epilogue: O = O^T / l, query row l32
    const float l = v7_xor32_sum(lsum[0]);
    const float inv = l > 0.f ? 1.f / l : 0.f;
    const int qr = q0 + l32;
    if (qr < Nq) {
        uint16_t* op = o + b * st.ob + hq * st.oh + (int64_t)qr * st.on;
        // group k = 4*dblk + i holds columns 8k+4*h32 .. +3 of row qr; after
        // swapping (k, k+1): lower lanes hold cols 8k..8k+7, upper 8k+8..8k+15
#pragma unroll
        for (int dblk = 0; dblk < D / 32; ++dblk)
#pragma unroll
            for (int i = 0; i < 4; i += 2) {
                const f32x16& a = oacc[dblk];
                const uint32_t ax = pack2<T>(a[4 * i] * inv, a[4 * i + 1] * inv);
                const uint32_t ay = pack2<T>(a[4 * i + 2] * inv, a[4 * i + 3] * inv);
                const uint32_t bx = pack2<T>(a[4 * i + 4] * inv, a[4 * i + 5] * inv);
                const uint32_t by = pack2<T>(a[4 * i + 6] * inv, a[4 * i + 7] * inv);
                const auto rx = __builtin_amdgcn_permlane32_swap(ax, bx, false, false);
                const auto ry = __builtin_amdgcn_permlane32_swap(ay, by, false, false);
                const int d = dblk * 32 + 8 * i + 8 * h32;
                *reinterpret_cast<i32x4*>(op + d) = i32x4{(int)rx[0], (int)ry[0], (int)rx[1], (int)ry[1]};
            }
    }
}

// --------------------------------------------------------------------------
// attn_fwd_v10 (D = 128): v7's body with the K/V staging moved off the
// registers and two tiles ahead.  Stamps of v7 (tools/flash_stamps.py) put
// ~19 % of a tile in the vmcnt wait before the LDS writes (the next tile's
// global loads, issued one tile earlier, had not landed) and ~15 % at the
// barrier.  Here every wave LDS-DMAs (global_load_lds_dwordx4, 1 KiB
// lane-linear pieces: 2 of K + 2 of V per wave per tile) tile t+2 into a
// 3-deep ring at the top of tile t, and only a counted vmcnt (tile t+1's
// pieces landed, t+2's still in flight) precedes the barrier.  The images are
// unpadded 256-byte rows with the 16-byte chunks XOR-swizzled by
// f(row) = (row&3)<<2 | (row>>2)&3 on the DMA source address (conflict-free
// for the b128 K-fragment read and the tr_b16 V^T read, cdna guide T10
// layout (b)); the fragment address of k-step kk is A0 ^ (kk<<5), of V block
// dblk B0 ^ (dblk<<6).  Rows past Nk re-read row Nk-1 (masked / weight 0).
// NW4: 4-wave workgroups (128 query rows), two per CU: the two waves of a
// SIMD then belong to different workgroups with their own barriers, so they
// drift apart instead of reaching the softmax together; 2-slot ring, K/V one
// tile ahead.
template <typename T, int PRE, bool STAMP = false, bool NW4 = false>
__global__ __launch_bounds__(NW4 ? 256 : 512, 2) void attn_fwd_v10(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
    const uint16_t* __restrict__ v, uint16_t* __restrict__ o, int H, int group,
    int Nq, int Nk, V7Strides st, float c, int causal, int qblocks, int nblocks) {
    constexpr int D = 128;
    constexpr int IMG = V7_KT * 256;  // one [64][128] 16-bit image
    constexpr int BUFB = 2 * IMG;     // K image + V image
    constexpr int NBUF = NW4 ? 2 : 3;
    constexpr int NW = NW4 ? 4 : V7_NW;   // waves per workgroup
    constexpr int PPW = 16 / NW;          // K (and V) 1-KiB pieces per wave per tile
    __shared__ __attribute__((aligned(1024))) char smem[NBUF * BUFB];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int h32 = lane >> 5, l32 = lane & 31;
    unsigned long long st_sum[8] = {0, 0, 0, 0, 0, 0, 0, 0}, st_last = 0;
    auto stamp = [&](int seg) __attribute__((always_inline)) {
        if constexpr (STAMP) {
            unsigned long long now;
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(now)::"memory");
            __builtin_amdgcn_sched_barrier(0);
            if (seg >= 0) st_sum[seg] += now - st_last;
            st_last = now;
        }
    };
    const int lb = xcd_remap(blockIdx.x, nblocks);
    const int bh = lb / qblocks;
    const int qblk = causal ? qblocks - 1 - lb % qblocks : lb % qblocks;
    const int b = bh / H, hq = bh % H, hk = hq / group;
    const int qbase = qblk * (NW * V7_QW);
    const int q0 = qbase + wave * V7_QW;
    const int off_diag = Nk - Nq;

    const uint16_t* qp = q + b * st.qb + hq * st.qh;
    const uint16_t* kp = k + b * st.kb + hk * st.kh;
    const uint16_t* vp = v + b * st.vb + hk * st.vh;

    int kv_end = Nk;
    if (causal) kv_end = min(Nk, qbase + NW * V7_QW + off_diag);
    const int nt = kv_end > 0 ? cdiv(kv_end, V7_KT) : 0;
    const int t_full = Nk / V7_KT;
    int t_mask = t_full;
    if (causal) t_mask = min(t_mask, max(0, (q0 + off_diag + 1) / V7_KT));
    // causal: tiles past this wave's last visible key are all -inf for its
    // rows; the wave skips their compute but still issues its DMA pieces and
    // meets the barriers (workgroup-uniform pipeline)
    int t_last = nt;
    if (causal) t_last = (q0 + V7_QW - 1 + off_diag) < 0 ? -1 : (q0 + V7_QW - 1 + off_diag) / V7_KT;

    // ---- LDS-DMA plan: wave w fills pieces 2w, 2w+1 of the K and V images;
    // lane -> row 4*piece + (lane>>4), stored chunk position lane&15 holds
    // logical chunk (lane&15) ^ f(row)
    auto fsw = [](int row) __attribute__((always_inline)) { return ((row & 3) << 2) | ((row >> 2) & 3); };
    int drow[PPW];
    uint32_t koff[PPW], voff[PPW];
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
        drow[i] = 4 * (PPW * wave + i) + (lane >> 4);
        const int ch = (lane & 15) ^ fsw(drow[i]);
        koff[i] = (uint32_t)(drow[i] * (int)st.kn + 8 * ch) * 2u;
        voff[i] = (uint32_t)(drow[i] * (int)st.vn + 8 * ch) * 2u;
    }
    auto dma = [&](const uint16_t* tbase, uint32_t off, uint32_t lds) __attribute__((always_inline)) {
        uint32_t keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %3\n\t"
                     "s_mov_b32 m0, %0"
                     : "=&s"(keep) : "s"(lds), "v"(off), "s"(tbase) : "memory");
    };
    const uint32_t lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem;
    auto dma_tile = [&](int t, int buf) __attribute__((always_inline)) {
        const uint16_t* kt = kp + (int64_t)t * V7_KT * st.kn;
        const uint16_t* vt = vp + (int64_t)t * V7_KT * st.vn;
        uint32_t ko[PPW], vo[PPW];
#pragma unroll
        for (int i = 0; i < PPW; ++i) {
            ko[i] = koff[i];
            vo[i] = voff[i];
        }
        if (t >= t_full) {  // ragged last tile: rows past Nk re-read row Nk-1
#pragma unroll
            for (int i = 0; i < PPW; ++i) {
                const int over = max(0, t * V7_KT + drow[i] - (Nk - 1));
                ko[i] -= (uint32_t)(over * (int)st.kn * 2);
                vo[i] -= (uint32_t)(over * (int)st.vn * 2);
            }
        }
        const uint32_t base = lds0 + buf * BUFB + (PPW * wave) * 1024;
#pragma unroll
        for (int i = 0; i < PPW; ++i) {
            dma(kt, ko[i], base + i * 1024);
            dma(vt, vo[i], base + IMG + i * 1024);
        }
    };

    // ---- Q^T fragments (B operand)
    i32x4 qf[D / 16];
    {
        const int qr = q0 + l32;
        // rows past Nq read row 0 (finite scores, never stored): no select,
        // which hipcc otherwise re-materialises inside the K loop (32 v_cndmask
        // per tile)
        const uint16_t* src = qp + (int64_t)(qr < Nq ? qr : 0) * st.qn + 8 * h32;
#pragma unroll
        for (int kk = 0; kk < D / 16; ++kk) qf[kk] = *reinterpret_cast<const i32x4*>(src + 16 * kk);
        // retire the Q loads here, before the first LDS-DMA: a volatile asm
        // that "reads" qf makes hipcc wait for the loads at this point (and
        // volatile asms keep their order, so the DMAs come after).  Otherwise
        // its vmcnt(N) waits for Q, placed at Q's first use, also wait for
        // every DMA issued since (its waitcnt pass does not count inline asm)
#pragma unroll
        for (int kk = 0; kk < D / 16; ++kk) asm volatile("" : "+v"(qf[kk]));
        if constexpr (PRE != 0) {
#pragma unroll
            for (int kk = 0; kk < D / 16; ++kk)
#pragma unroll
                for (int j = 0; j < 4; ++j) qf[kk][j] = v7_scale_pair<T>(qf[kk][j], c);
        }
    }

    // ---- fragment addresses (byte offsets inside a buffer)
    const int g = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;
    const int A0 = l32 * 256 + ((h32 ^ fsw(l32)) << 4);
    const int c0 = 2 * (g & 1) + (pp >> 1);
    const int B0 = IMG + (4 * h32 + qq) * 256 + ((c0 ^ ((qq << 2) | h32)) << 4) + 8 * (pp & 1);

    const bool sel_on = (i16 == 0 && (g & 1) == 0) || (i16 == 4 && (g & 1) == 1);
    const int one = sel_on ? V7Ones<T>::pair : 0;
    const i32x4 sel = {one, one, one, one};

    f32x16 oacc[D / 32];
#pragma unroll
    for (int d = 0; d < D / 32; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[d][r] = 0.f;
    f32x16 negm;
#pragma unroll
    for (int r = 0; r < 16; ++r) negm[r] = 0.f;
    float m_run = PRE != 0 ? 0.f : -1e30f;
    f32x4 lsum = {0.f, 0.f, 0.f, 0.f};

    i32x4 pb[2][2];
    auto X = [&](int t, int buf, auto first_tag) __attribute__((always_inline)) {
        constexpr bool FIRST = decltype(first_tag)::value;
        const char* kb = smem + buf * BUFB;
        f32x16 s[2];
        auto qk = [&]() __attribute__((always_inline)) {
#pragma unroll
            for (int tt = 0; tt < 2; ++tt) {
                const i32x4 k0 = lds_read_b128(kb, A0 + tt * 8192);
                if constexpr (PRE != 0) {
                    s[tt] = mfma32x32x16<T>(k0, qf[0], negm);
                } else {
                    f32x16 z;
#pragma unroll
                    for (int r = 0; r < 16; ++r) z[r] = 0.f;
                    s[tt] = mfma32x32x16<T>(k0, qf[0], z);
                }
#pragma unroll
                for (int kk = 1; kk < D / 16; ++kk)
                    s[tt] = mfma32x32x16<T>(lds_read_b128(kb, (A0 ^ (kk << 5)) + tt * 8192), qf[kk], s[tt]);
            }
            if (t >= t_mask) {
                // last visible key of this lane's row, relative to the lane's
                // first key of the tile: one compare against a constant per score
                const int lim = (causal ? min(q0 + l32 + off_diag, Nk - 1) : Nk - 1) - t * V7_KT - 4 * h32;
#pragma unroll
                for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        if (tt * 32 + (r & 3) + 8 * (r >> 2) > lim) s[tt][r] = -INFINITY;
            }
        };
        auto expo = [&]() __attribute__((always_inline)) {
            if constexpr (PRE != 0) {
#pragma unroll
                for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) s[tt][r] = __builtin_amdgcn_exp2f(s[tt][r]);
            } else {
                // s*c - m two scores at a time (v_pk_fma_f32)
                const f32x2 c2 = {c, c}, nm2 = {-m_run, -m_run};
#pragma unroll
                for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                    for (int r = 0; r < 16; r += 2) {
                        const f32x2 y = __builtin_elementwise_fma(f32x2{s[tt][r], s[tt][r + 1]}, c2, nm2);
                        s[tt][r] = __builtin_amdgcn_exp2f(y.x);
                        s[tt][r + 1] = __builtin_amdgcn_exp2f(y.y);
                    }
            }
        };
        stamp(0);
        qk();
        float mx = fmaxf(s[0][0], s[1][0]), my = fmaxf(s[0][1], s[1][1]);
#pragma unroll
        for (int r = 2; r < 16; r += 2) {
            mx = fmaxf(fmaxf(mx, s[0][r]), s[1][r]);
            my = fmaxf(fmaxf(my, s[0][r + 1]), s[1][r + 1]);
        }
        mx = v7_xor32_max(fmaxf(mx, my));
        if constexpr (STAMP) asm volatile("" ::"v"(mx));
        stamp(1);
        if constexpr (FIRST) {
            if constexpr (PRE != 0) {
                const float delta = mx == -INFINITY ? 0.f : mx;
                m_run = delta;
#pragma unroll
                for (int r = 0; r < 16; ++r) negm[r] = -m_run;
#pragma unroll
                for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) s[tt][r] -= delta;
            } else {
                m_run = mx == -INFINITY ? -1e30f : mx * c;
            }
            expo();
        } else {
            expo();
            asm volatile("" : "+v"(s[0]), "+v"(s[1]));
            stamp(2);
            const bool up = PRE != 0 ? mx > v7_thr<T>() : mx * c > m_run + v7_thr<T>();
            if (__ballot(up)) {
                float alpha;
                if constexpr (PRE != 0) {
                    const float delta = up ? mx : 0.f;
                    m_run += delta;
#pragma unroll
                    for (int r = 0; r < 16; ++r) negm[r] = -m_run;
                    alpha = __builtin_amdgcn_exp2f(-delta);
                } else {
                    const float m_new = up ? mx * c : m_run;
                    alpha = __builtin_amdgcn_exp2f(m_run - m_new);
                    m_run = m_new;
                }
                qk();
                expo();
#pragma unroll
                for (int d = 0; d < D / 32; ++d)
#pragma unroll
                    for (int r = 0; r < 16; ++r) oacc[d][r] *= alpha;
                lsum[0] *= alpha;
            }
        }
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
        if constexpr (STAMP) asm volatile("" ::"v"(pb[0][0]), "v"(pb[0][1]), "v"(pb[1][0]), "v"(pb[1][1]));
        stamp(3);
    };
    auto Y = [&](int buf) __attribute__((always_inline)) {
        const char* vb = smem + buf * BUFB;
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) lsum = mfma16x16x32<T>(sel, pb[tt][s2], lsum);
#pragma unroll
        for (int dblk = 0; dblk < D / 32; ++dblk) {
            const int alo = B0 ^ (dblk << 6), ahi = (alo ^ 32) + 2048;
#pragma unroll
            for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    const int ro = (tt * 32 + 16 * s2) * 256;
                    const i32x2 lo = lds_read_tr16(vb, alo + ro);
                    const i32x2 hi = lds_read_tr16(vb, ahi + ro);
                    oacc[dblk] = mfma32x32x16<T>(i32x4{lo.x, lo.y, hi.x, hi.y}, pb[tt][s2], oacc[dblk]);
                }
        }
        stamp(4);
    };
    // counted wait: tile t+1's pieces landed while t+2's (4 per wave) fly
    auto wait_next = [&](bool two_in_flight) __attribute__((always_inline)) {
        if (two_in_flight) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        stamp(5);
        __syncthreads();
        stamp(6);
    };

    if constexpr (NW4) {
        if (nt > 0) {
            dma_tile(0, 0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            auto tile4 = [&](int t, auto first_tag) __attribute__((always_inline)) {
                stamp(-1);
                if (t + 1 < nt) dma_tile(t + 1, (t + 1) & 1);
                if (t <= t_last) {
                    X(t, t & 1, first_tag);
                    Y(t & 1);
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                stamp(5);
                __syncthreads();
                stamp(6);
            };
            tile4(0, std::true_type{});
            for (int t = 1; t < nt; ++t) tile4(t, std::false_type{});
        }
    } else if (nt > 0) {
        dma_tile(0, 0);
        if (nt > 1) dma_tile(1, 1);
        // (Q's own loads were waited for by the compiler above)
        wait_next(nt > 1);
        int cur = 0;
        auto tile = [&](int t, auto first_tag) __attribute__((always_inline)) {
            stamp(-1);
            const int n2 = cur == 0 ? 2 : cur - 1;  // (cur + 2) % 3
            if (t + 2 < nt) dma_tile(t + 2, n2);
            if (t <= t_last) {
                X(t, cur, first_tag);
                Y(cur);
            }
            wait_next(t + 2 < nt);
            cur = cur == 2 ? 0 : cur + 1;
        };
        tile(0, std::true_type{});
        for (int t = 1; t < nt; ++t) tile(t, std::false_type{});
    }

#ifdef PLI_FLASH_STAMPS
    if constexpr (STAMP) {
        if (lane == 0) {
#pragma unroll
            for (int i = 0; i < 7; ++i) atomicAdd(&g_v7_stamps[i], st_sum[i]);
            atomicAdd(&g_v7_stamps[8], (unsigned long long)nt);
            atomicAdd(&g_v7_stamps[9], 1ull);
        }
    }
#endif
    const float l = v7_xor32_sum(lsum[0]);
    const float inv = l > 0.f ? 1.f / l : 0.f;
    const int qr = q0 + l32;
    if (qr < Nq) {
        uint16_t* op = o + b * st.ob + hq * st.oh + (int64_t)qr * st.on;
#pragma unroll
        for (int dblk = 0; dblk < D / 32; ++dblk)
#pragma unroll
            for (int i = 0; i < 4; i += 2) {
                const f32x16& a = oacc[dblk];
                const uint32_t ax = pack2<T>(a[4 * i] * inv, a[4 * i + 1] * inv);
                const uint32_t ay = pack2<T>(a[4 * i + 2] * inv, a[4 * i + 3] * inv);
                const uint32_t bx = pack2<T>(a[4 * i + 4] * inv, a[4 * i + 5] * inv);
                const uint32_t by = pack2<T>(a[4 * i + 6] * inv, a[4 * i + 7] * inv);
                const auto rx = __builtin_amdgcn_permlane32_swap(ax, bx, false, false);
                const auto ry = __builtin_amdgcn_permlane32_swap(ay, by, false, false);
                const int d = dblk * 32 + 8 * i + 8 * h32;
                *reinterpret_cast<i32x4*>(op + d) = i32x4{(int)rx[0], (int)ry[0], (int)rx[1], (int)ry[1]};
            }
    }
}

template <typename T, int D>
int launch_v7_typed(const void* q, const void* k, const void* v, void* o, int B, int H, int group,
                    int Nq, int Nk, const V7Strides& st, float c, int causal, hipStream_t stream,
                    int sub) {
    const int qblocks = cdiv(Nq, V7_NW * V7_QW);
    const int64_t nb = (int64_t)B * H * qblocks;
    PLI_REQUIRE(nb < (1ll << 31), "pli_flash_attn_fwd: grid too large");
    const auto* qq = (const uint16_t*)q;
    const auto* kk = (const uint16_t*)k;
    const auto* vv = (const uint16_t*)v;
    auto* oo = (uint16_t*)o;
    const dim3 grid((unsigned)nb), block(V7_NW * 64);
    switch (sub) {
        case 0:
            hipLaunchKernelGGL((attn_fwd_v7<T, D, 1>), grid, block, 0, stream, qq, kk, vv, oo, H, group,
                               Nq, Nk, st, c, causal, qblocks, (int)nb);
            break;
        case 1:
            hipLaunchKernelGGL((attn_fwd_v7<T, D, 0>), grid, block, 0, stream, qq, kk, vv, oo, H, group,
                               Nq, Nk, st, c, causal, qblocks, (int)nb);
            break;
        case 10:
            if constexpr (D == 128) {
                const int qb4 = cdiv(Nq, 4 * V7_QW);
                const int64_t nb4 = (int64_t)B * H * qb4;
                hipLaunchKernelGGL((attn_fwd_v10<T, 0, false, true>), dim3((unsigned)nb4), dim3(256), 0, stream, qq,
                                   kk, vv, oo, H, group, Nq, Nk, st, c, causal, qb4, (int)nb4);
                break;
            }
            [[fallthrough]];
        case 4:
        case 5:
            // v10 is D = 128 only; other head dims take the matching v7 body
            if constexpr (D == 128) {
                if (sub == 4)
                    hipLaunchKernelGGL((attn_fwd_v10<T, 1>), grid, block, 0, stream, qq, kk, vv, oo, H, group,
                                       Nq, Nk, st, c, causal, qblocks, (int)nb);
                else
                    hipLaunchKernelGGL((attn_fwd_v10<T, 0>), grid, block, 0, stream, qq, kk, vv, oo, H, group,
                                       Nq, Nk, st, c, causal, qblocks, (int)nb);
            } else if (sub == 4) {
                hipLaunchKernelGGL((attn_fwd_v7<T, D, 1>), grid, block, 0, stream, qq, kk, vv, oo, H, group,
                                   Nq, Nk, st, c, causal, qblocks, (int)nb);
            } else {
                hipLaunchKernelGGL((attn_fwd_v7<T, D, 0>), grid, block, 0, stream, qq, kk, vv, oo, H, group,
                                   Nq, Nk, st, c, causal, qblocks, (int)nb);
            }
            break;
        default:
            set_error("pli_flash_attn_fwd: unknown v7 body %d", sub);
            return PLI_EINVAL;
    }
    return launch_status("attn_fwd_v7");
}

}  // namespace

int launch_attn_v7(const void* q, const void* k, const void* v, void* o, int B, int H, int group,
                   int Nq, int Nk, int D, const V7Strides& st, float scale, int causal, int is_bf16,
                   hipStream_t stream, int sub) {
    const float c = scale * 1.4426950408889634f;  // log2(e) folded into the Q prescale
    if (is_bf16)
        return D == 128 ? launch_v7_typed<bf16_t, 128>(q, k, v, o, B, H, group, Nq, Nk, st, c, causal, stream, sub)
                        : launch_v7_typed<bf16_t, 64>(q, k, v, o, B, H, group, Nq, Nk, st, c, causal, stream, sub);
    return D == 128 ? launch_v7_typed<f16_t, 128>(q, k, v, o, B, H, group, Nq, Nk, st, c, causal, stream, sub)
                    : launch_v7_typed<f16_t, 64>(q, k, v, o, B, H, group, Nq, Nk, st, c, causal, stream, sub);
}

}  // namespace pli

#ifdef PLI_FLASH_STAMPS
// Diagnostic entry (tools/libpli_diag.so only): one launch of the v7 body
// `sub` (0..3 as launch_attn_v7) with stamps, contiguous [B,H,N,D] bf16,
// then the 16 stamp words (segment sums, tiles, waves) copied to `out`.
extern "C" int pli_diag_flash_stamps(const void* q, const void* k, const void* v, void* o, int B, int H,
                                     int N, int sub, unsigned long long* out) {
    using namespace pli;
    constexpr int D = 128;
    const int64_t sn = D, sh = (int64_t)N * D, sb = (int64_t)H * N * D;
    const V7Strides st{sb, sh, sn, sb, sh, sn, sb, sh, sn, sb, sh, sn};
    const int qblocks = cdiv(N, V7_NW * V7_QW);
    const int nb = B * H * qblocks;
    const float c = (1.f / sqrtf((float)D)) * 1.4426950408889634f;
    unsigned long long zero[16] = {0};
    hipMemcpyToSymbol(HIP_SYMBOL(g_v7_stamps), zero, sizeof(zero));
    const auto* qq = (const uint16_t*)q;
    const auto* kk = (const uint16_t*)k;
    const auto* vv = (const uint16_t*)v;
    auto* oo = (uint16_t*)o;
#define PLI_DIAG(PRE_) \
    hipLaunchKernelGGL((attn_fwd_v7<bf16_t, D, PRE_, true>), dim3(nb), dim3(512), 0, 0, qq, kk, vv, oo, H, 1, \
                       N, N, st, c, 0, qblocks, nb)
    switch (sub) {
        case 0: PLI_DIAG(1); break;
        case 1: PLI_DIAG(0); break;
        case 4:
            hipLaunchKernelGGL((attn_fwd_v10<bf16_t, 1, true>), dim3(nb), dim3(512), 0, 0, qq, kk, vv, oo, H, 1, N, N,
                               st, c, 0, qblocks, nb);
            break;
        case 5:
            hipLaunchKernelGGL((attn_fwd_v10<bf16_t, 0, true>), dim3(nb), dim3(512), 0, 0, qq, kk, vv, oo, H, 1, N, N,
                               st, c, 0, qblocks, nb);
            break;
        case 10: {
            const int qb4 = cdiv(N, 4 * V7_QW), nb4 = B * H * qb4;
            hipLaunchKernelGGL((attn_fwd_v10<bf16_t, 0, true, true>), dim3(nb4), dim3(256), 0, 0, qq, kk, vv, oo, H, 1,
                               N, N, st, c, 0, qb4, nb4);
            break;
        }
        default: return PLI_EINVAL;
    }
#undef PLI_DIAG
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    hipMemcpyFromSymbol(out, HIP_SYMBOL(g_v7_stamps), 16 * sizeof(unsigned long long));
    return 0;
}
#endif
