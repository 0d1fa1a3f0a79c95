// attn_fwd_w4: flash-attention forward, ONE wave per SIMD (gfx950, D = 128).
//
// Same arithmetic as attn_fwd_v2 variant 21 (flash_attn.hip; reference
// ch06/flash_attention.py:14-74): S^T = K Q^T and O^T += V^T P^T on
// v_mfma_f32_32x32x16, the query row on the lane, fp32 statistics, defer-max
// (the running max moves only when a tile raises it by more than 8 in log2
// units) and the row sum taken over the 16-bit-rounded P.
//
// What changes is the schedule.  A workgroup is 4 waves x 64 query rows (two
// 32-row blocks r0, r1 per wave) and each wave owns its SIMD's whole register
// file (O in the accumulator half), so no partner wave hides the softmax:
// the wave overlaps it with its OWN matrix work.  Per 64-key tile t:
//
//   slot 1:  MFMA  QK^T r0(t+1) (16) + PV r0(t) (16)   ||  VALU softmax r1(t)
//   slot 2:  MFMA  QK^T r1(t+1) (16) + PV r1(t) (16)   ||  VALU softmax r0(t+1)
//
// Every MFMA gap then carries about four softmax instructions and one or two
// LDS fragment reads; the two blocks' softmax never sits on the critical path.
// K runs one tile ahead of V: iteration t reads K(t+1) and V(t) and LDS-DMAs
// (global_load_lds, 1 KiB lane-linear pieces, XOR swizzle applied on the
// source address) K(t+2) and V(t+1) into 2-deep rings; one barrier per tile.
#include <cmath>
#include <type_traits>

#include "flash_w4.h"
#include "pli_common.h"

namespace pli {
namespace {

constexpr int W4_KT = 64;       // keys per tile
constexpr int W4_IMG = 64 * 256;  // one [64][128] 16-bit tile image (16 KiB)
constexpr float W4_DEFER = 8.f;   // defer-max threshold (log2 units)

__device__ __forceinline__ uint32_t w4_lds_addr(const char* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
__device__ __forceinline__ float w4_xor32_max(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float w4_xor32_sum(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// XOR swizzle of a [64][256 B] image: chunk' = chunk ^ fsw(row), conflict-free
// for the b128 K-fragment read and the tr_b16 V^T read (flash_attn.hip seg).
__device__ __forceinline__ int w4_fsw(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

// O^T += A.B with the accumulator pinned to AGPRs (inline asm: the compiler
// neither schedules it as an MFMA nor pads its hazards; callers keep every
// VALU producer of A/B and every reader of acc well away from it)
template <typename T> __device__ __forceinline__ void w4_mfma_acc(f32x16& acc, i32x4 a, i32x4 b);
template <> __device__ __forceinline__ void w4_mfma_acc<bf16_t>(f32x16& acc, i32x4 a, i32x4 b) {
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
template <> __device__ __forceinline__ void w4_mfma_acc<f16_t>(f32x16& acc, i32x4 a, i32x4 b) {
    asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// S^T = A.B (C = 0) and S^T += A.B: accumulator in VGPRs, B (= Q) in AGPRs
template <typename T> __device__ __forceinline__ void w4_mfma_v0(f32x16& acc, i32x4 a, i32x4 b) {
    if constexpr (std::is_same<T, bf16_t>::value)
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "a"(b));
    else
        asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "a"(b));
}
template <typename T> __device__ __forceinline__ void w4_mfma_v(f32x16& acc, i32x4 a, i32x4 b) {
    if constexpr (std::is_same<T, bf16_t>::value)
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "a"(b));
    else
        asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "a"(b));
}

// empty volatile asm: the value must be computed before this point and is
// read after it -- pins VALU work between the (volatile asm) MFMAs
__device__ __forceinline__ void w4_pin(float& a) { asm volatile("" : "+v"(a)); }
__device__ __forceinline__ void w4_pin(float& a, float& b) { asm volatile("" : "+v"(a), "+v"(b)); }
__device__ __forceinline__ void w4_pin(float& a, float& b, float& c, float& d) {
    asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
}
__device__ __forceinline__ void w4_pin(f32x16& a, f32x16& b) { asm volatile("" : "+v"(a), "+v"(b)); }
__device__ __forceinline__ void w4_pin(f32x16& a) { asm volatile("" : "+v"(a)); }
__device__ __forceinline__ void w4_pin(f32x16& a, float& b, float& c) {
    asm volatile("" : "+v"(a), "+v"(b), "+v"(c));
}

template <typename T, int W4_PD>
__global__ __launch_bounds__(256, 1) void attn_fwd_w4(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
    const uint16_t* __restrict__ v, uint16_t* __restrict__ o, int H, int group,
    int Nq, int Nk, W4Strides st, float c, int causal, int qblocks, int nblocks) {
    constexpr int KT = W4_KT;
    __shared__ __attribute__((aligned(1024))) char smem[4 * W4_IMG];  // K ring 0-1, V ring 2-3

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int h32 = lane >> 5, l32 = lane & 31;
    const int lb = xcd_remap(blockIdx.x, nblocks);
    const int bh = lb / qblocks;
    const int qblk = causal ? qblocks - 1 - lb % qblocks : lb % qblocks;
    const int b = bh / H, hq = bh % H, hk = hq / group;
    const int qbase = qblk * 256;
    const int q0 = qbase + wave * 64;  // rows q0 .. q0+31 = block 0, +32 .. +63 = block 1
    const int off_diag = Nk - Nq;

    const uint16_t* qp = q + b * st.qb + hq * st.qh;
    const uint16_t* kp = k + b * st.kb + hk * st.kh;
    const uint16_t* vp = v + b * st.vb + hk * st.vh;

    int kv_end = Nk;
    if (causal) kv_end = min(Nk, qbase + 256 + off_diag);
    const int nt = kv_end > 0 ? cdiv(kv_end, KT) : 0;
    int t_mask = Nk / KT;  // first tile block 0 of this wave must mask
    if (causal) t_mask = min(t_mask, max(0, (q0 + off_diag + 1) / KT));

    // ---- LDS-DMA plan: the wave fills pieces 4*wave+i (rows 16*wave+4i+(lane>>4))
    int drow[4], koff[4], voff[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        drow[i] = 16 * wave + 4 * i + (lane >> 4);
        const int ch = (lane & 15) ^ w4_fsw(drow[i]);
        koff[i] = drow[i] * (int)st.kn + 8 * ch;
        voff[i] = drow[i] * (int)st.vn + 8 * ch;
    }
    // piece i of tile t of one operand into ring image img
    auto dma_piece = [&](const uint16_t* base, int64_t sn, int off, int i, int t, int img) {
        const uint16_t* tb = base + (int64_t)t * KT * sn;
        // rows past Nk re-read row Nk-1 (masked / weight 0); branch-free
        const int over = t * KT + KT > Nk ? max(0, t * KT + drow[i] - (Nk - 1)) : 0;
        const uint32_t m0v = w4_lds_addr(smem + img * W4_IMG + (4 * wave + i) * 1024);
        // inline asm: invisible to hipcc's waitcnt pass (no vmcnt(0) drain
        // before the LDS reads); the explicit vmcnt(0) + barrier order it
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
                     :: "s"(m0v), "v"(tb + (off - over * (int)sn)) : "memory", "m0");
    };

    // ---- fragment addresses (byte offsets inside an image)
    //   K (A of S^T = K Q^T): row tt*32 + l32, chunk 2kk + h32 -> (A0 ^ (kk<<5)) + tt*8192
    //   V^T (A of O^T += V^T P^T): (B0 ^ (dblk<<6)) + ro, hi half ((.. ^ 32) + 2048)
    const int g = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;
    int A0 = l32 * 256 + ((h32 ^ w4_fsw(l32)) << 4);
    const int c0 = 2 * (g & 1) + (pp >> 1);
    int B0 = (4 * h32 + qq) * 256 + ((c0 ^ ((qq << 2) | h32)) << 4) + 8 * (pp & 1);

    // ---- Q fragments (B operand): row q0 + 32r + l32, columns 16kk + 8h32 .. +7
    i32x4 qf[2][8];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const int qr = q0 + 32 * r + l32;
        const bool ok = qr < Nq;
        const uint16_t* src = qp + (int64_t)(ok ? qr : 0) * st.qn + 8 * h32;
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
            const i32x4 x = *reinterpret_cast<const i32x4*>(src + 16 * kk);
            qf[r][kk] = ok ? x : i32x4{0, 0, 0, 0};
        }
    }

    f32x16 oacc[2][4];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int d = 0; d < 4; ++d)
#pragma unroll
            for (int e = 0; e < 16; ++e) oacc[r][d][e] = 0.f;
    float m_run[2] = {-1e30f, -1e30f}, l_run[2] = {0.f, 0.f}, alpha[2] = {1.f, 1.f};
    f32x16 sc[2][2];   // S^T of block r: [tt] = keys tt*32.., lane = query row
    i32x4 pk[2][2][2]; // P of block r packed to 16 bits: [tt][s2]

    // ------------------------------------------------------------------
    // one slot = up to 32 MFMAs (QK^T of block rq over K image kimg, then PV
    // of block rp over V image vimg) with the softmax of block rs cut into 32
    // chunks, chunk k placed after MFMA k.  MFMAs are volatile asm, so the
    // LDS fragment reads (issued PD MFMAs ahead) and the DMA pieces keep their
    // source order around them; each softmax chunk is held between MFMAs by
    // empty asm "pins" on its inputs and outputs.
    // dma_tag: DMA kind (-1 none, 0 K tile t_dma, 1 V tile t_dma); t_dma is
    // clamped to nt-1 by the caller (a dummy refill of an image nobody reads
    // again keeps the slot free of branches)
    auto slot = [&](auto next_tag, auto pv_tag, auto sm_tag, auto mask_tag, auto dma_tag, int rq,
                    int rp, int rs, int t_sm, int kimg, int vimg, int t_dma) {
        constexpr int DMAK = decltype(dma_tag)::value;
        constexpr bool NEXT = decltype(next_tag)::value;  // QK^T present
        constexpr bool PVP = decltype(pv_tag)::value;     // PV present
        constexpr bool SM = decltype(sm_tag)::value;      // softmax present
        constexpr bool MASK = decltype(mask_tag)::value;
        constexpr int NQK = NEXT ? 16 : 0, NM = NQK + (PVP ? 16 : 0);
        constexpr int PD = W4_PD;
        const int kab = kimg * W4_IMG + A0;
        const int vbb = vimg * W4_IMG + B0;
        i32x4 fr[NM];
        auto read = [&](int j) {
            if (j < NQK) {
                const int tt = j >> 3, kk = j & 7;
                fr[j] = lds_read_b128(smem, (kab ^ (kk << 5)) + tt * 8192);
            } else {
                const int jj = j - NQK, dblk = jj >> 2, tt = (jj >> 1) & 1, s2 = jj & 1;
                const int alo = vbb ^ (dblk << 6), ahi = (alo ^ 32) + 2048;
                const int ro = (tt * 32 + 16 * s2) * 256;
                const i32x2 lo = lds_read_tr16(smem, alo + ro);
                const i32x2 hi = lds_read_tr16(smem, ahi + ro);
                fr[j] = i32x4{lo.x, lo.y, hi.x, hi.y};
            }
        };
        auto mfma = [&](int j) {
            if (j < NQK) {
                const int tt = j >> 3, kk = j & 7;
                if (kk == 0) w4_mfma_v0<T>(sc[rq][tt], fr[j], qf[rq][kk]);
                else w4_mfma_v<T>(sc[rq][tt], fr[j], qf[rq][kk]);
            } else {
                const int jj = j - NQK, dblk = jj >> 2, tt = (jj >> 1) & 1, s2 = jj & 1;
                w4_mfma_acc<T>(oacc[rp][dblk], fr[j], pk[rp][tt][s2]);
            }
        };
        // softmax state of block rs
        float ch[4], mx = 0.f, mnew = 0.f, alph = 1.f, pe[32], rs0 = 0.f, rs1 = 0.f;
        auto S = [&](int idx) -> float { return sc[rs][idx >> 4][idx & 15]; };
        auto chunk = [&](int k) {
            if (k == 0 && MASK) {
                const int last = causal ? min(q0 + 32 * rs + l32 + off_diag, Nk - 1) : Nk - 1;
                const int thr = last - t_sm * KT - 4 * h32;
#pragma unroll
                for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                    for (int e = 0; e < 16; ++e)
                        if (tt * 32 + (e & 3) + 8 * (e >> 2) > thr) sc[rs][tt][e] = -INFINITY;
            }
            if (k < 4) {  // four independent max chains over 8 scores each
                if (k == 0) w4_pin(sc[rs][0], sc[rs][1]);
#pragma unroll
                for (int cc = 0; cc < 4; ++cc) {
                    const int b8 = 8 * cc;
                    if (k == 0) ch[cc] = max3(S(b8), S(b8 + 1), S(b8 + 2));
                    else if (k == 1) ch[cc] = max3(ch[cc], S(b8 + 3), S(b8 + 4));
                    else if (k == 2) ch[cc] = max3(ch[cc], S(b8 + 5), S(b8 + 6));
                    else ch[cc] = max3(ch[cc], S(b8 + 7), S(b8 + 7));
                }
                w4_pin(ch[0], ch[1], ch[2], ch[3]);
            } else if (k == 4) {
                mx = max3(ch[0], ch[1], ch[2]);
                mx = w4_xor32_max(max3(mx, ch[3], ch[3]));
                w4_pin(mx);
            } else if (k == 5) {
                const float mc = mx * c, mr = m_run[rs];
                mnew = mc > mr + W4_DEFER ? fmaxf(mr, mc) : mr;
                w4_pin(mnew);
            } else if (k == 6) {
                alph = __builtin_amdgcn_exp2f(m_run[rs] - mnew);
                w4_pin(alph);
            } else if (k < 23) {  // 16 chunks x 2 scores: p = exp2(s*c - m)
                const int i0 = 2 * (k - 7);
                float a = S(i0), b2 = S(i0 + 1);
                w4_pin(a, b2);
                pe[i0] = __builtin_amdgcn_exp2f(fmaf(a, c, -mnew));
                pe[i0 + 1] = __builtin_amdgcn_exp2f(fmaf(b2, c, -mnew));
                w4_pin(pe[i0], pe[i0 + 1]);
            } else if (k < 31) {  // 8 chunks x 2 packed words + rounded row sums
                const int w0 = 2 * (k - 23);  // words w0, w0+1: word w = scores 2w, 2w+1
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int w = w0 + u, tt = w >> 3, s2 = (w >> 2) & 1, cpn = w & 3;
                    const uint32_t pw = pack2<T>(pe[2 * w], pe[2 * w + 1]);
                    pk[rs][tt][s2][cpn] = (int)pw;
                    if (u == 0) rs0 = add_pair<T>(pw, rs0);
                    else rs1 = add_pair<T>(pw, rs1);
                }
                w4_pin(rs0, rs1);
            } else {
                l_run[rs] = fmaf(l_run[rs], alph, rs0 + rs1);
                m_run[rs] = mnew;
                alpha[rs] = alph;
            }
        };
#pragma unroll
        for (int j = 0; j < PD && j < NM; ++j) read(j);
#pragma unroll
        for (int j = 0; j < NM; ++j) {
            if (j + PD < NM) read(j + PD);
            mfma(j);
            if (DMAK >= 0 && (j & 7) == 2) {  // one DMA piece every 8 MFMAs
                const int i = j >> 3;
                if (i < 4) {
                    if (DMAK == 0) dma_piece(kp, st.kn, koff[i], i, t_dma, t_dma & 1);
                    else dma_piece(vp, st.vn, voff[i], i, t_dma, 2 + (t_dma & 1));
                }
            }
            if constexpr (SM) {
                if (NM == 32) chunk(j);
                else { chunk(2 * j); chunk(2 * j + 1); }
            }
        }
        if (DMAK >= 0 && NM < 32) {  // short slot: the remaining pieces
#pragma unroll
            for (int i = (NM + 5) / 8; i < 4; ++i) {
                if (DMAK == 0) dma_piece(kp, st.kn, koff[i], i, t_dma, t_dma & 1);
                else dma_piece(vp, st.vn, voff[i], i, t_dma, 2 + (t_dma & 1));
            }
        }
    };
    auto rescale = [&](int r) {
        if (__builtin_amdgcn_ballot_w64(alpha[r] != 1.f)) {
            // O lives in AGPRs: 12 wait states after its last MFMA before the
            // compiler's v_accvgpr_read (inline asm is not hazard-tracked)
            asm volatile("s_nop 7\n\ts_nop 7" : "+a"(oacc[r][0]), "+a"(oacc[r][1]), "+a"(oacc[r][2]),
                         "+a"(oacc[r][3]));
#pragma unroll
            for (int d = 0; d < 4; ++d)
#pragma unroll
                for (int e = 0; e < 16; ++e) oacc[r][d][e] *= alpha[r];
            asm volatile("s_nop 7\n\ts_nop 7" : "+a"(oacc[r][0]), "+a"(oacc[r][1]), "+a"(oacc[r][2]),
                         "+a"(oacc[r][3]));
        }
    };
    auto barrier = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };
    const std::true_type Y{};
    const std::false_type N{};
    const std::integral_constant<int, -1> DN{};
    const std::integral_constant<int, 0> DK{};
    const std::integral_constant<int, 1> DV{};

    // iteration t: slot 1 = QK r0(t+1) + PV r0(t) || softmax r1(t)
    //              slot 2 = QK r1(t+1) + PV r1(t) || softmax r0(t+1)
    // reads K(t+1) (image (t+1)&1) and V(t) (image 2 + (t&1)); DMAs K(t+2)
    // (slot 1) and V(t+1) (slot 2) into the images read in iteration t-1
    auto iter = [&](auto next_tag, auto mask_tag, int t) {
        constexpr bool NEXT = decltype(next_tag)::value;
        asm volatile("" : "+v"(A0), "+v"(B0));
        rescale(0);
        if constexpr (!NEXT) asm volatile("s_nop 4" : "+v"(pk[0][0][0]), "+v"(pk[0][0][1]),
                                          "+v"(pk[0][1][0]), "+v"(pk[0][1][1]));
        // K(t+2) -> image t&1 (held K(t)); V(t+1) -> image 2 + ((t+1)&1) (held V(t-1))
        slot(next_tag, Y, Y, mask_tag, DK, 0, 0, 1, t, (t + 1) & 1, 2 + (t & 1), min(t + 2, nt - 1));
        __builtin_amdgcn_sched_barrier(0);
        rescale(1);
        if constexpr (!NEXT) asm volatile("s_nop 4" : "+v"(pk[1][0][0]), "+v"(pk[1][0][1]),
                                          "+v"(pk[1][1][0]), "+v"(pk[1][1][1]));
        slot(next_tag, Y, next_tag, mask_tag, DV, 1, 1, 0, t + 1, (t + 1) & 1, 2 + (t & 1),
             min(t + 1, nt - 1));
        barrier();
    };

    if (nt > 0) {
        // prologue: K(0) -> image 0, K(1) -> image 1, V(0) -> image 2
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            dma_piece(kp, st.kn, koff[i], i, 0, 0);
            if (nt > 1) dma_piece(kp, st.kn, koff[i], i, 1, 1);
            dma_piece(vp, st.vn, voff[i], i, 0, 2);
        }
        // Q in AGPRs (the MFMA B operand), padded for the v_accvgpr_write -> MFMA hazard
        asm volatile("s_nop 4" : "+a"(qf[0][0]), "+a"(qf[0][1]), "+a"(qf[0][2]), "+a"(qf[0][3]),
                     "+a"(qf[0][4]), "+a"(qf[0][5]), "+a"(qf[0][6]), "+a"(qf[0][7]));
        asm volatile("s_nop 4" : "+a"(qf[1][0]), "+a"(qf[1][1]), "+a"(qf[1][2]), "+a"(qf[1][3]),
                     "+a"(qf[1][4]), "+a"(qf[1][5]), "+a"(qf[1][6]), "+a"(qf[1][7]));
        barrier();
        // S r0(0) (QK only), then S r1(0) beside softmax r0(0)
        {
            const int kab = A0;
#pragma unroll
            for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                for (int kk = 0; kk < 8; ++kk) {
                    const i32x4 kf = lds_read_b128(smem, (kab ^ (kk << 5)) + tt * 8192);
                    if (kk == 0) w4_mfma_v0<T>(sc[0][tt], kf, qf[0][kk]);
                    else w4_mfma_v<T>(sc[0][tt], kf, qf[0][kk]);
                }
            asm volatile("s_nop 7\n\ts_nop 7" : "+v"(sc[0][0]), "+v"(sc[0][1]));
        }
        if (0 >= t_mask) slot(Y, N, Y, Y, DN, 1, 0, 0, 0, 0, 0, 0);
        else slot(Y, N, Y, N, DN, 1, 0, 0, 0, 0, 0, 0);
        // every wave has read K(0) (image 0) before iteration 0 DMAs K(2) into it
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        // straight-line phases (no per-iteration mask switch: one loop body
        // per phase keeps the register assignment of O / S / P stable)
        const int t_a = max(0, min(nt - 1, t_mask - 1));  // iterations [0, t_a) need no mask
        int t = 0;
        for (; t < t_a; ++t) iter(Y, N, t);
        for (; t + 1 < nt; ++t) iter(Y, Y, t);
        iter(N, Y, t);
        asm volatile("s_nop 7\n\ts_nop 7" : "+a"(oacc[0][0]), "+a"(oacc[0][1]), "+a"(oacc[0][2]),
                     "+a"(oacc[0][3]), "+a"(oacc[1][0]), "+a"(oacc[1][1]), "+a"(oacc[1][2]),
                     "+a"(oacc[1][3]));
    }

    // ---- epilogue: O / l, 16-bit, row q0 + 32r + l32
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const float l = w4_xor32_sum(l_run[r]);
        const float inv = l > 0.f ? 1.f / l : 0.f;
        const int qr = q0 + 32 * r + l32;
        if (qr < Nq) {
            uint16_t* op = o + b * st.ob + hq * st.oh + (int64_t)qr * st.on;
#pragma unroll
            for (int dblk = 0; dblk < 4; ++dblk)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int d = dblk * 32 + 8 * i + 4 * h32;
                    const i32x2 w = {(int)pack2<T>(oacc[r][dblk][4 * i] * inv, oacc[r][dblk][4 * i + 1] * inv),
                                     (int)pack2<T>(oacc[r][dblk][4 * i + 2] * inv, oacc[r][dblk][4 * i + 3] * inv)};
                    *reinterpret_cast<i32x2*>(op + d) = w;
                }
        }
    }
}


// --------------------------------------------------------------------------
// attn_fwd_w4p: the same 4 waves x 64 rows, one wave per SIMD, as two phases
// of 32 MFMAs per 64-key tile in which every LDS fragment feeds BOTH row
// blocks (half the fragment reads and waits of attn_fwd_w4):
//
//   phase 1:  S(t+1) = K(t+1) Q^T for r0, r1   ||  finish softmax(t):
//             second half of the exps, 16-bit pack -> P(t), rounded row sums
//   phase 2:  O += P(t) V(t) for r0, r1        ||  start softmax(t+1):
//             mask, row max, deferred running max, alpha, first half of exps
//
// S is double-buffered (set t&1 holds tile t from its QK^T to its finish);
// the loop is unrolled by two so every register index is a constant.  The O
// rescale by alpha(t) (rare under defer-max) runs between the phases.  K(t+2)
// and V(t+1) are DMA'd during phase 1 into the ring images last read in
// iteration t-1; vmcnt(0) + one barrier per tile.
// diagnostic cycle stamps (variant 46 only): per-wave sums of the s_memtime
// deltas of {phase 1, between phases, phase 2, barrier, prologue, epilogue}
// and the number of waves, read back by pli_debug_w4_stamps
__device__ unsigned long long g_w4_stamps[8];

template <typename T, int PD, bool STAMP = false>
__global__ __launch_bounds__(256, 1) void attn_fwd_w4p(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
    const uint16_t* __restrict__ v, uint16_t* __restrict__ o, int H, int group,
    int Nq, int Nk, W4Strides st, float c, int causal, int qblocks, int nblocks) {
    constexpr int KT = W4_KT;
    __shared__ __attribute__((aligned(1024))) char smem[4 * W4_IMG];  // K ring 0-1, V ring 2-3

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int h32 = lane >> 5, l32 = lane & 31;
    const int lb = xcd_remap(blockIdx.x, nblocks);
    const int bh = lb / qblocks;
    const int qblk = causal ? qblocks - 1 - lb % qblocks : lb % qblocks;
    const int b = bh / H, hq = bh % H, hk = hq / group;
    const int qbase = qblk * 256;
    const int q0 = qbase + wave * 64;
    const int off_diag = Nk - Nq;
    uint64_t st_acc[6] = {0, 0, 0, 0, 0, 0}, st_last = 0;
    auto stamp = [&](int slot) {
        if constexpr (STAMP) {
            __builtin_amdgcn_sched_barrier(0);
            const uint64_t now = __builtin_amdgcn_s_memtime();
            if (slot >= 0) st_acc[slot] += now - st_last;
            st_last = now;
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    stamp(-1);

    const uint16_t* qp = q + b * st.qb + hq * st.qh;
    const uint16_t* kp = k + b * st.kb + hk * st.kh;
    const uint16_t* vp = v + b * st.vb + hk * st.vh;

    int kv_end = Nk;
    if (causal) kv_end = min(Nk, qbase + 256 + off_diag);
    const int nt = kv_end > 0 ? cdiv(kv_end, KT) : 0;
    int t_mask = Nk / KT;
    if (causal) t_mask = min(t_mask, max(0, (q0 + off_diag + 1) / KT));

    // LDS-DMA: piece i of this wave = rows 16*wave + 4i + (lane>>4); byte
    // offsets (32-bit, VGPR) against a wave-uniform 64-bit tile base (SGPRs):
    // global_load_lds in its saddr form needs no per-piece VALU.  Nk % 64 == 0
    // only: the launcher routes ragged key counts to attn_fwd_w4 (a per-piece
    // clamp of the offset gave wrong r = 1 rows on ragged tails, cause not
    // found -- see DESIGN.md 3.1)
    uint32_t koff[4], voff[4];
    const int tl = nt - 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int drow = 16 * wave + 4 * i + (lane >> 4);
        const int ch = (lane & 15) ^ w4_fsw(drow);
        koff[i] = (uint32_t)(drow * (int)st.kn + 8 * ch) * 2u;
        voff[i] = (uint32_t)(drow * (int)st.vn + 8 * ch) * 2u;
    }
    auto dma_piece = [&](bool is_v, int i, int t, int img) {
        const int64_t sn = is_v ? st.vn : st.kn;
        const uint16_t* tb = (is_v ? vp : kp) + (int64_t)t * KT * sn;
        const uint32_t ob = is_v ? voff[i] : koff[i];
        const uint32_t m0v = w4_lds_addr(smem + img * W4_IMG + (4 * wave + i) * 1024);
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2"
                     :: "s"(m0v), "v"(ob), "s"(tb) : "memory", "m0");
    };

    const int g = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;
    int A0 = l32 * 256 + ((h32 ^ w4_fsw(l32)) << 4);
    const int c0 = 2 * (g & 1) + (pp >> 1);
    int B0 = (4 * h32 + qq) * 256 + ((c0 ^ ((qq << 2) | h32)) << 4) + 8 * (pp & 1);

    i32x4 qf[2][8];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const int qr = q0 + 32 * r + l32;
        const bool ok = qr < Nq;
        const uint16_t* src = qp + (int64_t)(ok ? qr : 0) * st.qn + 8 * h32;
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
            const i32x4 x = *reinterpret_cast<const i32x4*>(src + 16 * kk);
            qf[r][kk] = ok ? x : i32x4{0, 0, 0, 0};
        }
    }

    f32x16 oacc[2][4];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int d = 0; d < 4; ++d)
#pragma unroll
            for (int e = 0; e < 16; ++e) oacc[r][d][e] = 0.f;
    float m_run[2] = {-1e30f, -1e30f}, l_run[2] = {0.f, 0.f}, alpha[2] = {1.f, 1.f};
    f32x16 sc[2][2][2];  // [set][block][tt]: S^T, then (tt = 0) the first 16 exps
    i32x4 pk[2][2][2];   // P(t) of block r, [tt][s2]
    float ch[2][4], mxv[2], rsa[2], rsb[2];

    // ---- softmax pieces (X = S set, r = block).  Every piece ends with an
    // in-place "pin" (empty volatile asm, "+v") of the registers it wrote; the
    // next piece reads them, so pieces cannot drift across the MFMAs they are
    // placed between, and no register is copied for the pin.
    auto start_chunk = [&](auto mask_tag, auto set_tag, int r, int k, int t_sm) {
        constexpr bool MASK = decltype(mask_tag)::value;
        constexpr int X = decltype(set_tag)::value;
        f32x16 (&s)[2] = sc[X][r];
        if (k == 0) {
            if constexpr (MASK) {
                const int last = causal ? min(q0 + 32 * r + l32 + off_diag, Nk - 1) : Nk - 1;
                const int thr = last - t_sm * KT - 4 * h32;
#pragma unroll
                for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                    for (int e = 0; e < 16; ++e)
                        if (tt * 32 + (e & 3) + 8 * (e >> 2) > thr) s[tt][e] = -INFINITY;
                w4_pin(s[0], s[1]);
            }
        }
        if (k < 4) {  // four max chains over 8 scores (idx = 16 tt + e)
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) {
                const int b8 = 8 * cc;
#define SV(i) s[(i) >> 4][(i) & 15]
                if (k == 0) ch[r][cc] = max3(SV(b8), SV(b8 + 1), SV(b8 + 2));
                else if (k == 1) ch[r][cc] = max3(ch[r][cc], SV(b8 + 3), SV(b8 + 4));
                else if (k == 2) ch[r][cc] = max3(ch[r][cc], SV(b8 + 5), SV(b8 + 6));
                else ch[r][cc] = max3(ch[r][cc], SV(b8 + 7), SV(b8 + 7));
#undef SV
            }
            w4_pin(ch[r][0], ch[r][1], ch[r][2], ch[r][3]);
        } else if (k == 4) {
            float mx = max3(ch[r][0], ch[r][1], ch[r][2]);
            mx = w4_xor32_max(max3(mx, ch[r][3], ch[r][3]));
            mxv[r] = mx * c;
            w4_pin(mxv[r]);
        } else if (k == 5) {
            const float mr = m_run[r], mc = mxv[r];
            const float mnew = mc > mr + W4_DEFER ? fmaxf(mr, mc) : mr;
            alpha[r] = __builtin_amdgcn_exp2f(mr - mnew);
            m_run[r] = mnew;
            w4_pin(m_run[r], alpha[r]);
        } else {  // k = 6..13: exps of scores 2(k-6), +1 (tt = 0), in place
            const int e0 = 2 * (k - 6);
            s[0][e0] = __builtin_amdgcn_exp2f(fmaf(s[0][e0], c, -m_run[r]));
            s[0][e0 + 1] = __builtin_amdgcn_exp2f(fmaf(s[0][e0 + 1], c, -m_run[r]));
            w4_pin(s[0]);
        }
    };
    auto finish_chunk = [&](auto set_tag, int r, int k) {
        constexpr int X = decltype(set_tag)::value;
        f32x16 (&s)[2] = sc[X][r];
        if (k < 8) {  // exps of scores 16 + 2k, +1 (tt = 1), in place
            const int e0 = 2 * k;
            s[1][e0] = __builtin_amdgcn_exp2f(fmaf(s[1][e0], c, -m_run[r]));
            s[1][e0 + 1] = __builtin_amdgcn_exp2f(fmaf(s[1][e0 + 1], c, -m_run[r]));
            w4_pin(s[1]);
        } else {  // k = 8..15: words 2(k-8), +1 -> 16-bit pack + rounded sums
            if (k == 8) { rsa[r] = 0.f; rsb[r] = 0.f; }
            const int w0 = 2 * (k - 8);  // words w0, w0+1 (same tt, s2): scores 2w, 2w+1
            const int tt = w0 >> 3, s2 = (w0 >> 2) & 1;
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int w = w0 + u, cpn = w & 3, e = 2 * (w & 7);
                const uint32_t pw = pack2<T>(s[tt][e], s[tt][e + 1]);
                pk[r][tt][s2][cpn] = (int)pw;
                if (u == 0) rsa[r] = add_pair<T>(pw, rsa[r]);
                else rsb[r] = add_pair<T>(pw, rsb[r]);
            }
            asm volatile("" : "+v"(pk[r][tt][s2]), "+v"(rsa[r]), "+v"(rsb[r]));
            if (k == 15) l_run[r] = fmaf(l_run[r], alpha[r], rsa[r] + rsb[r]);
        }
    };

    // ---- MFMA phases: 16 fragments x 2 blocks, reads PD fragments ahead
    auto phase_qk = [&](auto set_tag, int kimg, auto&& work) {
        constexpr int Y = decltype(set_tag)::value;
        const int kab = kimg * W4_IMG + A0;
        i32x4 fr[16];
        auto ftt = [](int f) { return f >> 3; };
        auto fkk = [](int f) { return f & 7; };
#pragma unroll
        for (int f = 0; f < 16; ++f) {
            if (f == 0) {
#pragma unroll
                for (int p2 = 0; p2 < PD; ++p2)
                    fr[p2] = lds_read_b128(smem, (kab ^ (fkk(p2) << 5)) + ftt(p2) * 8192);
            }
            if (f + PD < 16) {
                const int fn = f + PD;
                fr[fn] = lds_read_b128(smem, (kab ^ (fkk(fn) << 5)) + ftt(fn) * 8192);
            }
            const int tt = ftt(f), kk = fkk(f);
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                if (kk == 0) w4_mfma_v0<T>(sc[Y][r][tt], fr[f], qf[r][kk]);
                else w4_mfma_v<T>(sc[Y][r][tt], fr[f], qf[r][kk]);
                work(2 * f + r);
            }
        }
    };
    auto phase_pv = [&](int vimg, auto&& work) {
        const int vbb = vimg * W4_IMG + B0;
        i32x4 fr[16];
        auto rd = [&](int f) {
            const int dblk = f >> 2, tt = (f >> 1) & 1, s2 = f & 1;
            const int alo = vbb ^ (dblk << 6), ahi = (alo ^ 32) + 2048;
            const int ro = (tt * 32 + 16 * s2) * 256;
            const i32x2 lo = lds_read_tr16(smem, alo + ro);
            const i32x2 hi = lds_read_tr16(smem, ahi + ro);
            fr[f] = i32x4{lo.x, lo.y, hi.x, hi.y};
        };
#pragma unroll
        for (int f = 0; f < 16; ++f) {
            if (f == 0) {
#pragma unroll
                for (int p2 = 0; p2 < PD; ++p2) rd(p2);
            }
            if (f + PD < 16) rd(f + PD);
            const int dblk = f >> 2, tt = (f >> 1) & 1, s2 = f & 1;
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                w4_mfma_acc<T>(oacc[r][dblk], fr[f], pk[r][tt][s2]);
                work(2 * f + r);
            }
        }
    };
    auto rescale = [&](int r) {
        if (__builtin_amdgcn_ballot_w64(alpha[r] != 1.f)) {
            asm volatile("s_nop 7\n\ts_nop 7" : "+a"(oacc[r][0]), "+a"(oacc[r][1]), "+a"(oacc[r][2]),
                         "+a"(oacc[r][3]));
#pragma unroll
            for (int d = 0; d < 4; ++d)
#pragma unroll
                for (int e = 0; e < 16; ++e) oacc[r][d][e] *= alpha[r];
            asm volatile("s_nop 7\n\ts_nop 7" : "+a"(oacc[r][0]), "+a"(oacc[r][1]), "+a"(oacc[r][2]),
                         "+a"(oacc[r][3]));
        }
    };
    auto barrier = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };
    const std::true_type Y{};
    const std::false_type N{};
    const std::integral_constant<int, 0> S0{};
    const std::integral_constant<int, 1> S1{};

    // iteration t with S(t) in set X (started), S(t+1) -> set Y = 1 - X
    auto iter = [&](auto next_tag, auto mask_tag, auto set_x, int t) {
        constexpr bool NEXT = decltype(next_tag)::value;
        constexpr int X = decltype(set_x)::value;
        const std::integral_constant<int, 1 - X> set_y{};
        // opaque per iteration: recompute addresses instead of holding hoisted
        // 64-bit pointers (the register file is full)
        asm volatile("" : "+v"(A0), "+v"(B0));
        // K(t+2) -> image t&1 (held K(t)), V(t+1) -> image 2+((t+1)&1) (held
        // V(t-1)); past the last tile the source is clamped (a harmless refill
        // of an image nobody reads again)
        const int tk = min(t + 2, tl), tv = min(t + 1, tl);
        // phase 1: QK^T(t+1) || finish(t); DMA pieces one every 4 MFMAs
        auto piece = [&](int pc) {  // 0-3 K(t+2), 4-7 V(t+1)
            dma_piece(pc >= 4, pc & 3, pc >= 4 ? tv : tk, pc >= 4 ? 2 + ((t + 1) & 1) : (t & 1));
        };
        auto w1 = [&](int j) {
            finish_chunk(set_x, j & 1, j >> 1);
            if ((j & 3) == 1) piece(j >> 2);
        };
        stamp(3);
        if constexpr (NEXT) {
            phase_qk(set_y, (t + 1) & 1, w1);
        } else {
#pragma unroll
            for (int j = 0; j < 32; ++j) w1(j);
            asm volatile("s_nop 4" : "+v"(pk[0][0][0]), "+v"(pk[0][0][1]), "+v"(pk[0][1][0]),
                         "+v"(pk[0][1][1]), "+v"(pk[1][0][0]), "+v"(pk[1][0][1]),
                         "+v"(pk[1][1][0]), "+v"(pk[1][1][1]));
        }
        __builtin_amdgcn_sched_barrier(0);
        stamp(0);
        rescale(0);
        rescale(1);
        // hazard guard (asm MFMAs are not tracked): S(t+1) was written by the
        // last QK^T MFMAs and is read by start(t+1) at once; P(t) written by
        // the last VALU of phase 1 feeds the first PV MFMA
        asm volatile("s_nop 7\n\ts_nop 4"
                     : "+v"(sc[1 - X][0][0]), "+v"(sc[1 - X][0][1]), "+v"(sc[1 - X][1][0]),
                       "+v"(sc[1 - X][1][1]), "+v"(pk[0][0][0]), "+v"(pk[0][0][1]), "+v"(pk[0][1][0]),
                       "+v"(pk[0][1][1]), "+v"(pk[1][0][0]), "+v"(pk[1][0][1]), "+v"(pk[1][1][0]),
                       "+v"(pk[1][1][1]));
        __builtin_amdgcn_sched_barrier(0);
        stamp(1);
        // phase 2: PV(t) || start(t+1)
        auto w2 = [&](int j) {
            if constexpr (NEXT) {
                if (j < 28) start_chunk(mask_tag, set_y, j & 1, j >> 1, t + 1);
            }
        };
        phase_pv(2 + (t & 1), w2);
        if constexpr (!NEXT)  // O is read (or copied) by compiler code next: 12 wait states
            asm volatile("s_nop 7\n\ts_nop 4" : "+a"(oacc[0][0]), "+a"(oacc[0][1]), "+a"(oacc[0][2]),
                         "+a"(oacc[0][3]), "+a"(oacc[1][0]), "+a"(oacc[1][1]), "+a"(oacc[1][2]),
                         "+a"(oacc[1][3]));
        stamp(2);
        barrier();
    };

    if (nt > 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            dma_piece(false, i, 0, 0);
            dma_piece(false, i, min(1, tl), 1);
            dma_piece(true, i, 0, 2);
        }
        asm volatile("s_nop 4" : "+a"(qf[0][0]), "+a"(qf[0][1]), "+a"(qf[0][2]), "+a"(qf[0][3]),
                     "+a"(qf[0][4]), "+a"(qf[0][5]), "+a"(qf[0][6]), "+a"(qf[0][7]));
        asm volatile("s_nop 4" : "+a"(qf[1][0]), "+a"(qf[1][1]), "+a"(qf[1][2]), "+a"(qf[1][3]),
                     "+a"(qf[1][4]), "+a"(qf[1][5]), "+a"(qf[1][6]), "+a"(qf[1][7]));
        barrier();
        // S(0) into set 0, then start(0)
        phase_qk(S0, 0, [&](int) {});
        asm volatile("s_nop 7\n\ts_nop 7" : "+v"(sc[0][0][0]), "+v"(sc[0][0][1]), "+v"(sc[0][1][0]),
                     "+v"(sc[0][1][1]));
        if (0 >= t_mask) {
#pragma unroll
            for (int j = 0; j < 28; ++j) start_chunk(Y, S0, j & 1, j >> 1, 0);
        } else {
#pragma unroll
            for (int j = 0; j < 28; ++j) start_chunk(N, S0, j & 1, j >> 1, 0);
        }
        // every wave has read K(0) (image 0) before iteration 0 DMAs K(2) into it
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        stamp(4);
        // iterations: pairs (even t: X = 0, odd t: X = 1); the mask-free phase first
        const int t_a = max(0, min(nt - 1, t_mask - 1));
        int t = 0;
        for (; t + 1 < t_a; t += 2) {
            iter(Y, N, S0, t);
            iter(Y, N, S1, t + 1);
        }
        for (; t + 1 < nt - 1; t += 2) {
            iter(Y, Y, S0, t);
            iter(Y, Y, S1, t + 1);
        }
        // 1 or 2 iterations left (t even): [t (NEXT)], last
        if (t + 1 == nt - 1) {
            iter(Y, Y, S0, t);
            iter(N, Y, S1, t + 1);
        } else {
            iter(N, Y, S0, t);
        }
        asm volatile("s_nop 7\n\ts_nop 7" : "+a"(oacc[0][0]), "+a"(oacc[0][1]), "+a"(oacc[0][2]),
                     "+a"(oacc[0][3]), "+a"(oacc[1][0]), "+a"(oacc[1][1]), "+a"(oacc[1][2]),
                     "+a"(oacc[1][3]));
    }

#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const float l = w4_xor32_sum(l_run[r]);
        const float inv = l > 0.f ? 1.f / l : 0.f;
        const int qr = q0 + 32 * r + l32;
        if (qr < Nq) {
            uint16_t* op = o + b * st.ob + hq * st.oh + (int64_t)qr * st.on;
#pragma unroll
            for (int dblk = 0; dblk < 4; ++dblk)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int d = dblk * 32 + 8 * i + 4 * h32;
                    const i32x2 w = {(int)pack2<T>(oacc[r][dblk][4 * i] * inv, oacc[r][dblk][4 * i + 1] * inv),
                                     (int)pack2<T>(oacc[r][dblk][4 * i + 2] * inv, oacc[r][dblk][4 * i + 3] * inv)};
                    *reinterpret_cast<i32x2*>(op + d) = w;
                }
        }
    }
    if constexpr (STAMP) {
        stamp(5);
        if (lane == 0) {
#pragma unroll
            for (int i = 0; i < 6; ++i) atomicAdd(&g_w4_stamps[i], (unsigned long long)st_acc[i]);
            atomicAdd(&g_w4_stamps[6], 1ull);
            atomicAdd(&g_w4_stamps[7], (unsigned long long)(nt > 0 ? nt : 0));
        }
    }
}

}  // namespace

int launch_attn_w4(const void* q, const void* k, const void* v, void* o, int B, int H, int group,
                   int Nq, int Nk, const W4Strides& st, float scale, int causal, int is_bf16,
                   hipStream_t stream, int sub) {
    const int qblocks = cdiv(Nq, 256);
    const int64_t nb = (int64_t)B * H * qblocks;
    PLI_REQUIRE(nb < (1ll << 31), "pli_flash_attn_fwd: grid too large");
    const float c = scale * 1.4426950408889634f;
    const auto* qq = (const uint16_t*)q;
    const auto* kk = (const uint16_t*)k;
    const auto* vv = (const uint16_t*)v;
    auto* oo = (uint16_t*)o;
    const dim3 grid((unsigned)nb), block(256);
#define PLI_W4(TT, PD)                                                                             \
    hipLaunchKernelGGL((attn_fwd_w4<TT, PD>), grid, block, 0, stream, qq, kk, vv, oo, H, group, Nq, \
                       Nk, st, c, causal, qblocks, (int)nb)
#define PLI_W4P_L(...)                                                                            \
    hipLaunchKernelGGL((attn_fwd_w4p<__VA_ARGS__>), grid, block, 0, stream, qq, kk, vv, oo, H, group, \
                       Nq, Nk, st, c, causal, qblocks, (int)nb)
#define PLI_W4P(TT, PD)                                                                           \
    do {                                                                                          \
        if (Nk % W4_KT) PLI_W4(TT, 3);                                                            \
        else if (sub == 6) PLI_W4P_L(TT, 3, true);                                                \
        else PLI_W4P_L(TT, PD);                                                                   \
    } while (0)
    if (sub >= 3) {  // two-phase shared-fragment form, fragments 2 / 3 / 4 ahead (6: 3 + stamps)
        const int pd = sub == 6 ? 3 : sub - 1;
        if (is_bf16) {
            if (pd == 2) PLI_W4P(bf16_t, 2);
            else if (pd == 3) PLI_W4P(bf16_t, 3);
            else PLI_W4P(bf16_t, 4);
        } else {
            if (pd == 2) PLI_W4P(f16_t, 2);
            else if (pd == 3) PLI_W4P(f16_t, 3);
            else PLI_W4P(f16_t, 4);
        }
        return launch_status("attn_fwd_w4p");
    }
#undef PLI_W4P
#undef PLI_W4P_L
    if (is_bf16) {
        if (sub == 1) PLI_W4(bf16_t, 2);
        else if (sub == 2) PLI_W4(bf16_t, 4);
        else PLI_W4(bf16_t, 3);
    } else {
        if (sub == 1) PLI_W4(f16_t, 2);
        else if (sub == 2) PLI_W4(f16_t, 4);
        else PLI_W4(f16_t, 3);
    }
#undef PLI_W4
    return launch_status("attn_fwd_w4");
}

}  // namespace pli

// Not in pli.h: diagnostic read-back of the variant-46 cycle stamps (8 words:
// phase-1, between-phase, phase-2, barrier, prologue, epilogue cycle sums over
// waves, wave count, tile count); reset = 1 zeroes them afterwards.
extern "C" int pli_debug_w4_stamps(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pli::g_w4_stamps), sizeof(unsigned long long) * 8) != hipSuccess)
        return 1;
    if (reset) {
        const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(pli::g_w4_stamps), z, sizeof(z)) != hipSuccess) return 1;
    }
    return 0;
}
