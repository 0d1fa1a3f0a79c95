// Decode-step fusion for gfx950: residual add + RMSNorm + the skinny NT GEMM
// that consumes the normalised row, in one launch.
//
// In the decode step of ch02/cached_generation.py every RMSNorm (:112-120,
// :140-160: input_norm before attention, post_attn_norm before the FFN, the
// final norm before lm_head) feeds exactly one projection.  pli_rms_gemm_nt
// runs, per 256-thread block:
//   1. the first batch of the block's weight-row loads (HBM latency overlaps 2-3);
//   2. h = a (+ residual), sum of squares, y = h * rsqrt(mean + eps) * g with
//      the thread layout and operation order of rmsnorm_vec (norm.hip), so y
//      is bitwise the row pli_rmsnorm would write; y goes to LDS (never to
//      HBM), block 0 writes h (the next residual);
//   3. one wave per output column: the skinny dot loop of gemm_skinny_nt /
//      gemm_skinny_multi (same per-lane chunk order) with x read from LDS.
// Output groups as pli_gemm_multi_nt (q / k / v straight into the caches at a
// device-resident position) or, with w_up, SwiGLU (silu(x.wg) * (x.wu)).
#include <cmath>

#include "pli_common.h"

namespace pli {
namespace {

struct RmsGroup {
    const uint16_t* w;
    const uint16_t* wu;
    uint16_t* c;
    int n;
    int64_t ldw, stride_batch, stride_token;
    const int* row_offset;
    int capacity;
};
struct RmsArgs {
    RmsGroup g[3];
    int ngroups;
};

__device__ __forceinline__ float rms_silu_mul(float g, float u) { return g / (1.f + __expf(-g)) * u; }

// block_sum of norm.hip (same order: wave butterfly, then the 4 wave partials in order)
__device__ __forceinline__ float rms_block_sum(float v, float* red) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wave] = v;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
}

template <typename T, int NB, bool SW, int RPT>
__global__ __launch_bounds__(256) void rms_gemm_skinny(const uint16_t* __restrict__ A, int64_t lda,
                                                       const uint16_t* __restrict__ R, int64_t ldr,
                                                       const uint16_t* __restrict__ G, float eps,
                                                       uint16_t* __restrict__ Hout, int64_t ldh,
                                                       int M, int S, int K, RmsArgs args) {
    extern __shared__ __attribute__((aligned(16))) char dsm[];  // y [M][K]
    __shared__ float red[4];
    constexpr int NWT = SW ? 2 : 1;
    // RPT == 1 <=> K <= 2048 (<= 256 chunks): 4 chunks per lane cover the row with
    // all 64 lanes (same per-lane chunk order as 8, so bitwise the same result)
    constexpr int CPL = (SW || RPT == 1) ? 4 : 8;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nch = K / 8;
    uint16_t* xs = reinterpret_cast<uint16_t*>(dsm);

    int n = blockIdx.x * 4 + wave;
    int gi = 0;
    while (gi < args.ngroups && n >= args.g[gi].n) n -= args.g[gi++].n;
    const bool active = gi < args.ngroups;  // inactive waves still join the norm's barriers
    const RmsGroup& Gp = args.g[active ? gi : 0];
    const uint16_t* wrow[NWT];
    wrow[0] = Gp.w + (int64_t)(active ? n : 0) * Gp.ldw;
    if constexpr (SW) wrow[NWT - 1] = Gp.wu + (int64_t)(active ? n : 0) * Gp.ldw;
    i32x4 wv[NWT][CPL];
    auto load_w = [&](int c0) {
#pragma unroll
        for (int w = 0; w < NWT; ++w)
#pragma unroll
            for (int u = 0; u < CPL; ++u) {
                const int cc = min(c0 + lane + 64 * u, nch - 1);
                wv[w][u] = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(wrow[w] + cc * 8));
            }
    };
    if (active) load_w(0);

    // ---- residual add + RMSNorm of the M rows into LDS (rmsnorm_vec's order)
    for (int bb = 0; bb < M; ++bb) {
        float v[RPT][8];
        float ss = 0.f;
#pragma unroll
        for (int i = 0; i < RPT; ++i) {
            const int c = tid + 256 * i;
            if (c < nch) {
                const i32x4 xv = *reinterpret_cast<const i32x4*>(A + bb * lda + 8 * c);
                i32x4 rv = {0, 0, 0, 0};
                if (R) rv = *reinterpret_cast<const i32x4*>(R + bb * ldr + 8 * c);
                uint32_t hw[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t xw = (uint32_t)xv[j], rw = (uint32_t)rv[j];
                    float a0 = elem<T>::to_f32(T{(uint16_t)(xw & 0xffff)});
                    float a1 = elem<T>::to_f32(T{(uint16_t)(xw >> 16)});
                    if (R) {
                        a0 = elem<T>::to_f32(elem<T>::from_f32(a0 + elem<T>::to_f32(T{(uint16_t)(rw & 0xffff)})));
                        a1 = elem<T>::to_f32(elem<T>::from_f32(a1 + elem<T>::to_f32(T{(uint16_t)(rw >> 16)})));
                    }
                    hw[j] = pack2<T>(a0, a1);
                    v[i][2 * j] = a0;
                    v[i][2 * j + 1] = a1;
                    ss = fmaf(a0, a0, fmaf(a1, a1, ss));
                }
                if (Hout && blockIdx.x == 0)
                    *reinterpret_cast<i32x4*>(Hout + bb * ldh + 8 * c) =
                        i32x4{(int)hw[0], (int)hw[1], (int)hw[2], (int)hw[3]};
            }
        }
        const float inv = 1.f / sqrtf(rms_block_sum(ss, red) / (float)K + eps);
#pragma unroll
        for (int i = 0; i < RPT; ++i) {
            const int c = tid + 256 * i;
            if (c < nch) {
                const i32x4 gv = *reinterpret_cast<const i32x4*>(G + 8 * c);
                uint32_t o[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t gw = (uint32_t)gv[j];
                    o[j] = pack2<T>(v[i][2 * j] * inv * elem<T>::to_f32(T{(uint16_t)(gw & 0xffff)}),
                                    v[i][2 * j + 1] * inv * elem<T>::to_f32(T{(uint16_t)(gw >> 16)}));
                }
                *reinterpret_cast<i32x4*>(xs + bb * K + 8 * c) =
                    i32x4{(int)o[0], (int)o[1], (int)o[2], (int)o[3]};
            }
        }
    }
    __syncthreads();
    if (!active) return;  // past the last barrier

    // ---- one output column per wave, x from LDS (gemm_skinny_nt's chunk order)
    float acc[NWT][NB];
#pragma unroll
    for (int w = 0; w < NWT; ++w)
#pragma unroll
        for (int bb = 0; bb < NB; ++bb) acc[w][bb] = 0.f;
    for (int c0 = 0; c0 < nch; c0 += 64 * CPL) {
        if (c0 > 0) load_w(c0);
#pragma unroll
        for (int u = 0; u < CPL; ++u) {
            const int cc = c0 + lane + 64 * u;
            if (cc < nch) {
#pragma unroll
                for (int bb = 0; bb < NB; ++bb) {
                    if (bb < M) {
                        const i32x4 xv = *reinterpret_cast<const i32x4*>(xs + bb * K + cc * 8);
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int xi = xv[i];
                            const float x0 = elem<T>::to_f32(T{(uint16_t)(xi & 0xffff)});
                            const float x1 = elem<T>::to_f32(T{(uint16_t)((uint32_t)xi >> 16)});
#pragma unroll
                            for (int w = 0; w < NWT; ++w) {
                                const int wi = wv[w][u][i];
                                const float w0 = elem<T>::to_f32(T{(uint16_t)(wi & 0xffff)});
                                const float w1 = elem<T>::to_f32(T{(uint16_t)((uint32_t)wi >> 16)});
                                acc[w][bb] = fmaf(w1, x1, fmaf(w0, x0, acc[w][bb]));
                            }
                        }
                    }
                }
            }
        }
    }
    const int off = Gp.row_offset ? *Gp.row_offset : 0;
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) {
        if (bb < M) {
            float r = wave_sum(acc[0][bb]);
            if constexpr (SW) r = rms_silu_mul(r, wave_sum(acc[NWT - 1][bb]));
            const int b = bb / S, srow = bb % S + off;
            if (lane == 0 && srow < Gp.capacity)
                Gp.c[b * Gp.stride_batch + (int64_t)srow * Gp.stride_token + n] =
                    __builtin_bit_cast(uint16_t, elem<T>::from_f32(r));
        }
    }
}

template <typename T, int NB, bool SW>
void launch_rms(int rpt, dim3 grid, size_t lds, hipStream_t s, const uint16_t* A, int64_t lda,
                const uint16_t* R, int64_t ldr, const uint16_t* G, float eps, uint16_t* Hout,
                int64_t ldh, int M, int S, int K, const RmsArgs& args) {
#define PLI_RMS(RPT)                                                                               \
    hipLaunchKernelGGL((rms_gemm_skinny<T, NB, SW, RPT>), grid, dim3(256), lds, s, A, lda, R, ldr, \
                       G, eps, Hout, ldh, M, S, K, args)
    if (rpt <= 1) PLI_RMS(1);
    else if (rpt <= 2) PLI_RMS(2);
    else PLI_RMS(4);
#undef PLI_RMS
}

}  // namespace
}  // namespace pli

extern "C" int pli_rms_gemm_nt(const void* a, int64_t lda, const void* residual, int64_t ldr,
                               const void* norm_weight, float eps, void* h_out, int64_t ldh, int m,
                               int k, int tokens_per_batch, const void* const* w,
                               const void* const* w_up, void* const* c, const int* n,
                               const int64_t* ldw, const int64_t* stride_batch,
                               const int64_t* stride_token, const int32_t* const* row_offset,
                               const int* capacity, int ngroups, int dtype, void* stream) {
    using namespace pli;
    clear_error();
    PLI_REQUIRE(a && norm_weight && w && c && n && ldw && stride_batch && stride_token &&
                    row_offset && capacity,
                "pli_rms_gemm_nt: null pointer");
    PLI_REQUIRE(ngroups >= 1 && ngroups <= 3, "pli_rms_gemm_nt: 1..3 groups, got %d", ngroups);
    PLI_REQUIRE(m >= 1 && m <= 4 && tokens_per_batch >= 1 && m % tokens_per_batch == 0,
                "pli_rms_gemm_nt: needs 1 <= m <= 4 rows (whole batches of tokens_per_batch)");
    PLI_REQUIRE(k > 0 && k % 8 == 0 && k <= 8192 && lda >= k && lda % 8 == 0 &&
                    (!residual || (ldr >= k && ldr % 8 == 0)) && (!h_out || (ldh >= k && ldh % 8 == 0)) &&
                    aligned16(a) && aligned16(norm_weight) && (!residual || aligned16(residual)) &&
                    (!h_out || aligned16(h_out)),
                "pli_rms_gemm_nt: needs k %% 8 == 0, k <= 8192, 16-byte aligned rows");
    PLI_REQUIRE(dtype == PLI_BF16 || dtype == PLI_F16, "pli_rms_gemm_nt: bf16/fp16 only");
    PLI_REQUIRE(std::isfinite(eps) && eps >= 0.f, "pli_rms_gemm_nt: bad eps");
    RmsArgs args{};
    int ntot = 0;
    for (int g = 0; g < ngroups; ++g) {
        PLI_REQUIRE(w[g] && c[g] && n[g] > 0 && ldw[g] >= k && ldw[g] % 8 == 0 && aligned16(w[g]) &&
                        (!w_up || (w_up[g] && aligned16(w_up[g]))),
                    "pli_rms_gemm_nt: bad group %d", g);
        args.g[g] = RmsGroup{(const uint16_t*)w[g], w_up ? (const uint16_t*)w_up[g] : nullptr,
                             (uint16_t*)c[g], n[g], ldw[g], stride_batch[g], stride_token[g],
                             row_offset[g], capacity[g]};
        ntot += n[g];
    }
    args.ngroups = ngroups;
    const dim3 grid((unsigned)cdiv(ntot, 4));
    const size_t lds = (size_t)m * k * 2;
    const int rpt = cdiv(k / 8, 256);
    hipStream_t s = (hipStream_t)stream;
    const auto* A = (const uint16_t*)a;
    const auto* R = (const uint16_t*)residual;
    const auto* G = (const uint16_t*)norm_weight;
    auto* Hh = (uint16_t*)h_out;
#define PLI_RMS_NB(TT, SW)                                                                                  \
    do {                                                                                                    \
        if (m <= 1) launch_rms<TT, 1, SW>(rpt, grid, lds, s, A, lda, R, ldr, G, eps, Hh, ldh, m, tokens_per_batch, k, args); \
        else if (m <= 2) launch_rms<TT, 2, SW>(rpt, grid, lds, s, A, lda, R, ldr, G, eps, Hh, ldh, m, tokens_per_batch, k, args); \
        else launch_rms<TT, 4, SW>(rpt, grid, lds, s, A, lda, R, ldr, G, eps, Hh, ldh, m, tokens_per_batch, k, args); \
    } while (0)
    if (dtype == PLI_BF16) {
        if (w_up) PLI_RMS_NB(bf16_t, true); else PLI_RMS_NB(bf16_t, false);
    } else {
        if (w_up) PLI_RMS_NB(f16_t, true); else PLI_RMS_NB(f16_t, false);
    }
#undef PLI_RMS_NB
    return launch_status("pli_rms_gemm_nt");
}
