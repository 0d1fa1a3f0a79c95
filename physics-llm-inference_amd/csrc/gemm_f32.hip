// fp32 GEMM for gfx950: the ch05 tiled-matmul demo (ch05/tiled_matmul.cu:9-61)
// on the matrix cores, and its naive contrast kernel.
//
// gemm_f32_mfma: C = A B (or A B^T) + bias, fp32 in / fp32 accumulate on
// v_mfma_f32_32x32x2_f32 (exact f32 fma chain, 64 FLOP/clk/SIMD -- the same
// rate as the fp32 VALU, but one instruction per 4096 FLOPs and no VALU left
// busy).  128x128 workgroup tile, 4 waves of 64x64 (2x2 MFMA tiles of
// 32x32; 8 waves of 64x32 when the grid is under two workgroups per CU), K tiles of 32 register-staged into a double-buffered LDS image
// ([k][m] / [k][n], rows padded to 129 floats where the transposed stores
// need it), one barrier per K tile.  Lane l feeds A[i = l&31][k = l>>5] and
// B[k = l>>5][j = l&31] of each k-pair: consecutive words for every half-wave.
//
// gemm_naive_f32: ch05/tiled_matmul.cu:9-20 naive_matmul, one thread per
// output element reading A and B straight from global memory (the contrast
// the tiled kernels are measured against in ch05).
#include "gemm_f32.h"
#include "pli_common.h"

namespace pli {
namespace {

constexpr int FT = 128, FP = FT + 1;
#ifndef F32_KT8
#define F32_KT8 32  // K tile of the eight-wave form (A/B knob)
#endif

// NW = 4: waves of 64x64 (2x2 MFMA tiles); NW = 8 (two waves per SIMD, for
// grids of fewer than two workgroups per CU, e.g. the ch05 demo's 2048^3):
// waves of 64x32 (2x1), the same per-output MFMA chains (bitwise equal).
template <bool TRANS_B, int NW = 4, int FK = 32>
__global__ __launch_bounds__(64 * NW, 8 / NW) void gemm_f32_mfma(const float* __restrict__ A,
                                                               const float* __restrict__ B,
                                                               float* __restrict__ C,
                                                               const float* __restrict__ bias, int M, int N,
                                                               int K, int64_t lda, int64_t ldb, int64_t ldc) {
    // As[buf][k][m] (pad 129), Bs[buf][k][n] (pad 129 when transposed on store)
    constexpr int BS_LD = TRANS_B ? FP : FT;
    constexpr int NT = 64 * NW, NJ = NW == 4 ? 2 : 1, WNS = 32 * NJ;  // threads, n-tiles per wave, wave width
    __shared__ float As[2][FK][FP];
    __shared__ __attribute__((aligned(16))) float Bs[2][FK][BS_LD];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = NW == 4 ? wave >> 1 : wave >> 2, wn = NW == 4 ? wave & 1 : wave & 3;
    const int h32 = lane >> 5, l32 = lane & 31;
    const int bm = blockIdx.y * FT, bn = blockIdx.x * FT;

    // staging: 32 FK float4 of A and of B per K tile
    constexpr int NS = 32 * FK / NT, RQ = FK / 4;  // float4 per thread, per A / NT-B row
    f32x4 ra[NS], rb[NS];
    auto load = [&](int k0) {
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            const int idx = tid + NT * i;
            {   // A[m][k0 + 4q .. +3]
                const int m = idx / RQ, q = idx % RQ;
                const int gm = bm + m, gk = k0 + 4 * q;
                ra[i] = (gm < M && gk < K) ? *reinterpret_cast<const f32x4*>(A + (int64_t)gm * lda + gk)
                                           : f32x4{0.f, 0.f, 0.f, 0.f};
            }
            if constexpr (TRANS_B) {  // B[n][k0 + 4q .. +3]
                const int n = idx / RQ, q = idx % RQ;
                const int gn = bn + n, gk = k0 + 4 * q;
                rb[i] = (gn < N && gk < K) ? *reinterpret_cast<const f32x4*>(B + (int64_t)gn * ldb + gk)
                                           : f32x4{0.f, 0.f, 0.f, 0.f};
            } else {  // B[k0 + k][n0 + 4q .. +3]
                const int k = idx >> 5, q = idx & 31;
                const int gk = k0 + k, gn = bn + 4 * q;
                rb[i] = (gk < K && gn < N) ? *reinterpret_cast<const f32x4*>(B + (int64_t)gk * ldb + gn)
                                           : f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            const int idx = tid + NT * i;
            {
                const int m = idx / RQ, q = idx % RQ;
#pragma unroll
                for (int j = 0; j < 4; ++j) As[buf][4 * q + j][m] = ra[i][j];
            }
            if constexpr (TRANS_B) {
                const int n = idx / RQ, q = idx % RQ;
#pragma unroll
                for (int j = 0; j < 4; ++j) Bs[buf][4 * q + j][n] = rb[i][j];
            } else {
                const int k = idx >> 5, q = idx & 31;
                *reinterpret_cast<f32x4*>(&Bs[buf][k][4 * q]) = rb[i];
            }
        }
    };

    f32x16 acc[2][NJ];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int nk = cdiv(K, FK);
    load(0);
    store(0);
    __syncthreads();
    for (int t = 0; t < nk; ++t) {
        const int buf = t & 1;
        if (t + 1 < nk) load((t + 1) * FK);
#pragma unroll
        for (int kp = 0; kp < FK; kp += 2) {
            const int kr = kp + h32;
            float a[2], b[NJ];
#pragma unroll
            for (int i = 0; i < 2; ++i) a[i] = As[buf][kr][wm * 64 + 32 * i + l32];
#pragma unroll
            for (int j = 0; j < NJ; ++j) b[j] = Bs[buf][kr][wn * WNS + 32 * j + l32];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        if (t + 1 < nk) store(buf ^ 1);
        __syncthreads();
    }

    // C/D map: col = l32, row = (r&3) + 8(r>>2) + 4h32 of each 32x32 tile
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int n = bn + wn * WNS + 32 * j + l32;
            if (n >= N) continue;
            const float bv = bias ? bias[n] : 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = bm + wm * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h32;
                if (m < M) C[(int64_t)m * ldc + n] = acc[i][j][r] + bv;
            }
        }
}

__global__ __launch_bounds__(256) void gemm_naive_f32(const float* __restrict__ A, const float* __restrict__ B,
                                                      float* __restrict__ C, int M, int N, int K, int64_t lda,
                                                      int64_t ldb, int64_t ldc) {
    const int n = blockIdx.x * 16 + (threadIdx.x & 15);
    const int m = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (m >= M || n >= N) return;
    float s = 0.f;
    for (int k = 0; k < K; ++k) s = fmaf(A[(int64_t)m * lda + k], B[(int64_t)k * ldb + n], s);
    C[(int64_t)m * ldc + n] = s;
}

}  // namespace

bool gemm_f32_mfma_ok(const void* a, const void* b, const void* c, int k, int n, int64_t lda, int64_t ldb,
                      int trans_b) {
    const bool al = aligned16(a) && aligned16(b) && aligned16(c);
    return al && k % 4 == 0 && lda % 4 == 0 && ldb % 4 == 0 && (trans_b || n % 4 == 0);
}

int launch_gemm_f32_mfma(const void* a, const void* b, void* c, const void* bias, int M, int N, int K,
                         int64_t lda, int64_t ldb, int64_t ldc, int trans_b, hipStream_t s) {
    const dim3 grid(cdiv(N, FT), cdiv(M, FT));
    // fewer than two workgroups per CU: eight waves per workgroup (two per
    // SIMD) so one wave's LDS reads and barrier overlap the other's MFMAs
    const bool w8 = (int64_t)grid.x * grid.y < 2 * (int64_t)cu_count(s);
#define F32_LAUNCH(TB, NW) \
    hipLaunchKernelGGL((gemm_f32_mfma<TB, NW, NW == 8 ? F32_KT8 : 32>), grid, dim3(64 * NW), 0, s, (const float*)a, \
                       (const float*)b, \
                       (float*)c, (const float*)bias, M, N, K, lda, ldb, ldc)
    if (trans_b) { if (w8) F32_LAUNCH(true, 8); else F32_LAUNCH(true, 4); }
    else { if (w8) F32_LAUNCH(false, 8); else F32_LAUNCH(false, 4); }
#undef F32_LAUNCH
    return launch_status("gemm_f32_mfma");
}

}  // namespace pli

extern "C" int pli_gemm_naive(const float* a, const float* b, float* c, int m, int n, int k, int64_t lda,
                              int64_t ldb, int64_t ldc, void* stream) {
    using namespace pli;
    clear_error();
    PLI_REQUIRE(m >= 0 && n >= 0 && k >= 0 && lda >= k && ldb >= n && ldc >= n,
                "pli_gemm_naive: bad shape / leading dimensions");
    if (m == 0 || n == 0) return PLI_OK;  // (empty operands may be NULL, pli.h)
    PLI_REQUIRE(c && (k == 0 || (a && b)), "pli_gemm_naive: null pointer");
    hipLaunchKernelGGL(gemm_naive_f32, dim3(cdiv(n, 16), cdiv(m, 16)), dim3(256), 0, (hipStream_t)stream, a, b,
                       c, m, n, k, lda, ldb, ldc);
    return launch_status("gemm_naive_f32");
}
