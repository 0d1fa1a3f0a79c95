// GEMM for gfx950 (MI355X): C = A op(B) (+ bias), fp32 accumulate.
//
// Replaces torch.mm of ch03/gemm_benchmark.py:35 (NN), the 16x16 shared-memory
// tiled_matmul of ch05/tiled_matmul.cu:22-61, and F.linear of
// ch09/tensor_parallel.py:39,67 / ch01/attention.py:59-71 (NT, + bias).
//
// MFMA kernel (bf16 / fp16): 128x128 output tile, BK = 64, 4 waves in 2x2,
// each wave a 64x64 sub-tile of 2x2 v_mfma_f32_32x32x16 blocks.  The MFMA is
// issued as C^T = op(B)^T A^T so the accumulator keeps the output ROW on the
// lane and 4 consecutive columns per register quad: the epilogue writes 8-byte
// row segments with the bias added in registers.
//   A tile  [128 m][64 k]   128-B rows, XOR-swizzled, fragments by ds_read_b128
//   B tile  NT: [128 n][64 k] same image as A
//           NN: [64 k][128 n] 256-B rows; the K-strided operand fragment comes
//               from two ds_read_b64_tr_b16 (gfx950 transposed LDS read), so
//               torch.mm's row-major B needs no transpose pass in HBM.
// Tiles are register-staged into double-buffered LDS (loads for k-tile t+1 in
// flight under the MFMAs of tile t), one barrier per k-tile; blocks are
// remapped so each XCD sweeps a contiguous band of output tiles (L2 reuse of
// the A row-panel / B column-panel).
//
// Generic kernel (fp32, ragged or unaligned shapes): 64x64 LDS-tiled VALU
// kernel, 4x4 outputs per thread, fp32 accumulate.
#include "pli_common.h"

namespace pli {
namespace {

constexpr int BM = 128, BN = 128, BK = 64;

// 128-byte rows (64 x 16-bit): chunk ^= g((row>>1)&7)
__device__ __forceinline__ int off128(int row, int ch) {
    const int i = (row >> 1) & 7;
    const int g = ((i & 1) << 2) | (i >> 1);
    return row * 128 + ((ch ^ g) << 4);
}
// 256-byte rows (128 x 16-bit): chunk ^= ((row&3)<<2 | (row>>2)&3)
__device__ __forceinline__ int off256(int row, int ch) {
    const int f = ((row & 3) << 2) | ((row >> 2) & 3);
    return row * 256 + ((ch ^ f) << 4);
}

template <typename T, bool TRANS_B, bool BIAS>
__global__ __launch_bounds__(256, 2) void gemm_mfma(const uint16_t* __restrict__ A,
                                                    const uint16_t* __restrict__ Bm,
                                                    uint16_t* __restrict__ C,
                                                    const uint16_t* __restrict__ bias, int M, int N,
                                                    int K, int64_t lda, int64_t ldb, int64_t ldc,
                                                    int tiles_n, int nblocks) {
    constexpr int TILE = BM * BK * 2;  // 16 KiB per operand tile
    __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h32 = lane >> 5, l32 = lane & 31;
    const int wm = wave >> 1, wn = wave & 1;  // 2x2 waves, 64x64 each

    const int lb = xcd_remap(blockIdx.x, nblocks);
    const int m0 = (lb / tiles_n) * BM, n0 = (lb % tiles_n) * BN;
    const int ktiles = cdiv(K, BK);

    // staging: 1024 chunks of 16 B per operand tile, 4 per thread
    i32x4 ast[4], bst[4];
    auto load_tile = [&](int kt) {
        const int k0 = kt * BK;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int c = tid + 256 * i;
            {   // A: row = c/8 (m), chunk c%8 (k)
                const int r = c >> 3, ch = c & 7;
                const int mm = min(m0 + r, M - 1), kk = k0 + ch * 8;
                const i32x4 x = *reinterpret_cast<const i32x4*>(A + (int64_t)mm * lda + min(kk, K - 8));
                ast[i] = (m0 + r < M && kk < K) ? x : i32x4{0, 0, 0, 0};
            }
            if constexpr (TRANS_B) {  // B [N][K]: row = n
                const int r = c >> 3, ch = c & 7;
                const int nn = min(n0 + r, N - 1), kk = k0 + ch * 8;
                const i32x4 x = *reinterpret_cast<const i32x4*>(Bm + (int64_t)nn * ldb + min(kk, K - 8));
                bst[i] = (n0 + r < N && kk < K) ? x : i32x4{0, 0, 0, 0};
            } else {  // B [K][N]: row = k (16 chunks of n)
                const int r = c >> 4, ch = c & 15;
                const int kk = min(k0 + r, K - 1), nn = n0 + ch * 8;
                const i32x4 x = *reinterpret_cast<const i32x4*>(Bm + (int64_t)kk * ldb + min(nn, N - 8));
                bst[i] = (k0 + r < K && nn < N) ? x : i32x4{0, 0, 0, 0};
            }
        }
    };
    auto store_tile = [&](int buf) {
        char* as = smem + buf * 2 * TILE;
        char* bs = as + TILE;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int c = tid + 256 * i;
            lds_write_b128(as, off128(c >> 3, c & 7), ast[i]);
            if constexpr (TRANS_B)
                lds_write_b128(bs, off128(c >> 3, c & 7), bst[i]);
            else
                lds_write_b128(bs, off256(c >> 4, c & 15), bst[i]);
        }
    };

    f32x16 acc[2][2];  // [n-block][m-block] of C^T
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int g = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;

    load_tile(0);
    store_tile(0);
    __syncthreads();
    for (int kt = 0; kt < ktiles; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < ktiles) load_tile(kt + 1);
        const char* as = smem + buf * 2 * TILE;
        const char* bs = as + TILE;
#pragma unroll
        for (int kk = 0; kk < BK / 16; ++kk) {
            i32x4 af[2], bf[2];
#pragma unroll
            for (int mi = 0; mi < 2; ++mi)
                af[mi] = lds_read_b128(as, off128(wm * 64 + mi * 32 + l32, 2 * kk + h32));
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) {
                if constexpr (TRANS_B) {
                    bf[ni] = lds_read_b128(bs, off128(wn * 64 + ni * 32 + l32, 2 * kk + h32));
                } else {
                    // rows k = 16kk + 8h32 + {0..3} and {4..7}; cols n = 32-block + lane
                    const int row = 16 * kk + 8 * h32 + qq;
                    const int ch = (wn * 64 + ni * 32) / 8 + 2 * (g & 1) + (pp >> 1);
                    const i32x2 lo = lds_read_tr16(bs, off256(row, ch) + 8 * (pp & 1));
                    const i32x2 hi = lds_read_tr16(bs, off256(row + 4, ch) + 8 * (pp & 1));
                    bf[ni] = i32x4{lo.x, lo.y, hi.x, hi.y};
                }
            }
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
#pragma unroll
                for (int mi = 0; mi < 2; ++mi)
                    acc[ni][mi] = mfma32x32x16<T>(bf[ni], af[mi], acc[ni][mi]);
        }
        if (kt + 1 < ktiles) store_tile(buf ^ 1);
        __syncthreads();
    }

    // epilogue: acc[ni][mi][r] = C[m = m0+wm*64+mi*32+l32][n = n0+wn*64+ni*32+(r&3)+8(r>>2)+4h32]
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
        const int m = m0 + wm * 64 + mi * 32 + l32;
        if (m >= M) continue;
        uint16_t* crow = C + (int64_t)m * ldc;
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int n = n0 + wn * 64 + ni * 32 + 8 * i + 4 * h32;
                if (n >= N) continue;  // N % 8 == 0 on this path: whole quads
                float v0 = acc[ni][mi][4 * i], v1 = acc[ni][mi][4 * i + 1];
                float v2 = acc[ni][mi][4 * i + 2], v3 = acc[ni][mi][4 * i + 3];
                if constexpr (BIAS) {
                    v0 += elem<T>::to_f32(T{bias[n]});
                    v1 += elem<T>::to_f32(T{bias[n + 1]});
                    v2 += elem<T>::to_f32(T{bias[n + 2]});
                    v3 += elem<T>::to_f32(T{bias[n + 3]});
                }
                *reinterpret_cast<i32x2*>(crow + n) =
                    i32x2{(int)pack2<T>(v0, v1), (int)pack2<T>(v2, v3)};
            }
    }
}

// ---------------------------------------------------------------------------
// Generic LDS-tiled kernel (any dtype, any shape/stride), fp32 accumulate.
constexpr int GT = 64, GKT = 16;

template <typename T, bool TRANS_B>
__global__ __launch_bounds__(256) void gemm_generic(const T* __restrict__ A, const T* __restrict__ Bm,
                                                    T* __restrict__ C, const T* __restrict__ bias,
                                                    int M, int N, int K, int64_t lda, int64_t ldb,
                                                    int64_t ldc) {
    __shared__ float As[GKT][GT + 4];
    __shared__ float Bs[GKT][GT + 4];
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    const int m0 = blockIdx.y * GT, n0 = blockIdx.x * GT;
    float acc[4][4] = {};
    for (int k0 = 0; k0 < K; k0 += GKT) {
        for (int i = tid; i < GT * GKT; i += 256) {
            {   // A[m][k] -> As[k][m]
                const int r = i / GKT, kk = i % GKT;
                const int m = m0 + r, kx = k0 + kk;
                As[kk][r] = (m < M && kx < K) ? elem<T>::to_f32(A[(int64_t)m * lda + kx]) : 0.f;
            }
            if constexpr (TRANS_B) {  // B[n][k] -> Bs[k][n]
                const int r = i / GKT, kk = i % GKT;
                const int n = n0 + r, kx = k0 + kk;
                Bs[kk][r] = (n < N && kx < K) ? elem<T>::to_f32(Bm[(int64_t)n * ldb + kx]) : 0.f;
            } else {  // B[k][n] -> Bs[k][n]
                const int kk = i / GT, r = i % GT;
                const int n = n0 + r, kx = k0 + kk;
                Bs[kk][r] = (n < N && kx < K) ? elem<T>::to_f32(Bm[(int64_t)kx * ldb + n]) : 0.f;
            }
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < GKT; ++kk) {
            float a[4], b[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = As[kk][ty + 16 * i];
#pragma unroll
            for (int j = 0; j < 4; ++j) b[j] = Bs[kk][tx + 16 * j];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a[i], b[j], acc[i][j]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = m0 + ty + 16 * i;
        if (m >= M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = n0 + tx + 16 * j;
            if (n >= N) continue;
            float vv = acc[i][j];
            if (bias) vv += elem<T>::to_f32(bias[n]);
            C[(int64_t)m * ldc + n] = elem<T>::from_f32(vv);
        }
    }
}

template <typename T>
int launch_mfma(const void* a, const void* b, void* c, const void* bias, int M, int N, int K,
                int64_t lda, int64_t ldb, int64_t ldc, int trans_b, hipStream_t s) {
    const int tm = cdiv(M, BM), tn = cdiv(N, BN);
    const int64_t nb = (int64_t)tm * tn;
    PLI_REQUIRE(nb < (1ll << 31), "pli_gemm: grid too large");
    const dim3 grid((unsigned)nb), block(256);
#define PLI_GEMM_LAUNCH(TB, BI)                                                               \
    hipLaunchKernelGGL((gemm_mfma<T, TB, BI>), grid, block, 0, s, (const uint16_t*)a,          \
                       (const uint16_t*)b, (uint16_t*)c, (const uint16_t*)bias, M, N, K, lda, \
                       ldb, ldc, tn, (int)nb)
    if (trans_b) {
        if (bias) PLI_GEMM_LAUNCH(true, true); else PLI_GEMM_LAUNCH(true, false);
    } else {
        if (bias) PLI_GEMM_LAUNCH(false, true); else PLI_GEMM_LAUNCH(false, false);
    }
#undef PLI_GEMM_LAUNCH
    return launch_status("gemm_mfma");
}

template <typename T>
int launch_generic(const void* a, const void* b, void* c, const void* bias, int M, int N, int K,
                   int64_t lda, int64_t ldb, int64_t ldc, int trans_b, hipStream_t s) {
    const dim3 grid(cdiv(N, GT), cdiv(M, GT)), block(256);
    if (trans_b)
        hipLaunchKernelGGL((gemm_generic<T, true>), grid, block, 0, s, (const T*)a, (const T*)b,
                           (T*)c, (const T*)bias, M, N, K, lda, ldb, ldc);
    else
        hipLaunchKernelGGL((gemm_generic<T, false>), grid, block, 0, s, (const T*)a, (const T*)b,
                           (T*)c, (const T*)bias, M, N, K, lda, ldb, ldc);
    return launch_status("gemm_generic");
}

inline bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace
}  // namespace pli

extern "C" int pli_gemm(const void* a, const void* b, void* c, const void* bias, int m, int n,
                        int k, int64_t lda, int64_t ldb, int64_t ldc, int trans_b, int dtype,
                        void* stream) {
    using namespace pli;
    clear_error();
    PLI_REQUIRE(a && b && c, "pli_gemm: null pointer");
    PLI_REQUIRE(m >= 0 && n >= 0 && k >= 0, "pli_gemm: bad shape m=%d n=%d k=%d", m, n, k);
    if (m == 0 || n == 0) return PLI_OK;
    PLI_REQUIRE(lda >= k && ldc >= n && ldb >= (trans_b ? k : n),
                "pli_gemm: leading dimension too small (lda=%lld ldb=%lld ldc=%lld)",
                (long long)lda, (long long)ldb, (long long)ldc);
    hipStream_t s = (hipStream_t)stream;
    if (k == 0) {  // C = bias (or 0): the generic kernel handles K == 0
        switch (dtype) {
            case PLI_F32: return launch_generic<float>(a, b, c, bias, m, n, k, lda, ldb, ldc, trans_b, s);
            case PLI_F16: return launch_generic<f16_t>(a, b, c, bias, m, n, k, lda, ldb, ldc, trans_b, s);
            case PLI_BF16: return launch_generic<bf16_t>(a, b, c, bias, m, n, k, lda, ldb, ldc, trans_b, s);
            default: set_error("pli_gemm: bad dtype %d", dtype); return PLI_EINVAL;
        }
    }
    const bool vec = (dtype == PLI_BF16 || dtype == PLI_F16) && k % 8 == 0 && n % 8 == 0 &&
                     lda % 8 == 0 && ldb % 8 == 0 && ldc % 8 == 0 && al16(a) && al16(b) &&
                     al16(c) && (bias == nullptr || ((uintptr_t)bias & 7) == 0);
    if (vec) {
        if (dtype == PLI_BF16)
            return launch_mfma<bf16_t>(a, b, c, bias, m, n, k, lda, ldb, ldc, trans_b, s);
        return launch_mfma<f16_t>(a, b, c, bias, m, n, k, lda, ldb, ldc, trans_b, s);
    }
    switch (dtype) {
        case PLI_F32: return launch_generic<float>(a, b, c, bias, m, n, k, lda, ldb, ldc, trans_b, s);
        case PLI_F16: return launch_generic<f16_t>(a, b, c, bias, m, n, k, lda, ldb, ldc, trans_b, s);
        case PLI_BF16: return launch_generic<bf16_t>(a, b, c, bias, m, n, k, lda, ldb, ldc, trans_b, s);
        default: set_error("pli_gemm: bad dtype %d", dtype); return PLI_EINVAL;
    }
}
