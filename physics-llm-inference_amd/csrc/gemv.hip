// Decode GEMV y = W x for gfx950 (MI355X): the torch.mv of
// ch03/gemv_benchmark.py:38.  HBM-bound (AI ~1 FLOP/B): no MFMA, no LDS.
//
// Each wave owns ROWS consecutive rows (default: 1 row per wave, 2-wave blocks;
// variants A/B-measured in tools/tune.py under HIP-graph timing).  Lane l streams the 16-byte chunks
// l, l+64, ... of every row with global_load_dwordx4 (non-temporal: W is read
// exactly once per call), all ROWS x CPL loads issued before the first use so
// a CU keeps ROWS*CPL KiB per wave in flight; the x chunks are loaded once per
// k-step and reused for the ROWS rows.  fp32 accumulate, one 64-lane
// shuffle reduction per row, output rounded once to the output dtype.
#include "pli_common.h"

namespace pli {
namespace {

template <typename T>
__device__ __forceinline__ void dot_chunk(const i32x4& w, const i32x4& x, float& acc);

template <>
__device__ __forceinline__ void dot_chunk<bf16_t>(const i32x4& w, const i32x4& x, float& acc) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t a = (uint32_t)w[i], b = (uint32_t)x[i];
        acc = fmaf(__uint_as_float(a << 16), __uint_as_float(b << 16), acc);
        acc = fmaf(__uint_as_float(a & 0xffff0000u), __uint_as_float(b & 0xffff0000u), acc);
    }
}
template <>
__device__ __forceinline__ void dot_chunk<f16_t>(const i32x4& w, const i32x4& x, float& acc) {
    typedef __attribute__((ext_vector_type(2))) _Float16 h2;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        // copy the lanes out first: __builtin_bit_cast of an ext-vector
        // element lvalue reads element 0 for every i (hipcc 7.2)
        const int wi = w[i], xi = x[i];
        const h2 a = __builtin_bit_cast(h2, wi), b = __builtin_bit_cast(h2, xi);
        acc = fmaf((float)a.x, (float)b.x, acc);
        acc = fmaf((float)a.y, (float)b.y, acc);
    }
}
template <>
__device__ __forceinline__ void dot_chunk<float>(const i32x4& w, const i32x4& x, float& acc) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc = fmaf(__int_as_float(w[i]), __int_as_float(x[i]), acc);
}

// EXACT: nchunks is a multiple of 64 * CPL, so no chunk index is clamped or
// predicated (4096 x 4096 bf16: 6.97 vs 7.42 us per launch in a graph,
// tools/gemv_stamps.py k0 vs the clamped kernel, profiles/r02/gemv/)
template <typename T, int ROWS, int CPL, bool NTL, int WPB = 4, bool EXACT = false>
__global__ __launch_bounds__(WPB * 64) void gemv_vec(const char* __restrict__ w,
                                                     const char* __restrict__ x, T* __restrict__ y,
                                                     int M, int nchunks, int64_t ldw_bytes) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int row0 = (blockIdx.x * WPB + wave) * ROWS;
    if (row0 >= M) return;
    float acc[ROWS];
#pragma unroll
    for (int r = 0; r < ROWS; ++r) acc[r] = 0.f;
    const char* wrow[ROWS];
#pragma unroll
    for (int r = 0; r < ROWS; ++r) wrow[r] = w + (int64_t)min(row0 + r, M - 1) * ldw_bytes;

    for (int c0 = 0; c0 < nchunks; c0 += 64 * CPL) {
        i32x4 xv[CPL], wv[ROWS][CPL];
#pragma unroll
        for (int u = 0; u < CPL; ++u) {
            const int cc = EXACT ? c0 + lane + 64 * u : min(c0 + lane + 64 * u, nchunks - 1);
            xv[u] = *reinterpret_cast<const i32x4*>(x + (int64_t)cc * 16);
#pragma unroll
            for (int r = 0; r < ROWS; ++r)
                wv[r][u] = NTL ? __builtin_nontemporal_load(
                                     reinterpret_cast<const i32x4*>(wrow[r] + (int64_t)cc * 16))
                               : *reinterpret_cast<const i32x4*>(wrow[r] + (int64_t)cc * 16);
        }
#pragma unroll
        for (int u = 0; u < CPL; ++u) {
            if (EXACT || c0 + lane + 64 * u < nchunks) {
#pragma unroll
                for (int r = 0; r < ROWS; ++r) dot_chunk<T>(wv[r][u], xv[u], acc[r]);
            }
        }
    }
#pragma unroll
    for (int r = 0; r < ROWS; ++r) acc[r] = wave_sum(acc[r]);
    if (lane < ROWS && row0 + lane < M) {
        float out = acc[0];
#pragma unroll
        for (int r = 1; r < ROWS; ++r) out = (lane == r) ? acc[r] : out;
        y[row0 + lane] = elem<T>::from_f32(out);
    }
}

// Scalar fallback for ragged K / unaligned operands: one wave per row.
template <typename T>
__global__ __launch_bounds__(256) void gemv_scalar(const T* __restrict__ w, const T* __restrict__ x,
                                                   T* __restrict__ y, int M, int K, int64_t ldw) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    float acc = 0.f;
    for (int kk = lane; kk < K; kk += 64)
        acc = fmaf(elem<T>::to_f32(w[(int64_t)row * ldw + kk]), elem<T>::to_f32(x[kk]), acc);
    acc = wave_sum(acc);
    if (lane == 0) y[row] = elem<T>::from_f32(acc);
}

// Variants (A/B via pli_gemv_variant): rows per wave x 16-B chunks per lane
// per k-step x non-temporal W loads.
//   0: 2x8 nt  1: 4x8 nt  2: 1x8 nt  3: 2x8 plain  4: 4x4 nt  5: 8x4 nt
//   6: 2x8 nt, 1-wave blocks   7: 2x8 nt, 8-wave blocks   8: 1x8 nt, 2-wave blocks
//   9: 1x4 nt, 2-wave blocks  10: 2x4 nt, 4-wave blocks  11: 1x4 nt, 4-wave blocks
//  12: 1x8 nt, 1-wave blocks  13: 1x8 nt, 4-wave blocks  14: 1x8 plain, 2-wave blocks
//  15: 1x2 nt, 2-wave blocks  16: 2x2 nt, 4-wave blocks
// Default: 8 (1 row per wave, 2-wave blocks, 8 chunks per lane).  Short rows
// leave lanes idle at 8 chunks per lane, so (median of 5 interleaved rounds,
// HBM-resident W, tools/gemv_vs_skinny.py, profiles/r01/gemm/gemv_*.log):
//  * <= 128 16-byte chunks per row (K <= 1024 bf16): variant 16 (2 rows x 2
//    chunks per lane): 32000x1024 4.58 -> 5.69 TB/s, 16384x1024 2.62 -> 4.71,
//    8192x1024 2.12 -> 2.66, equal at 4096x1024;
//  * <= 256 chunks and M >= 16384 (the 32000 x 2048 LM head): variant 9 (4
//    chunks per lane): 32000x2048 5.03 -> 6.36 TB/s, 128256x2048 5.51 -> 7.09.
constexpr int kDefaultGemvVariant = 8;
constexpr int kVeryShortRowVariant = 16;
constexpr int kVeryShortRowChunks = 128;
constexpr int kTallShortGemvVariant = 9;
constexpr int kTallGemvRows = 16384;
constexpr int kShortRowChunks = 256;

template <typename T, int ROWS, int CPL, bool NTL, int WPB = 4>
int launch_vec(const void* w, const void* x, void* y, int m, int nchunks, int64_t ldw_b,
               hipStream_t s) {
    if (nchunks % (64 * CPL) == 0)
        hipLaunchKernelGGL((gemv_vec<T, ROWS, CPL, NTL, WPB, true>), dim3(cdiv(m, WPB * ROWS)),
                           dim3(WPB * 64), 0, s, (const char*)w, (const char*)x, (T*)y, m, nchunks,
                           ldw_b);
    else
        hipLaunchKernelGGL((gemv_vec<T, ROWS, CPL, NTL, WPB, false>), dim3(cdiv(m, WPB * ROWS)),
                           dim3(WPB * 64), 0, s, (const char*)w, (const char*)x, (T*)y, m, nchunks,
                           ldw_b);
    return launch_status("gemv_vec");
}

template <typename T>
int launch(const void* w, const void* x, void* y, int m, int k, int64_t ldw, hipStream_t s,
           int variant) {
    constexpr int EPC = 16 / elem<T>::bytes;  // elements per 16-byte chunk
    const bool vec = (k % EPC == 0) && (ldw % EPC == 0) &&
                     ((reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(x)) & 15) == 0;
    if (!vec) {
        hipLaunchKernelGGL(gemv_scalar<T>, dim3(cdiv(m, 4)), dim3(256), 0, s, (const T*)w,
                           (const T*)x, (T*)y, m, k, ldw);
        return launch_status("gemv_scalar");
    }
    const int nchunks = k / EPC;
    const int64_t ldw_b = ldw * elem<T>::bytes;
    if (variant < 0)
        variant = nchunks <= kVeryShortRowChunks                        ? kVeryShortRowVariant
                  : (m >= kTallGemvRows && nchunks <= kShortRowChunks) ? kTallShortGemvVariant
                                                                       : kDefaultGemvVariant;
    switch (variant) {
        case 0: return launch_vec<T, 2, 8, true>(w, x, y, m, nchunks, ldw_b, s);
        case 1: return launch_vec<T, 4, 8, true>(w, x, y, m, nchunks, ldw_b, s);
        case 2: return launch_vec<T, 1, 8, true>(w, x, y, m, nchunks, ldw_b, s);
        case 3: return launch_vec<T, 2, 8, false>(w, x, y, m, nchunks, ldw_b, s);
        case 4: return launch_vec<T, 4, 4, true>(w, x, y, m, nchunks, ldw_b, s);
        case 5: return launch_vec<T, 8, 4, true>(w, x, y, m, nchunks, ldw_b, s);
        case 6: return launch_vec<T, 2, 8, true, 1>(w, x, y, m, nchunks, ldw_b, s);
        case 7: return launch_vec<T, 2, 8, true, 8>(w, x, y, m, nchunks, ldw_b, s);
        case 8: return launch_vec<T, 1, 8, true, 2>(w, x, y, m, nchunks, ldw_b, s);
        case 9: return launch_vec<T, 1, 4, true, 2>(w, x, y, m, nchunks, ldw_b, s);
        case 10: return launch_vec<T, 2, 4, true, 4>(w, x, y, m, nchunks, ldw_b, s);
        case 11: return launch_vec<T, 1, 4, true, 4>(w, x, y, m, nchunks, ldw_b, s);
        case 12: return launch_vec<T, 1, 8, true, 1>(w, x, y, m, nchunks, ldw_b, s);
        case 13: return launch_vec<T, 1, 8, true, 4>(w, x, y, m, nchunks, ldw_b, s);
        case 14: return launch_vec<T, 1, 8, false, 2>(w, x, y, m, nchunks, ldw_b, s);
        case 15: return launch_vec<T, 1, 2, true, 2>(w, x, y, m, nchunks, ldw_b, s);
        case 16: return launch_vec<T, 2, 2, true, 4>(w, x, y, m, nchunks, ldw_b, s);
        default: set_error("pli_gemv: unknown variant %d", variant); return PLI_EINVAL;
    }
}

}  // namespace
}  // namespace pli

// Not in pli.h: pli_gemv with an explicit kernel variant (tuning / A-B runs).
extern "C" int pli_gemv_variant(const void* w, const void* x, void* y, int m, int k, int64_t ldw,
                                int dtype, void* stream, int variant) {
    using namespace pli;
    clear_error();
    PLI_REQUIRE(m >= 0 && k >= 0 && ldw >= k, "pli_gemv: bad shape m=%d k=%d ldw=%lld", m, k,
                (long long)ldw);
    PLI_REQUIRE(dtype == PLI_F32 || dtype == PLI_F16 || dtype == PLI_BF16, "pli_gemv: bad dtype %d", dtype);
    // empty operands may be NULL (pli.h): no rows -> nothing to do; K == 0 ->
    // y = 0 (torch.mv of an m x 0 matrix), W and x not read
    if (m == 0) return PLI_OK;
    PLI_REQUIRE(y && (k == 0 || (w && x)), "pli_gemv: null pointer");
    hipStream_t s = (hipStream_t)stream;
    if (k == 0) {
        const hipError_t e = hipMemsetAsync(y, 0, (size_t)m * (dtype == PLI_F32 ? 4 : 2), s);
        if (e != hipSuccess) {
            set_error("pli_gemv: hipMemsetAsync: %s", hipGetErrorString(e));
            return (int)e;
        }
        return PLI_OK;
    }
    switch (dtype) {
        case PLI_F32: return launch<float>(w, x, y, m, k, ldw, s, variant);
        case PLI_F16: return launch<f16_t>(w, x, y, m, k, ldw, s, variant);
        case PLI_BF16: return launch<bf16_t>(w, x, y, m, k, ldw, s, variant);
        default: set_error("pli_gemv: bad dtype %d", dtype); return PLI_EINVAL;
    }
}

extern "C" int pli_gemv(const void* w, const void* x, void* y, int m, int k, int64_t ldw,
                        int dtype, void* stream) {
    return pli_gemv_variant(w, x, y, m, k, ldw, dtype, stream, -1);
}
