// RMSNorm with an optional fused residual add, for gfx950.
//
// Replaces ch02/cached_generation.py:101-109 (RMSNorm.forward: x**2, mean,
// + eps, sqrt, divide, * weight -- six elementwise/reduction launches on the
// torch path) and the residual adds of CachedTransformerBlock.forward
// (:143-145) that feed it: one launch reads x (and the residual branch r),
// writes h = x + r (rounded to the storage type, as the torch add would) and
// y = h / sqrt(mean(h^2) + eps) * weight, statistics in fp32.
//
// One 256-thread workgroup per row; 16-byte loads when n % 8 == 0; the row
// is kept in registers between the sum-of-squares pass and the scaling pass
// (n <= 256 * 8 * RPT), otherwise re-read from L2.
#include <type_traits>

#include "pli_common.h"

namespace pli {
namespace {

template <typename T>
__device__ __forceinline__ float block_sum(float v, float* red) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();  // red may be reused by a previous call
    if (lane == 0) red[wave] = v;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
}

// vector path: n % 8 == 0, 16-byte aligned rows
template <typename T, int RPT>
__global__ __launch_bounds__(256) void rmsnorm_vec(const uint16_t* __restrict__ x,
                                                   const uint16_t* __restrict__ r,
                                                   const uint16_t* __restrict__ w,
                                                   uint16_t* __restrict__ y,
                                                   uint16_t* __restrict__ h, int n, int64_t ldx,
                                                   int64_t ldr, int64_t ldy, int64_t ldh, float eps) {
    __shared__ float red[4];
    const int64_t row = blockIdx.x;
    const int nch = n / 8;
    const uint16_t* xr = x + row * ldx;
    float v[RPT][8];
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
        const int c = threadIdx.x + 256 * i;
        if (c < nch) {
            const i32x4 xv = *reinterpret_cast<const i32x4*>(xr + 8 * c);
            i32x4 rv = {0, 0, 0, 0};
            if (r) rv = *reinterpret_cast<const i32x4*>(r + row * ldr + 8 * c);
            uint32_t hw[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t xw = (uint32_t)xv[j], rw = (uint32_t)rv[j];
                float a0 = elem<T>::to_f32(T{(uint16_t)(xw & 0xffff)});
                float a1 = elem<T>::to_f32(T{(uint16_t)(xw >> 16)});
                if (r) {
                    // round the sum to T: h is what the torch residual add stores
                    a0 = elem<T>::to_f32(elem<T>::from_f32(a0 + elem<T>::to_f32(T{(uint16_t)(rw & 0xffff)})));
                    a1 = elem<T>::to_f32(elem<T>::from_f32(a1 + elem<T>::to_f32(T{(uint16_t)(rw >> 16)})));
                }
                hw[j] = pack2<T>(a0, a1);
                v[i][2 * j] = a0;
                v[i][2 * j + 1] = a1;
                ss = fmaf(a0, a0, fmaf(a1, a1, ss));
            }
            if (h) *reinterpret_cast<i32x4*>(h + row * ldh + 8 * c) =
                i32x4{(int)hw[0], (int)hw[1], (int)hw[2], (int)hw[3]};
        }
    }
    const float inv = 1.f / sqrtf(block_sum<T>(ss, red) / (float)n + eps);
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
        const int c = threadIdx.x + 256 * i;
        if (c < nch) {
            const i32x4 wv = *reinterpret_cast<const i32x4*>(w + 8 * c);
            uint32_t o[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t ww = (uint32_t)wv[j];
                o[j] = pack2<T>(v[i][2 * j] * inv * elem<T>::to_f32(T{(uint16_t)(ww & 0xffff)}),
                                v[i][2 * j + 1] * inv * elem<T>::to_f32(T{(uint16_t)(ww >> 16)}));
            }
            *reinterpret_cast<i32x4*>(y + row * ldy + 8 * c) =
                i32x4{(int)o[0], (int)o[1], (int)o[2], (int)o[3]};
        }
    }
}

// generic path: any n / alignment, 16-bit or fp32 storage
template <typename T>
__global__ __launch_bounds__(256) void rmsnorm_generic(const T* __restrict__ x, const T* __restrict__ r,
                                                       const T* __restrict__ w, T* __restrict__ y,
                                                       T* __restrict__ h, int n, int64_t ldx,
                                                       int64_t ldr, int64_t ldy, int64_t ldh,
                                                       float eps) {
    __shared__ float red[4];
    const int64_t row = blockIdx.x;
    float ss = 0.f;
    for (int i = threadIdx.x; i < n; i += 256) {
        float a = elem<T>::to_f32(x[row * ldx + i]);
        if (r) a = elem<T>::to_f32(elem<T>::from_f32(a + elem<T>::to_f32(r[row * ldr + i])));
        if (h) h[row * ldh + i] = elem<T>::from_f32(a);
        ss = fmaf(a, a, ss);
    }
    const float inv = 1.f / sqrtf(block_sum<T>(ss, red) / (float)n + eps);
    for (int i = threadIdx.x; i < n; i += 256) {
        float a = elem<T>::to_f32(x[row * ldx + i]);
        if (r) a = elem<T>::to_f32(elem<T>::from_f32(a + elem<T>::to_f32(r[row * ldr + i])));
        y[row * ldy + i] = elem<T>::from_f32(a * inv * elem<T>::to_f32(w[i]));
    }
}

template <typename T>
int launch_rmsnorm(const void* x, const void* r, const void* w, void* y, void* h, int64_t rows,
                   int n, int64_t ldx, int64_t ldr, int64_t ldy, int64_t ldh, float eps,
                   hipStream_t s) {
    const dim3 grid((unsigned)rows), block(256);
    const bool vec = !std::is_same_v<T, float> && n % 8 == 0 && ldx % 8 == 0 && ldy % 8 == 0 &&
                     (!r || ldr % 8 == 0) && (!h || ldh % 8 == 0) && aligned16(x) && aligned16(y) &&
                     aligned16(w) && (!r || aligned16(r)) && (!h || aligned16(h));
    if constexpr (!std::is_same_v<T, float>) {
        if (vec && n <= 256 * 8 * 4) {
            const auto* X = (const uint16_t*)x;
            const auto* R = (const uint16_t*)r;
            const auto* W = (const uint16_t*)w;
            auto* Y = (uint16_t*)y;
            auto* Hh = (uint16_t*)h;
            if (n <= 256 * 8)
                hipLaunchKernelGGL((rmsnorm_vec<T, 1>), grid, block, 0, s, X, R, W, Y, Hh, n, ldx, ldr, ldy, ldh, eps);
            else if (n <= 256 * 8 * 2)
                hipLaunchKernelGGL((rmsnorm_vec<T, 2>), grid, block, 0, s, X, R, W, Y, Hh, n, ldx, ldr, ldy, ldh, eps);
            else
                hipLaunchKernelGGL((rmsnorm_vec<T, 4>), grid, block, 0, s, X, R, W, Y, Hh, n, ldx, ldr, ldy, ldh, eps);
            return launch_status("rmsnorm_vec");
        }
    }
    hipLaunchKernelGGL((rmsnorm_generic<T>), grid, block, 0, s, (const T*)x, (const T*)r,
                       (const T*)w, (T*)y, (T*)h, n, ldx, ldr, ldy, ldh, eps);
    return launch_status("rmsnorm_generic");
}

}  // namespace
}  // namespace pli

extern "C" int pli_rmsnorm(const void* x, const void* residual, const void* weight, void* y,
                           void* h_out, int64_t rows, int n, int64_t ldx, int64_t ldr, int64_t ldy,
                           int64_t ldh, float eps, int dtype, void* stream) {
    using namespace pli;
    clear_error();
    PLI_REQUIRE(rows >= 0 && n > 0 && rows < (1ll << 31), "pli_rmsnorm: bad shape rows=%lld n=%d",
                (long long)rows, n);
    PLI_REQUIRE(ldx >= n && ldy >= n && (!residual || ldr >= n) && (!h_out || ldh >= n),
                "pli_rmsnorm: leading dimension too small");
    PLI_REQUIRE(eps >= 0.f, "pli_rmsnorm: negative eps");
    if (rows == 0) return PLI_OK;  // (empty operands may be NULL, pli.h)
    PLI_REQUIRE(x && weight && y, "pli_rmsnorm: null pointer");
    hipStream_t s = (hipStream_t)stream;
    switch (dtype) {
        case PLI_BF16: return launch_rmsnorm<bf16_t>(x, residual, weight, y, h_out, rows, n, ldx, ldr, ldy, ldh, eps, s);
        case PLI_F16: return launch_rmsnorm<f16_t>(x, residual, weight, y, h_out, rows, n, ldx, ldr, ldy, ldh, eps, s);
        case PLI_F32: return launch_rmsnorm<float>(x, residual, weight, y, h_out, rows, n, ldx, ldr, ldy, ldh, eps, s);
        default: set_error("pli_rmsnorm: bad dtype %d", dtype); return PLI_EINVAL;
    }
}
