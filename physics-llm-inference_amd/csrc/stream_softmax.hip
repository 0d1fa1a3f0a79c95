// HBM calibration (ch05/coalescing.cu) and row-softmax (ch06/online_softmax.py)
// kernels for gfx950.
#include <cmath>

#include "pli_common.h"

namespace pli {
namespace {

// out[i] = 2 * in[i]: coalesced_read of ch05/coalescing.cu:7-12, widened to
// 16-byte vector loads/stores with a grid-stride loop (grid capped at
// 8 blocks/CU), non-temporal on both sides (each byte touched once).
__global__ __launch_bounds__(256) void scale_copy_vec(const f32x4* __restrict__ in,
                                                      f32x4* __restrict__ out, int64_t n4) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        const f32x4 x = __builtin_nontemporal_load(in + i);
        __builtin_nontemporal_store(x * 2.f, out + i);
    }
}

// out[i] = 2 * in[i * stride]: strided_read of ch05/coalescing.cu:14-20.
__global__ __launch_bounds__(256) void scale_copy_strided(const float* __restrict__ in,
                                                          float* __restrict__ out, int64_t n,
                                                          int stride) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = in[i * stride] * 2.f;
}

// One wave per row: pass 1 keeps a per-lane online (m, d) pair -- the
// recurrence of ch06/online_softmax.py:13-25 -- merged across the wave with
// (m, d) (+) (m', d') = (max, d e^{m-max} + d' e^{m'-max}); pass 2 writes
// e^{x-m}/d.  fp32 statistics.
template <typename T>
__global__ __launch_bounds__(256) void softmax_rows(const T* __restrict__ x, T* __restrict__ y,
                                                    int64_t rows, int n) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const T* xr = x + row * n;
    float m = -INFINITY, d = 0.f;
    for (int i = lane; i < n; i += 64) {
        const float v = elem<T>::to_f32(xr[i]);
        const float mn = fmaxf(m, v);
        d = (mn == -INFINITY ? 0.f : d * expf(m - mn) + expf(v - mn));
        m = mn;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float m2 = __shfl_xor(m, o, 64), d2 = __shfl_xor(d, o, 64);
        const float mn = fmaxf(m, m2);
        d = (mn == -INFINITY) ? 0.f : d * expf(m - mn) + d2 * expf(m2 - mn);
        m = mn;
    }
    const float inv = 1.f / d;
    T* yr = y + row * n;
    for (int i = lane; i < n; i += 64) yr[i] = elem<T>::from_f32(expf(elem<T>::to_f32(xr[i]) - m) * inv);
}

// One wave per row: (m, d) as above, then o = sum_i e^{x_i - m} v_i / d with
// lanes over dv; d is returned relative to the final max, like the
// reference's running denominator (ch06/online_softmax.py:28-53).
template <typename T>
__global__ __launch_bounds__(256) void softmax_with_output(const T* __restrict__ x,
                                                           const T* __restrict__ v,
                                                           T* __restrict__ o, T* __restrict__ dout,
                                                           int64_t rows, int n, int dv) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const T* xr = x + row * n;
    float m = -INFINITY;
    for (int i = lane; i < n; i += 64) m = fmaxf(m, elem<T>::to_f32(xr[i]));
    m = wave_max(m);
    float d = 0.f;
    for (int i = lane; i < n; i += 64) d += expf(elem<T>::to_f32(xr[i]) - m);
    d = wave_sum(d);
    const float inv = 1.f / d;
    const T* vr = v + row * (int64_t)n * dv;
    for (int c = lane; c < dv; c += 64) {
        float acc = 0.f;
        for (int i = 0; i < n; ++i)
            acc = fmaf(expf(elem<T>::to_f32(xr[i]) - m), elem<T>::to_f32(vr[(int64_t)i * dv + c]), acc);
        o[row * dv + c] = elem<T>::from_f32(acc * inv);
    }
    if (lane == 0) dout[row] = elem<T>::from_f32(d);
}

}  // namespace
}  // namespace pli

extern "C" int pli_scale_copy(const float* in, float* out, int64_t n_out, int stride,
                              void* stream) {
    using namespace pli;
    clear_error();
    PLI_REQUIRE(n_out >= 0 && stride >= 1, "pli_scale_copy: bad n=%lld stride=%d",
                (long long)n_out, stride);
    if (n_out == 0) return PLI_OK;  // (empty operands may be NULL, pli.h)
    PLI_REQUIRE(in && out, "pli_scale_copy: null pointer");
    hipStream_t s = (hipStream_t)stream;
    const bool vec = stride == 1 && n_out % 4 == 0 &&
                     (((uintptr_t)in | (uintptr_t)out) & 15) == 0;
    if (vec) {
        const int64_t n4 = n_out / 4;
        const int64_t want = (n4 + 255) / 256;
        const int grid = (int)(want < 2048 ? want : 2048);
        hipLaunchKernelGGL(scale_copy_vec, dim3(grid), dim3(256), 0, s, (const f32x4*)in,
                           (f32x4*)out, n4);
        return launch_status("scale_copy_vec");
    }
    const int64_t grid = (n_out + 255) / 256;
    PLI_REQUIRE(grid < (1ll << 31), "pli_scale_copy: too large");
    hipLaunchKernelGGL(scale_copy_strided, dim3((unsigned)grid), dim3(256), 0, s, in, out, n_out,
                       stride);
    return launch_status("scale_copy_strided");
}

extern "C" int pli_softmax_rows(const void* x, void* y, int64_t rows, int n, int dtype,
                                void* stream) {
    using namespace pli;
    clear_error();
    PLI_REQUIRE(rows >= 0 && n >= 0, "pli_softmax_rows: bad shape rows=%lld n=%d",
                (long long)rows, n);
    if (rows == 0 || n == 0) return PLI_OK;  // (empty operands may be NULL, pli.h)
    PLI_REQUIRE(x && y, "pli_softmax_rows: null pointer");
    const int64_t grid = (rows + 3) / 4;
    PLI_REQUIRE(grid < (1ll << 31), "pli_softmax_rows: too many rows");
    hipStream_t s = (hipStream_t)stream;
    switch (dtype) {
        case PLI_F32:
            hipLaunchKernelGGL(softmax_rows<float>, dim3((unsigned)grid), dim3(256), 0, s,
                               (const float*)x, (float*)y, rows, n);
            break;
        case PLI_F16:
            hipLaunchKernelGGL(softmax_rows<f16_t>, dim3((unsigned)grid), dim3(256), 0, s,
                               (const f16_t*)x, (f16_t*)y, rows, n);
            break;
        case PLI_BF16:
            hipLaunchKernelGGL(softmax_rows<bf16_t>, dim3((unsigned)grid), dim3(256), 0, s,
                               (const bf16_t*)x, (bf16_t*)y, rows, n);
            break;
        default: set_error("pli_softmax_rows: bad dtype %d", dtype); return PLI_EINVAL;
    }
    return launch_status("softmax_rows");
}

extern "C" int pli_online_softmax_with_output(const void* x, const void* v, void* o, void* d,
                                              int64_t rows, int n, int dv, int dtype,
                                              void* stream) {
    using namespace pli;
    clear_error();
    PLI_REQUIRE(rows >= 0 && n > 0 && dv > 0, "pli_online_softmax_with_output: bad shape");
    if (rows == 0) return PLI_OK;  // (empty operands may be NULL, pli.h)
    PLI_REQUIRE(x && v && o && d, "pli_online_softmax_with_output: null pointer");
    const int64_t grid = (rows + 3) / 4;
    PLI_REQUIRE(grid < (1ll << 31), "pli_online_softmax_with_output: too many rows");
    hipStream_t s = (hipStream_t)stream;
    switch (dtype) {
        case PLI_F32:
            hipLaunchKernelGGL(softmax_with_output<float>, dim3((unsigned)grid), dim3(256), 0, s,
                               (const float*)x, (const float*)v, (float*)o, (float*)d, rows, n, dv);
            break;
        case PLI_F16:
            hipLaunchKernelGGL(softmax_with_output<f16_t>, dim3((unsigned)grid), dim3(256), 0, s,
                               (const f16_t*)x, (const f16_t*)v, (f16_t*)o, (f16_t*)d, rows, n, dv);
            break;
        case PLI_BF16:
            hipLaunchKernelGGL(softmax_with_output<bf16_t>, dim3((unsigned)grid), dim3(256), 0, s,
                               (const bf16_t*)x, (const bf16_t*)v, (bf16_t*)o, (bf16_t*)d, rows, n,
                               dv);
            break;
        default:
            set_error("pli_online_softmax_with_output: bad dtype %d", dtype);
            return PLI_EINVAL;
    }
    return launch_status("softmax_with_output");
}
