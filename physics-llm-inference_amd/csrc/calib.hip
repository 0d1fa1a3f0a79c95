// Roofline calibration kernels (ch03/roofline.py measured ceilings).
//
// mfma_probe: every wave issues `iters` rounds of four independent bf16
// MFMAs from registers (no memory traffic in the loop), operands a pseudo-
// random bf16 pattern (zeros would let the chip hold a higher clock than any
// real kernel gets: MI355X_MICROARCH.md 'DVFS give-back').  FLOP count =
// waves x iters x 4 x (2*M*N*K of the shape).  Gives the matrix-core rate the
// chip sustains at the clock it holds under that load -- the measured roof
// beside the 2.5166 PF/s datasheet number.
#include "pli_common.h"

namespace pli {
namespace {

__device__ __forceinline__ uint32_t probe_hash(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
// a bf16 pair with exponents in [2^-4, 2^3): finite, random mantissas and signs
__device__ __forceinline__ int probe_pair(uint32_t h) {
    const uint32_t lo = (h & 0x807fu) | ((123u + ((h >> 8) & 7u)) << 7);
    const uint32_t hi = ((h >> 16) & 0x807fu) | ((123u + ((h >> 24) & 7u)) << 7);
    return (int)(lo | (hi << 16));
}

template <int SHAPE>
__global__ __launch_bounds__(256) void mfma_probe(float* __restrict__ out, int iters) {
    const uint32_t seed = probe_hash(blockIdx.x * 256u + threadIdx.x);
    i32x4 a, b;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        a[j] = probe_pair(probe_hash(seed + 2 * j));
        b[j] = probe_pair(probe_hash(seed + 2 * j + 1));
    }
    float s = 0.f;
    if constexpr (SHAPE == 0) {
        f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
        for (int i = 0; i < iters; ++i) {
            c0 = mfma32x32x16<bf16_t>(a, b, c0);
            c1 = mfma32x32x16<bf16_t>(b, a, c1);
            c2 = mfma32x32x16<bf16_t>(a, a, c2);
            c3 = mfma32x32x16<bf16_t>(b, b, c3);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
    } else {
        f32x4 c0 = {}, c1 = {}, c2 = {}, c3 = {};
        for (int i = 0; i < iters; ++i) {
            c0 = mfma16x16x32<bf16_t>(a, b, c0);
            c1 = mfma16x16x32<bf16_t>(b, a, c1);
            c2 = mfma16x16x32<bf16_t>(a, a, c2);
            c3 = mfma16x16x32<bf16_t>(b, b, c3);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
    }
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void hbm_read_probe(const i32x4* __restrict__ src, int64_t n16,
                                                      uint32_t* __restrict__ out) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    uint32_t acc = 0;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        const i32x4 a = __builtin_nontemporal_load(src + i);
        const i32x4 b = __builtin_nontemporal_load(src + i + stride);
        const i32x4 c = __builtin_nontemporal_load(src + i + 2 * stride);
        const i32x4 d = __builtin_nontemporal_load(src + i + 3 * stride);
        acc ^= (uint32_t)(a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w);
        acc ^= (uint32_t)(c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w);
    }
    for (; i < n16; i += stride) {
        const i32x4 a = __builtin_nontemporal_load(src + i);
        acc ^= (uint32_t)(a.x ^ a.y ^ a.z ^ a.w);
    }
    out[(int64_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

// mode 1: block b streams its own contiguous slice of the buffer; each wave
// reads 8 KiB per step (8 x 16-B non-temporal loads per lane in flight,
// consecutive lanes on consecutive 16 B), so every DRAM page is opened by one
// wave at a time.
__global__ __launch_bounds__(256) void hbm_read_probe_chunked(const i32x4* __restrict__ src, int64_t n16,
                                                              uint32_t* __restrict__ out) {
    const int64_t per_block = (n16 + gridDim.x - 1) / gridDim.x;
    const int64_t lo = (int64_t)blockIdx.x * per_block, hi = min(n16, lo + per_block);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t acc = 0;
    int64_t i = lo + wave * 512 + lane;
    for (; i + 7 * 64 < hi; i += 4 * 512) {
        i32x4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(src + i + 64 * u);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc ^= (uint32_t)(v[u].x ^ v[u].y ^ v[u].z ^ v[u].w);
    }
    for (; i < hi; i += 64) {
        const i32x4 a = __builtin_nontemporal_load(src + i);
        acc ^= (uint32_t)(a.x ^ a.y ^ a.z ^ a.w);
    }
    out[(int64_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

}  // namespace
}  // namespace pli

extern "C" int pli_hbm_read_probe(const void* buf, int64_t bytes, uint32_t* out, int blocks, int mode,
                                  void* stream) {
    using namespace pli;
    clear_error();
    PLI_REQUIRE(buf != nullptr && out != nullptr, "pli_hbm_read_probe: null pointer");
    PLI_REQUIRE(aligned16(buf) && bytes > 0 && bytes % 16 == 0 && blocks > 0,
                "pli_hbm_read_probe: need a 16-byte aligned buffer of 16k bytes and blocks > 0");
    PLI_REQUIRE(mode == 0 || mode == 1, "pli_hbm_read_probe: mode %d", mode);
    if (mode == 0)
        hipLaunchKernelGGL(hbm_read_probe, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const i32x4*)buf,
                           bytes / 16, out);
    else
        hipLaunchKernelGGL(hbm_read_probe_chunked, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                           (const i32x4*)buf, bytes / 16, out);
    return launch_status("hbm_read_probe");
}

extern "C" int pli_mfma_probe(float* out, int blocks, int iters, int shape, void* stream) {
    using namespace pli;
    clear_error();
    PLI_REQUIRE(out != nullptr, "pli_mfma_probe: null output");
    PLI_REQUIRE(blocks > 0 && iters > 0 && (shape == 0 || shape == 1),
                "pli_mfma_probe: bad blocks %d / iters %d / shape %d", blocks, iters, shape);
    hipStream_t s = (hipStream_t)stream;
    if (shape == 0) hipLaunchKernelGGL((mfma_probe<0>), dim3(blocks), dim3(256), 0, s, out, iters);
    else hipLaunchKernelGGL((mfma_probe<1>), dim3(blocks), dim3(256), 0, s, out, iters);
    return launch_status("mfma_probe");
}
