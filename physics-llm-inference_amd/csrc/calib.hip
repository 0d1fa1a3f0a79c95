// Roofline calibration kernels (ch03/roofline.py measured ceilings).
//
// mfma_probe: ONE wave per SIMD (256-thread workgroups holding 96 KiB of LDS,
// so one per CU), each wave issuing `iters` rounds of back-to-back bf16 MFMAs
// from registers into independent accumulators, on pseudo-random operands
// (zeros would let the chip hold a higher clock than any real kernel gets:
// MI355X_MICROARCH.md 'DVFS give-back').  Both shapes compute the same output
// tile per wave (a 64x64 f32 block: four 32x32 or sixteen 16x16 accumulators)
// and the same FLOPs per round (262,144: 8 x 32x32x16 or 16 x 16x16x32), so
// the two rates compare at equal work -- the guide measures the 16x16x32
// loop at about 1.15x the FLOP/s of the 32x32x16 one on random data (item 7),
// a clock effect.  Every wave stamps s_memtime / s_memrealtime around its
// loop (item 6): the in-kernel clock is dtime / drealtime x 100 MHz.
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
__global__ __launch_bounds__(256, 1) void mfma_probe(float* __restrict__ out,
                                                     unsigned long long* __restrict__ clocks, int iters) {
    const uint32_t seed = probe_hash(blockIdx.x * 256u + threadIdx.x);
    i32x4 a, b;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        a[j] = probe_pair(probe_hash(seed + 2 * j));
        b[j] = probe_pair(probe_hash(seed + 2 * j + 1));
    }
    float s = 0.f;
    unsigned long long t0, r0, t1, r1;
    asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0), "=s"(r0)::"memory");
    // the MFMAs are asm statements with the accumulators pinned in VGPRs:
    // compiled from the builtins, hipcc rotates the 16x16x32 accumulators
    // through AGPR copies inside the loop (v_accvgpr_mov per MFMA), which is
    // what made the earlier probe read the 16x16x32 rate low.  An accumulator
    // is re-used 8 (16) MFMAs after its last write, far past the XDL latency;
    // the s_nops after the loop cover the MFMA -> VALU read.
    if constexpr (SHAPE == 0) {
        f32x16 c[4] = {};
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const i32x4 x = (j & 1) ? b : a, y = ((j >> 1) ^ (j >> 2)) & 1 ? b : a;
                asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c[j & 3]) : "v"(x), "v"(y));
            }
        }
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]));
        asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1), "=s"(r1)::"memory");
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) s += c[j][r];
    } else {
        f32x4 c[16] = {};
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const i32x4 x = (j & 1) ? b : a, y = (j & 2) ? b : a;
                asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c[j]) : "v"(x), "v"(y));
            }
        }
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]),
                     "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]), "+v"(c[8]), "+v"(c[9]), "+v"(c[10]),
                     "+v"(c[11]), "+v"(c[12]), "+v"(c[13]), "+v"(c[14]), "+v"(c[15]));
        asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1), "=s"(r1)::"memory");
#pragma unroll
        for (int j = 0; j < 16; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) s += c[j][r];
    }
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (clocks != nullptr && (threadIdx.x & 63) == 0) {
        const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
        clocks[2 * w] = t1 - t0;
        clocks[2 * w + 1] = r1 - r0;
    }
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

extern "C" int pli_mfma_probe(float* out, uint64_t* clocks, int blocks, int iters, int shape, void* stream) {
    using namespace pli;
    clear_error();
    PLI_REQUIRE(out != nullptr, "pli_mfma_probe: null output");
    PLI_REQUIRE(blocks > 0 && iters > 0 && (shape == 0 || shape == 1),
                "pli_mfma_probe: bad blocks %d / iters %d / shape %d", blocks, iters, shape);
    hipStream_t s = (hipStream_t)stream;
    // 96 KiB of (unused) LDS per workgroup: one workgroup per CU, so one wave per SIMD
    constexpr size_t kLds = 96 * 1024;
    auto* ck = reinterpret_cast<unsigned long long*>(clocks);
    if (shape == 0) hipLaunchKernelGGL((mfma_probe<0>), dim3(blocks), dim3(256), kLds, s, out, ck, iters);
    else hipLaunchKernelGGL((mfma_probe<1>), dim3(blocks), dim3(256), kLds, s, out, ck, iters);
    return launch_status("mfma_probe");
}
