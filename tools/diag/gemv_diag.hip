// Diagnostic GEMV kernels (never the product library; tools/build_diag.sh ->
// tools/libpli_diag.so, driven by tools/gemv_stamps.py on the GPU box).
//
// Where do the 7.6-7.9 us of a 4096 x 4096 bf16 GEMV go?  Each wave records
// s_memrealtime (100 MHz, one clock for the whole chip) at entry, when its W
// loads have returned, and at exit, plus its XCC id, so the host can split a
// launch into dispatch ramp, first-byte latency, streaming and tail.
//
//   kind 0: the product shape (gemv.hip variant 8: one row per wave, 8 x 16-B
//           chunks per lane, 2-wave blocks, non-temporal loads)
//   kind 1: persistent: `grid` blocks x WPB waves stride over the rows, the
//           next row's loads issued before the current row is reduced
#include "pli_common.h"

namespace pli {
namespace {

__device__ __forceinline__ uint64_t rt_now() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ int xcc_id() {
    // HW_REG_XCC_ID (gfx940+): bits [3:0] = XCC
    return __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11)) & 15;
}

__device__ __forceinline__ void dot8(const i32x4& w, const i32x4& x, float& acc) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t a = (uint32_t)w[i], b = (uint32_t)x[i];
        acc = fmaf(__uint_as_float(a << 16), __uint_as_float(b << 16), acc);
        acc = fmaf(__uint_as_float(a & 0xffff0000u), __uint_as_float(b & 0xffff0000u), acc);
    }
}

// K = 4096 bf16 = 512 chunks = 8 per lane: one row is one load batch.
template <bool STAMP>
__global__ __launch_bounds__(128) void gemv_rowwave(const char* __restrict__ w, const char* __restrict__ x,
                                                    bf16_t* __restrict__ y, int M, int64_t ldw,
                                                    uint64_t* __restrict__ st) {
    uint64_t t0 = 0, t1 = 0;
    if constexpr (STAMP) t0 = rt_now();
    const int lane = threadIdx.x & 63, gw = blockIdx.x * 2 + (threadIdx.x >> 6);
    if (gw >= M) return;
    const char* wr = w + (int64_t)gw * ldw;
    i32x4 xv[8], wv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        const int c = lane + 64 * u;
        xv[u] = *reinterpret_cast<const i32x4*>(x + (int64_t)c * 16);
        wv[u] = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(wr + (int64_t)c * 16));
    }
    if constexpr (STAMP) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        t1 = rt_now();
    }
    float acc = 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u) dot8(wv[u], xv[u], acc);
    acc = wave_sum(acc);
    if (lane == 0) y[gw] = elem<bf16_t>::from_f32(acc);
    if constexpr (STAMP) {
        const uint64_t t2 = rt_now();
        if (lane == 0) {
            st[4 * gw + 0] = t0;
            st[4 * gw + 1] = t1;
            st[4 * gw + 2] = t2;
            st[4 * gw + 3] = (uint64_t)xcc_id();
        }
    }
}

// persistent: wave gw handles rows gw, gw + nw, ... (double-buffered)
template <bool STAMP, int WPB>
__global__ __launch_bounds__(WPB * 64) void gemv_persist(const char* __restrict__ w, const char* __restrict__ x,
                                                         bf16_t* __restrict__ y, int M, int64_t ldw,
                                                         uint64_t* __restrict__ st) {
    uint64_t t0 = 0, t1 = 0;
    if constexpr (STAMP) t0 = rt_now();
    const int lane = threadIdx.x & 63, gw = blockIdx.x * WPB + (threadIdx.x >> 6);
    const int nw = gridDim.x * WPB;
    i32x4 xv[8], wa[8], wb[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) xv[u] = *reinterpret_cast<const i32x4*>(x + (int64_t)(lane + 64 * u) * 16);
    int row = gw;
    auto ld = [&](i32x4* dst, int r) __attribute__((always_inline)) {
        const char* wr = w + (int64_t)min(r, M - 1) * ldw;
#pragma unroll
        for (int u = 0; u < 8; ++u)
            dst[u] = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(wr + (int64_t)(lane + 64 * u) * 16));
    };
    auto fin = [&](const i32x4* src, int r) __attribute__((always_inline)) {
        float acc = 0.f;
#pragma unroll
        for (int u = 0; u < 8; ++u) dot8(src[u], xv[u], acc);
        acc = wave_sum(acc);
        if (lane == 0 && r < M) y[r] = elem<bf16_t>::from_f32(acc);
    };
    if (row < M) ld(wa, row);
    bool first = true;
    while (row < M) {
        const int nxt = row + nw;
        if (nxt < M) ld(wb, nxt);
        if constexpr (STAMP) {
            if (first) {
                asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                t1 = rt_now();
                first = false;
            }
        }
        fin(wa, row);
        row = nxt;
        if (row >= M) break;
        const int nx2 = row + nw;
        if (nx2 < M) ld(wa, nx2);
        fin(wb, row);
        row = nx2;
    }
    if constexpr (STAMP) {
        const uint64_t t2 = rt_now();
        if (lane == 0) {
            st[4 * gw + 0] = t0;
            st[4 * gw + 1] = t1;
            st[4 * gw + 2] = t2;
            st[4 * gw + 3] = (uint64_t)xcc_id();
        }
    }
}

// contiguous: wave gw handles rows gw*R .. gw*R + R - 1 (R = ceil(M / waves)),
// the next row's loads issued before the current row is reduced
template <bool STAMP, int WPB>
__global__ __launch_bounds__(WPB * 64) void gemv_contig(const char* __restrict__ w, const char* __restrict__ x,
                                                        bf16_t* __restrict__ y, int M, int64_t ldw,
                                                        uint64_t* __restrict__ st) {
    uint64_t t0 = 0, t1 = 0;
    if constexpr (STAMP) t0 = rt_now();
    const int lane = threadIdx.x & 63, gw = blockIdx.x * WPB + (threadIdx.x >> 6);
    const int nw = gridDim.x * WPB;
    const int R = (M + nw - 1) / nw;
    const int r0 = gw * R, r1 = min(M, r0 + R);
    i32x4 xv[8], wa[8], wb[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) xv[u] = *reinterpret_cast<const i32x4*>(x + (int64_t)(lane + 64 * u) * 16);
    auto ld = [&](i32x4* dst, int r) __attribute__((always_inline)) {
        const char* wr = w + (int64_t)min(r, M - 1) * ldw;
#pragma unroll
        for (int u = 0; u < 8; ++u)
            dst[u] = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(wr + (int64_t)(lane + 64 * u) * 16));
    };
    auto fin = [&](const i32x4* src, int r) __attribute__((always_inline)) {
        float acc = 0.f;
#pragma unroll
        for (int u = 0; u < 8; ++u) dot8(src[u], xv[u], acc);
        acc = wave_sum(acc);
        if (lane == 0 && r < M) y[r] = elem<bf16_t>::from_f32(acc);
    };
    int row = r0;
    if (row < r1) ld(wa, row);
    bool first = true;
    while (row < r1) {
        if (row + 1 < r1) ld(wb, row + 1);
        if constexpr (STAMP) {
            if (first) {
                asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                t1 = rt_now();
                first = false;
            }
        }
        fin(wa, row);
        if (++row >= r1) break;
        if (row + 1 < r1) ld(wa, row + 1);
        fin(wb, row);
        ++row;
    }
    if constexpr (STAMP) {
        const uint64_t t2 = rt_now();
        if (lane == 0) {
            st[4 * gw + 0] = t0;
            st[4 * gw + 1] = t1;
            st[4 * gw + 2] = t2;
            st[4 * gw + 3] = (uint64_t)xcc_id();
        }
    }
}

}  // namespace
}  // namespace pli

// kind 0: row-per-wave (product shape), 1: persistent 4-wave blocks, 2:
// persistent 8-wave blocks, 3: persistent 2-wave blocks, 4 / 5: contiguous
// row ranges per wave, 4- / 2-wave blocks.  stamps: null or
// 4 x u64 per wave (row-per-wave: M waves; persistent: grid * WPB waves).
// K must be 4096 (512 chunks), operands 16-byte aligned.
extern "C" int pli_diag_gemv(int kind, const void* w, const void* x, void* y, int m, int k, int64_t ldw,
                             int grid, uint64_t* stamps, void* stream) {
    using namespace pli;
    if (k != 4096 || ldw % 8 || m <= 0 || (kind != 0 && grid <= 0)) return PLI_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const char* wc = (const char*)w;
    const char* xc = (const char*)x;
    bf16_t* yb = (bf16_t*)y;
    const int64_t ldb = ldw * 2;
    const bool st = stamps != nullptr;
    switch (kind) {
        case 0:
            if (st) hipLaunchKernelGGL(gemv_rowwave<true>, dim3(cdiv(m, 2)), dim3(128), 0, s, wc, xc, yb, m, ldb, stamps);
            else hipLaunchKernelGGL(gemv_rowwave<false>, dim3(cdiv(m, 2)), dim3(128), 0, s, wc, xc, yb, m, ldb, stamps);
            break;
        case 1:
            if (st) hipLaunchKernelGGL((gemv_persist<true, 4>), dim3(grid), dim3(256), 0, s, wc, xc, yb, m, ldb, stamps);
            else hipLaunchKernelGGL((gemv_persist<false, 4>), dim3(grid), dim3(256), 0, s, wc, xc, yb, m, ldb, stamps);
            break;
        case 2:
            if (st) hipLaunchKernelGGL((gemv_persist<true, 8>), dim3(grid), dim3(512), 0, s, wc, xc, yb, m, ldb, stamps);
            else hipLaunchKernelGGL((gemv_persist<false, 8>), dim3(grid), dim3(512), 0, s, wc, xc, yb, m, ldb, stamps);
            break;
        case 3:
            if (st) hipLaunchKernelGGL((gemv_persist<true, 2>), dim3(grid), dim3(128), 0, s, wc, xc, yb, m, ldb, stamps);
            else hipLaunchKernelGGL((gemv_persist<false, 2>), dim3(grid), dim3(128), 0, s, wc, xc, yb, m, ldb, stamps);
            break;
        case 4:
            if (st) hipLaunchKernelGGL((gemv_contig<true, 4>), dim3(grid), dim3(256), 0, s, wc, xc, yb, m, ldb, stamps);
            else hipLaunchKernelGGL((gemv_contig<false, 4>), dim3(grid), dim3(256), 0, s, wc, xc, yb, m, ldb, stamps);
            break;
        case 5:
            if (st) hipLaunchKernelGGL((gemv_contig<true, 2>), dim3(grid), dim3(128), 0, s, wc, xc, yb, m, ldb, stamps);
            else hipLaunchKernelGGL((gemv_contig<false, 2>), dim3(grid), dim3(128), 0, s, wc, xc, yb, m, ldb, stamps);
            break;
        default: return PLI_EINVAL;
    }
    return hipGetLastError() == hipSuccess ? PLI_OK : PLI_EINVAL;
}
