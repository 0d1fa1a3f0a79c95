// Timing probe for head dim 64 at two waves per SIMD, 64 rows per wave
// (tools/v14/probe64.py; results meaningless).  pp64_launch(variant, buf, out,
// niter, grid, c, mu, stream): buf = 32 MiB of bf16, out = 4 x 2048 words
// (cycles, checksum, barrier waits after the matrix / vector phase per wave).
#include <hip/hip_runtime.h>
#include <cstdint>

#include "probe64_asm.h"

struct PPArgs {
    uint32_t w[16];
};

#define PP64_KERNEL(name)                                                                     \
    __global__ __launch_bounds__(512) void pp64_##name(PPArgs args) {                         \
        __shared__ __attribute__((aligned(1024))) char smem[163840];                        \
        (void)args;                                                                         \
        const void* kp = (const void*)__builtin_amdgcn_kernarg_segment_ptr();               \
        const unsigned wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);             \
        const unsigned wg = blockIdx.x;                                                     \
        asm volatile(PP64_BODY_##name::"s"(kp), "s"(wg), "s"(wave), "s"((unsigned)(uintptr_t)smem) \
                     : PP64_CLOBBERS);                                                        \
    }
PP64_VARIANTS(PP64_KERNEL)

typedef void (*PPK)(PPArgs);
#define PP64_PTR(name) pp64_##name,
static const PPK kKernels[] = {PP64_VARIANTS(PP64_PTR)};

extern "C" int pp64_count() { return (int)(sizeof(kKernels) / sizeof(kKernels[0])); }

extern "C" int pp64_launch(int variant, const void* buf, void* out, int niter, int grid, float c, float mu,
                         hipStream_t s) {
    if (variant < 0 || variant >= pp64_count() || niter < 1 || grid < 1 || grid > 256) return -1;
    PPArgs a = {};
    a.w[0] = (uint32_t)(uintptr_t)buf;
    a.w[1] = (uint32_t)((uintptr_t)buf >> 32);
    a.w[2] = (uint32_t)(uintptr_t)out;
    a.w[3] = (uint32_t)((uintptr_t)out >> 32);
    a.w[4] = (uint32_t)niter;
    __builtin_memcpy(&a.w[5], &c, 4);
    __builtin_memcpy(&a.w[6], &mu, 4);
    hipLaunchKernelGGL(kKernels[variant], dim3(grid), dim3(512), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
