// attn_fwd_pp64: flash-attention forward at head dim 64 with two waves per
// SIMD in ping-pong (reference ch06/flash_attention.py:14-74, the ch06 GPU
// tests' head_dim 64 and ch01 MHA's d = 512 h = 8; gfx950, bf16 / fp16, non-causal,
// Nk a multiple of 64).  Eight waves of 64 query rows per workgroup (a
// 512-row block): waves w and w + 4 share a SIMD and alternate, barrier by
// barrier, between a matrix phase (PV(t-1) and QK(t), 64 MFMAs) and a vector
// phase (the softmax of tile t, its row sums, the LDS-DMA of tile t+4), so one
// wave's VALU stream runs under the other's MFMAs.  The body is one generated
// instruction stream (flash_pp64_asm.h from tools/v14/pp64.py, which also
// holds the register plan and the wait-count reasoning); the numerics are
// attn_fwd_v13's (bf16: the l >= 1 check; fp16: the P-bit check, no QSCALE).  The arguments are launch_attn_v13's (flash_v13.hip)
// with 512-row blocks; one block per workgroup.
#include "flash_v13.h"
#ifdef PLI_PP64_AB_HEADER  // timing A/B builds (tools/v14/build_pp64_ab.sh)
#include PLI_PP64_AB_HEADER
#else
#include "flash_pp64_asm.h"
#endif
#include "pli_common.h"

namespace pli {
namespace {

#define PLI_PP64_KERNEL(name, body)                                                                  \
    __global__ __launch_bounds__(512, 1) void name(V13Args args) {                                   \
        __shared__ __attribute__((aligned(1024))) char smem[98304];                                  \
        (void)args;                                                                                  \
        const void* kp = (const void*)__builtin_amdgcn_kernarg_segment_ptr();                        \
        const unsigned wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);                      \
        const unsigned wg = blockIdx.x;                                                              \
        asm volatile(body::"s"(kp), "s"(wg), "s"(wave), "s"((unsigned)(uintptr_t)smem) : PLI_PP64_CLOBBERS); \
    }

PLI_PP64_KERNEL(attn_fwd_pp64, PLI_PP64_BODY)
// fp16: P packed to fp16 and checked by the bit-14 test at the end of each
// vector phase (v13's fp16 rule), the mu offset from the launcher's
// v13_muoff_f16
PLI_PP64_KERNEL(attn_fwd_pp64h, PLI_PP64H_BODY)
// causal (bottom-right, Nq and Nk - Nq multiples of 64): per wave, the
// diagonal key tile masked by VALU, the tiles past it P = 0; one block per
// workgroup, heaviest first (block_params' remap walk)
PLI_PP64_KERNEL(attn_fwd_pp64c, PLI_PP64C_BODY)
PLI_PP64_KERNEL(attn_fwd_pp64hc, PLI_PP64HC_BODY)

}  // namespace

int launch_pp64(bool fp16, bool causal, unsigned grid, const V13Args& a, hipStream_t stream) {
    if (causal) {
        if (fp16) {
            hipLaunchKernelGGL(attn_fwd_pp64hc, dim3(grid), dim3(512), 0, stream, a);
            return launch_status("attn_fwd_pp64hc");
        }
        hipLaunchKernelGGL(attn_fwd_pp64c, dim3(grid), dim3(512), 0, stream, a);
        return launch_status("attn_fwd_pp64c");
    }
    if (fp16) {
        hipLaunchKernelGGL(attn_fwd_pp64h, dim3(grid), dim3(512), 0, stream, a);
        return launch_status("attn_fwd_pp64h");
    }
    hipLaunchKernelGGL(attn_fwd_pp64, dim3(grid), dim3(512), 0, stream, a);
    return launch_status("attn_fwd_pp64");
}

}  // namespace pli
