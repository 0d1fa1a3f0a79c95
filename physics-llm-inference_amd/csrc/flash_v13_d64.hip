// attn_fwd_v13 at head dim 64 (reference ch01/attention.py:45-72 MHA d=512
// h=8, and the ch06 GPU tests, run head_dim 64): the generated program of
// tools/v13/kernel.py with Gen(hd=64) -- the D = 64 K / V tile images are the
// first halves of the D = 128 ones (same swizzle, fragment offsets and DMA
// piece map), 4 LDS-DMA pieces per wave and 32 + 32 MFMAs per 64 x 64
// wave-tile.  bf16 and fp16, plain, causal and ragged (Nk % 64 != 0); flash_v13.hip's launcher
// fills the arguments and calls launch_v13_d64.
#include "flash_v13.h"
#ifdef PLI_V13D64_AB_HEADER  // timing-only A/B builds (tools/build_v13_ab.sh)
#include PLI_V13D64_AB_HEADER
#else
#include "flash_v13_d64_asm.h"
#endif
#include "pli_common.h"

namespace pli {
namespace {

#define PLI_V13_D64_KERNEL(name, body)                                                              \
    __global__ __launch_bounds__(256, 1) void name(V13Args args) {                                  \
        __shared__ __attribute__((aligned(1024))) char smem[163840];                                \
        (void)args;                                                                                 \
        const void* kp = (const void*)__builtin_amdgcn_kernarg_segment_ptr();                       \
        const unsigned wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);                     \
        const unsigned wg = blockIdx.x;                                                             \
        asm volatile(body::"s"(kp), "s"(wg), "s"(wave), "s"((unsigned)(uintptr_t)smem)              \
                     : PLI_V13D64_CLOBBERS);                                                        \
    }

PLI_V13_D64_KERNEL(attn_fwd_v13_d64, PLI_V13_D64_BODY)
PLI_V13_D64_KERNEL(attn_fwd_v13c_d64, PLI_V13C_D64_BODY)
PLI_V13_D64_KERNEL(attn_fwd_v13h_d64, PLI_V13H_D64_BODY)
PLI_V13_D64_KERNEL(attn_fwd_v13hc_d64, PLI_V13HC_D64_BODY)
PLI_V13_D64_KERNEL(attn_fwd_v13r_d64, PLI_V13R_D64_BODY)
PLI_V13_D64_KERNEL(attn_fwd_v13hr_d64, PLI_V13HR_D64_BODY)
PLI_V13_D64_KERNEL(attn_fwd_v13rc_d64, PLI_V13RC_D64_BODY)
PLI_V13_D64_KERNEL(attn_fwd_v13hrc_d64, PLI_V13HRC_D64_BODY)

}  // namespace

int launch_v13_d64(bool fp16, bool causal, bool ragged, unsigned grid, const V13Args& a, hipStream_t stream) {
    if (ragged && causal) {
        if (fp16) {
            hipLaunchKernelGGL(attn_fwd_v13hrc_d64, dim3(grid), dim3(256), 0, stream, a);
            return launch_status("attn_fwd_v13hrc_d64");
        }
        hipLaunchKernelGGL(attn_fwd_v13rc_d64, dim3(grid), dim3(256), 0, stream, a);
        return launch_status("attn_fwd_v13rc_d64");
    }
    if (ragged) {
        if (fp16) {
            hipLaunchKernelGGL(attn_fwd_v13hr_d64, dim3(grid), dim3(256), 0, stream, a);
            return launch_status("attn_fwd_v13hr_d64");
        }
        hipLaunchKernelGGL(attn_fwd_v13r_d64, dim3(grid), dim3(256), 0, stream, a);
        return launch_status("attn_fwd_v13r_d64");
    }
    if (fp16 && causal) {
        hipLaunchKernelGGL(attn_fwd_v13hc_d64, dim3(grid), dim3(256), 0, stream, a);
        return launch_status("attn_fwd_v13hc_d64");
    }
    if (fp16) {
        hipLaunchKernelGGL(attn_fwd_v13h_d64, dim3(grid), dim3(256), 0, stream, a);
        return launch_status("attn_fwd_v13h_d64");
    }
    if (causal) {
        hipLaunchKernelGGL(attn_fwd_v13c_d64, dim3(grid), dim3(256), 0, stream, a);
        return launch_status("attn_fwd_v13c_d64");
    }
    hipLaunchKernelGGL(attn_fwd_v13_d64, dim3(grid), dim3(256), 0, stream, a);
    return launch_status("attn_fwd_v13_d64");
}

}  // namespace pli
