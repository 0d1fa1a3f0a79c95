// attn_fwd_v13's kernel argument block, shared by the D = 128 bodies
// (flash_v13.hip) and the D = 64 ones (flash_v13_d64.hip): 64 dwords in the
// layout of tools/v13/kernel.py ARG_LAYOUT (the generated body reads it
// through the kernarg pointer).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace pli {

struct V13Args {
    uint32_t w[64];
};
static_assert(sizeof(V13Args) == 256, "V13Args layout");

// launch one of the head-dim-64 bodies (bf16 / fp16, plain / causal /
// ragged -- Nk % 64 != 0, non-causal) on `grid` workgroups of 256 threads;
// returns the launch status
int launch_v13_d64(bool fp16, bool causal, bool ragged, unsigned grid, const V13Args& a, hipStream_t stream);
// attn_fwd_pp64 / pp64h / pp64c / pp64hc (flash_pp64.hip): head dim 64, bf16 /
// fp16, Nk % 64 == 0 (causal: Nq and Nk - Nq too), the arguments with
// 512-row blocks, workgroups of 512 threads
int launch_pp64(bool fp16, bool causal, unsigned grid, const V13Args& a, hipStream_t stream);

}  // namespace pli
