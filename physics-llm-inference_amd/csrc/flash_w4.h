// One-wave-per-SIMD flash forward (flash_w4.hip), called from the variant
// dispatch of flash_attn.hip.  D = 128, 16-bit operands, 16-byte aligned.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pli {

struct W4Strides {
    int64_t qb, qh, qn, kb, kh, kn, vb, vh, vn, ob, oh, on;
};

// sub: 0 = compiler schedule, 1 = sched_group_barrier interleave
int launch_attn_w4(const void* q, const void* k, const void* v, void* o, int B, int H, int group,
                   int Nq, int Nk, const W4Strides& st, float scale, int causal, int is_bf16,
                   hipStream_t stream, int sub);

}  // namespace pli
