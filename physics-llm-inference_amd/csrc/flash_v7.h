// Lean-softmax flash forward (flash_v7.hip), called from the dispatch of
// flash_attn.hip.  D in {64, 128}, 16-bit operands, 16-byte aligned rows.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pli {

struct V7Strides {
    int64_t qb, qh, qn, kb, kh, kn, vb, vh, vn, ob, oh, on;
};

// sub selects a build of the body (A/B levers, see flash_v7.hip); 0 = default
int launch_attn_v7(const void* q, const void* k, const void* v, void* o, int B, int H, int group,
                   int Nq, int Nk, int D, const V7Strides& st, float scale, int causal, int is_bf16,
                   hipStream_t stream, int sub);

}  // namespace pli
