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

// attn_fwd_v12 (flash_v12.hip): one wave per SIMD, 64 rows per wave, O/Q/K in
// the accumulator file; bf16, D = 128, non-causal, Nk a multiple of 64
// (attn_v13_ok: bf16 or fp16 -- is_bf16 only picks the program)
bool attn_v12_ok(int D, int is_bf16, int causal, int Nk);
bool attn_v13_ok(int D, int is_bf16, int causal, int Nq, int Nk, const V7Strides& st);
// attn_fwd_v13 (flash_v13.hip, flash_v13_d64.hip): bf16 or fp16 (fp16 =
// true), head dim D = 128 or 64; pp64: attn_fwd_pp64 (flash_pp64.hip) where
// it applies (D = 64, bf16 / fp16, Nk % 64 == 0; causal: Nq % 64 == 0 and
// Nk - Nq a non-negative multiple of 64)
bool attn_pp64_ok(int D, bool fp16, bool causal, int Nq, int Nk);
int launch_attn_v13(const void* q, const void* k, const void* v, void* o, int B, int H, int group, int Nq,
                    int Nk, const V7Strides& st, float scale, hipStream_t stream, bool persistent, float muoff,
                    uint32_t* stamps = nullptr, bool causal = false, bool fp16 = false, int D = 128,
                    bool pp64 = false);
// thr: the defer-max threshold (log2 units); 64 and 0 are the built forms
int launch_attn_v12(const void* q, const void* k, const void* v, void* o, int B, int H, int group, int Nq,
                    int Nk, const V7Strides& st, float scale, hipStream_t stream, bool persistent,
                    float thr = 64.f, bool causal = false);

}  // namespace pli
