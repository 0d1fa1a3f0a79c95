// gemm_w5 (gemm_w5.hip): gemm_w4v's 256x256 one-wave-per-SIMD tile with K
// staged 64 deep through two 64 KiB LDS slots.  Called from gemm.hip's dispatch.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pli {

// 16-bit operands (is_bf16: bf16, else fp16), K % 64 == 0, 16-byte aligned
// rows and bases, N % 8 == 0; trans_b: B is [N, K] (F.linear), else [K, N]
bool gemm_w5_ok(int m, int n, int k, int64_t lda, int64_t ldb, int64_t ldc, int trans_b);
// persistent: variant 43's walk (M, N multiples of 256); f32out: c is float
// [m][ldc] (NT, no bias: pli_gemm_f32out)
int launch_gemm_w5(const void* a, const void* b, void* c, const void* bias, int m, int n, int k, int64_t lda,
                   int64_t ldb, int64_t ldc, int trans_b, int is_bf16, hipStream_t stream, int group_m,
                   bool persistent = false, bool f32out = false);

// h = silu(x Wg^T) * (x Wu^T) (pli_gemm_swiglu prefill): 256 x 128 output
// tiles, K % 64 == 0, N % 8 == 0, 16-byte aligned rows and bases
int launch_gemm_w5_swiglu(const void* x, const void* wg, const void* wu, void* h, int m, int n, int k, int64_t ldx,
                          int64_t ldwg, int64_t ldwu, int64_t ldh, int is_bf16, hipStream_t stream);

}  // namespace pli
