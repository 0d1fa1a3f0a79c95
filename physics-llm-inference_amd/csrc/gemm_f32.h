// fp32 GEMM on v_mfma_f32_32x32x2_f32 (gemm_f32.hip), called from the
// pli_gemm dispatch in gemm.hip for fp32 operands.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pli {

// 16-byte aligned operands, K and the leading dimensions multiples of 4
bool gemm_f32_mfma_ok(const void* a, const void* b, const void* c, int k, int n, int64_t lda, int64_t ldb,
                      int trans_b);
int launch_gemm_f32_mfma(const void* a, const void* b, void* c, const void* bias, int M, int N, int K,
                         int64_t lda, int64_t ldb, int64_t ldc, int trans_b, hipStream_t s);

}  // namespace pli
