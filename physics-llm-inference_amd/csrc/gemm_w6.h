// gemm_w6 (gemm_w6.hip): gemm_w5's tile with the operands staged through VGPRs
// (global_load_dwordx4 + ds_write_b128) instead of LDS-DMA.  Called from
// gemm.hip's dispatch.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pli {

// 16-bit operands (is_bf16: bf16, else fp16), K % 64 == 0, 16-byte aligned
// rows and bases, N % 8 == 0; trans_b: B is [N, K] (F.linear), else [K, N]
bool gemm_w6_ok(int m, int n, int k, int64_t lda, int64_t ldb, int64_t ldc, int trans_b);
int launch_gemm_w6(const void* a, const void* b, void* c, const void* bias, int m, int n, int k, int64_t lda,
                   int64_t ldb, int64_t ldc, int trans_b, int is_bf16, hipStream_t stream, int group_m);

}  // namespace pli
