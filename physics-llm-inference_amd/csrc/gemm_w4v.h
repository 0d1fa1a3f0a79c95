// gemm_w4v (gemm_w4v.hip): 256x256 tile, one wave per SIMD, 128x128 of C per
// wave in the accumulator file, K staged 32 deep through a 5-slot LDS-DMA ring.
// Called from gemm.hip's dispatch.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pli {

// 16-bit operands (is_bf16: bf16, else fp16), K % 32 == 0, 16-byte aligned
// rows and bases, N % 8 == 0; trans_b: B is [N, K] (F.linear), else [K, N]
bool gemm_w4v_ok(int m, int n, int k, int64_t lda, int64_t ldb, int64_t ldc, int trans_b);
int launch_gemm_w4v(const void* a, const void* b, void* c, const void* bias, int m, int n, int k, int64_t lda,
                    int64_t ldb, int64_t ldc, int trans_b, int is_bf16, hipStream_t stream, int group_m);

}  // namespace pli
