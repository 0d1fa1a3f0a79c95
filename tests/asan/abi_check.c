/*
 * The C-ABI's host-side checks under AddressSanitizer (CPU
 * only).  Linked against build_asan/libpli_hip_asan.so (every source compiled
 * host-only with -fsanitize=address, physics-llm-inference_amd/build.py
 * --asan), so every argument check, the empty-operand rules, the workspace
 * sizing and the error / route strings run with ASan watching their reads and
 * writes.  No call here reaches a kernel launch: each one is refused or
 * finishes before any HIP call, which is what lets it run without a GPU.
 * The same calls are made through ctypes in tests/test_capi.py.
 * Exit status 0 = every check held (ASan aborts the process on a bad access).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "pli.h"

static int failures = 0;

#define CHECK(cond)                                                        \
    do {                                                                   \
        if (!(cond)) {                                                     \
            fprintf(stderr, "abi_check:%d: %s (last error: %s)\n", __LINE__, \
                    #cond, pli_last_error());                              \
            ++failures;                                                    \
        }                                                                  \
    } while (0)

static int err_has(const char* s) { return strstr(pli_last_error(), s) != NULL; }

int main(void) {
    void* p = (void*)(uintptr_t)16; /* never dereferenced: validation fails first */
    int64_t st0[12] = {0}, st8[12];
    for (int i = 0; i < 12; ++i) st8[i] = 8;

    CHECK(strncmp(pli_version(), "pli_hip", 7) == 0);
    CHECK(pli_last_error() != NULL && pli_last_route() != NULL);

    /* debug mode: query, set, restore (no launch happens here) */
    const int sync0 = pli_debug_sync(-1);
    CHECK(pli_debug_sync(1) == sync0);
    CHECK(pli_debug_sync(-1) == 1);
    CHECK(pli_debug_sync(sync0) == 1);

    /* null pointers and bad shapes: PLI_EINVAL with a message */
    CHECK(pli_gemv(NULL, NULL, NULL, 16, 16, 16, PLI_BF16, NULL) == PLI_EINVAL && err_has("null"));
    CHECK(pli_gemv(p, p, p, 16, 32, 16, PLI_BF16, NULL) == PLI_EINVAL && err_has("bad shape"));
    CHECK(pli_gemm(p, p, p, NULL, 8, 8, 8, 8, 8, 8, 0, 7, NULL) == PLI_EINVAL);
    CHECK(pli_flash_attn_fwd(p, p, p, p, 1, 6, 4, 8, 8, 64, st0, 0.1f, 0, PLI_BF16, NULL) == PLI_EINVAL &&
          err_has("multiple of kv_heads"));
    CHECK(pli_flash_attn_fwd(p, p, p, p, 1, 4, 4, 8, 8, 64, st0, NAN, 0, PLI_BF16, NULL) == PLI_EINVAL);
    CHECK(pli_flash_attn_fwd_variant(p, p, p, p, 1, 6, 4, 8, 8, 64, st0, 0.1f, 0, PLI_BF16, NULL, 80) ==
          PLI_EINVAL);
    CHECK(pli_scale_copy((const float*)p, (float*)p, 16, 0, NULL) == PLI_EINVAL);
    CHECK(pli_softmax_rows(p, p, 4, -1, 0, NULL) == PLI_EINVAL);
    CHECK(pli_attn_decode(p, p, p, p, 1, 6, 4, 1, 64, 64, st0, 0.1f, 0, NULL, 0, PLI_BF16, NULL) == PLI_EINVAL &&
          err_has("multiple of kv_heads"));
    CHECK(pli_attn_decode(p, p, p, p, 1, 8, 2, 4, 2, 64, st0, 0.1f, 1, NULL, 0, PLI_BF16, NULL) == PLI_EINVAL &&
          err_has("n_q"));

    /* split-K decode: its workspace is required, not silently dropped */
    const size_t need = pli_attn_decode_workspace_size(1, 32, 8, 1, 32768, 128);
    CHECK(need == (size_t)8 * 128 * 4 * (128 + 2) * 4);
    CHECK(pli_attn_decode(p, p, p, p, 1, 32, 8, 1, 32768, 128, st8, 0.1f, 0, NULL, need - 1, PLI_BF16, NULL) ==
              PLI_EINVAL &&
          err_has("workspace"));
    CHECK(pli_attn_decode_workspace_size(128, 32, 8, 1, 4096, 128) == 0);
    CHECK(pli_attn_decode_workspace_size(64, 32, 8, 1, 4096, 128) == (size_t)512 * 2 * 4 * (128 + 2) * 4);
    CHECK(pli_attn_decode_workspace_size(1, 8, 8, 1, 4096, 80) == 0);
    /* GEMM workspaces: sizes only (0 = the plain call) */
    (void)pli_gemm_workspace_size(128, 8192, 8192, 1, PLI_BF16);
    (void)pli_gemm_swiglu_workspace_size(64, 14336, 4096, PLI_BF16);
    CHECK(pli_gemm_workspace_size(8192, 8192, 8192, 1, PLI_BF16) == 0);

    /* fused decode projections: row / group limits */
    const void* w3[3] = {p, p, p};
    void* c3[3] = {p, p, p};
    int n3[3] = {64, 64, 64}, cap3[3] = {9, 9, 9};
    int64_t ld3[3] = {64, 64, 64};
    const int32_t* ro3[3] = {NULL, NULL, NULL};
    CHECK(pli_gemm_multi_nt(p, 64, 129, 64, 1, w3, c3, n3, ld3, ld3, ld3, ro3, cap3, 3, PLI_BF16, NULL) ==
              PLI_EINVAL &&
          err_has("m <= 128"));
    CHECK(pli_gemm_multi_nt(p, 64, 17, 64, 1, w3, c3, n3, ld3, ld3, ld3, ro3, cap3, 3, PLI_BF16, NULL) ==
              PLI_EINVAL &&
          err_has("k % 128"));
    CHECK(pli_gemm_multi_nt(p, 64, 6, 64, 4, w3, c3, n3, ld3, ld3, ld3, ro3, cap3, 3, PLI_BF16, NULL) ==
          PLI_EINVAL);
    CHECK(pli_gemm_multi_nt(p, 64, 4, 64, 1, w3, c3, n3, ld3, ld3, ld3, ro3, cap3, 4, PLI_BF16, NULL) ==
              PLI_EINVAL &&
          err_has("groups"));
    CHECK(pli_rms_gemm_nt(p, 8192, NULL, 0, p, 1e-6f, NULL, 0, 5, 64, 1, w3, NULL, c3, n3, ld3, ld3, ld3, ro3,
                          cap3, 3, PLI_BF16, NULL) == PLI_EINVAL &&
          err_has("m <= 4"));
    CHECK(pli_rms_gemm_nt(p, 8192, NULL, 0, p, 1e-6f, NULL, 0, 1, 16384, 1, w3, NULL, c3, n3, ld3, ld3, ld3,
                          ro3, cap3, 3, PLI_BF16, NULL) == PLI_EINVAL &&
          err_has("k <= 8192"));

    /* empty operands: NULL allowed where there are no elements; an empty
     * output is PLI_OK and launches nothing */
    for (int c = 0; c < 2; ++c) {
        const int B = c ? 2 : 0, Nq = c ? 0 : 8;
        CHECK(pli_flash_attn_fwd(NULL, NULL, NULL, NULL, B, 4, 4, Nq, 8, 64, NULL, 0.1f, 0, PLI_BF16, NULL) ==
              PLI_OK);
        CHECK(strcmp(pli_last_route(), "") == 0);
        CHECK(pli_attn_decode(NULL, NULL, NULL, NULL, B, 4, 4, Nq, 8, 64, NULL, 0.1f, 0, NULL, 0, PLI_BF16,
                              NULL) == PLI_OK);
    }
    CHECK(pli_flash_attn_fwd(NULL, NULL, NULL, NULL, 1, 4, 4, 8, 0, 64, st8, 0.1f, 0, PLI_BF16, NULL) ==
              PLI_EINVAL &&
          err_has("null"));
    const int mnk[3][3] = {{0, 8, 8}, {8, 0, 8}, {0, 0, 0}};
    for (int i = 0; i < 3; ++i) {
        const int m = mnk[i][0], n = mnk[i][1], k = mnk[i][2];
        CHECK(pli_gemm(NULL, NULL, NULL, NULL, m, n, k, 8, 8, 8, 1, PLI_BF16, NULL) == PLI_OK);
        CHECK(pli_gemm_f32out(NULL, NULL, NULL, m, n, k, 8, 8, PLI_BF16, NULL) == PLI_OK);
        CHECK(pli_gemm_swiglu(NULL, NULL, NULL, NULL, m, n, k, 8, 8, 8, 8, PLI_BF16, NULL) == PLI_OK);
        CHECK(pli_gemm_naive(NULL, NULL, NULL, m, n, k, 8, 8, 8, NULL) == PLI_OK);
    }
    CHECK(pli_gemm(NULL, NULL, NULL, NULL, 8, 8, 0, 8, 8, 8, 1, PLI_BF16, NULL) == PLI_EINVAL);
    CHECK(pli_gemv(NULL, NULL, NULL, 0, 16, 16, PLI_BF16, NULL) == PLI_OK);
    CHECK(pli_gemv(NULL, NULL, NULL, 16, 0, 16, PLI_BF16, NULL) == PLI_EINVAL);
    CHECK(pli_rmsnorm(NULL, NULL, NULL, NULL, NULL, 0, 64, 64, 64, 64, 64, 1e-6f, PLI_BF16, NULL) == PLI_OK);
    CHECK(pli_softmax_rows(NULL, NULL, 0, 64, PLI_BF16, NULL) == PLI_OK);
    CHECK(pli_softmax_rows(NULL, NULL, 4, 0, PLI_BF16, NULL) == PLI_OK);
    CHECK(pli_online_softmax_with_output(NULL, NULL, NULL, NULL, 0, 64, 64, PLI_BF16, NULL) == PLI_OK);
    CHECK(pli_scale_copy(NULL, NULL, 0, 1, NULL) == PLI_OK);
    CHECK(pli_kv_append(NULL, NULL, NULL, NULL, 2, 0, 4, 64, 128, NULL, NULL, PLI_BF16, NULL) == PLI_OK);
    CHECK(pli_moe_combine(NULL, 64, NULL, NULL, NULL, 64, 0, 2, 64, PLI_BF16, NULL) == PLI_OK);
    CHECK(pli_gemm_grouped(NULL, NULL, NULL, NULL, NULL, NULL, 4, 0, 64, 128, 128, 128, 64, PLI_BF16, NULL) ==
          PLI_OK);

    /* a long message is truncated into the thread-local buffer, never past it */
    for (int i = 0; i < 4; ++i)
        CHECK(pli_gemv(p, p, p, 16, 32 + i, 16, PLI_BF16, NULL) == PLI_EINVAL && strlen(pli_last_error()) < 512);

    if (failures) {
        fprintf(stderr, "abi_check: %d check(s) failed\n", failures);
        return 1;
    }
    printf("abi_check: all checks passed under AddressSanitizer\n");
    return 0;
}
