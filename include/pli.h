/*
 * pli.h -- C ABI of libpli_hip.so, the MI355X (gfx950) hot path of
 * Infatoshi/physics-llm-inference re-built as hand-written HIP kernels.
 *
 * Conventions (every entry point):
 *   - plain pointers and sizes only; no torch / HIP types in signatures.
 *     `stream` is a hipStream_t passed as void* (NULL = the null stream).
 *   - the CALLER owns every buffer, outputs included; the library never
 *     allocates, frees or synchronises (calls are graph-capturable).
 *   - device pointers must be 16-byte aligned for the vectorised kernels;
 *     misaligned / oddly strided operands are routed to the generic kernels.
 *   - strides are in ELEMENTS; the innermost (head_dim / K) stride is 1.
 *   - empty operands: a pointer to an operand with zero elements may be NULL
 *     (torch hands out a NULL data_ptr for empty tensors).  A call whose
 *     output is empty does nothing and returns PLI_OK; an empty reduction
 *     (no keys, K == 0) writes what torch gives for it (O = 0, C = bias or
 *     0, y = 0).
 *   - return value: PLI_OK (0), a hipError_t code (1..999) from the launch,
 *     or one of the PLI_E* codes below.  pli_last_error() returns a
 *     thread-local message for the last failing call on this thread.
 *
 * The reference has no FFI layer: its boundary is a set of
 * Python call signatures.  Each entry point below names the reference
 * function whose device arithmetic it replaces; the Python mirror packages
 * (physics-llm-inference_amd/ch0X) keep those signatures and call in here.
 */
#ifndef PLI_H
#define PLI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif
/* the library is built with -fvisibility=hidden: exactly the entry points
 * declared here are exported */
#if defined(__GNUC__) || defined(__clang__)
#pragma GCC visibility push(default)
#endif

/* element types */
enum {
    PLI_F32 = 0,
    PLI_F16 = 1,
    PLI_BF16 = 2
};

/* status codes beyond hipError_t */
enum {
    PLI_OK = 0,
    PLI_EINVAL = 1000,      /* bad argument (shape, stride, dtype, null)     */
    PLI_EUNSUPPORTED = 1001 /* valid but not implemented on this path        */
};

/* Library version string, e.g. "pli_hip 0.1.0 gfx950". */
const char* pli_version(void);

/* Message for the last non-zero return on the calling thread ("" if none). */
const char* pli_last_error(void);

/* The kernels the calling thread's last entry-point call launched, in launch
 * order, '+'-separated (e.g. "attn_fwd_v13c", "gemm_splitk_lds_nt+
 * gemm_splitk_reduce"); "" when it launched none (an empty output).  For
 * tests and tuning: which route the dispatch took. */
const char* pli_last_route(void);

/* Synchronous debug mode: when on, every kernel launch is
 * followed by hipDeviceSynchronize + hipGetLastError, and a failure is
 * returned by the entry point that launched the kernel, its name in
 * pli_last_error() ("<kernel>: kernel failed (PLI_SYNC): ...").  Starts as
 * the environment says (PLI_SYNC=1 or HIP_LAUNCH_BLOCKING=1: on; else off).
 * mode 0 / 1 sets
 * it, mode < 0 only queries; returns the previous state.  Debugging only:
 * it serialises every call and must not be on while a stream is captured. */
int pli_debug_sync(int mode);

/*
 * Fused attention forward:  O = softmax(Q K^T * scale [+ causal mask]) V.
 *
 * Replaces the device work of
 *   ch06/flash_attention.py:14-74   flash_attention_forward (tile loop)
 *   ch06/attention_memory.py:19-33  naive_attention
 *   ch01/attention.py:65-69         MultiHeadAttention.forward core
 *   ch01/gqa.py:30-34               GQA (kv head = h / (H / Hkv), no repeat)
 *
 * Layout: logical [batch, heads, n, head_dim]; q/o have `heads` heads and
 * n_q rows, k/v have `kv_heads` heads and n_kv rows.  strides[12] holds, in
 * elements, {q_b, q_h, q_n, k_b, k_h, k_n, v_b, v_h, v_n, o_b, o_h, o_n}.
 * causal != 0 masks key j for query i when j > i + (n_kv - n_q)
 * (bottom-right aligned, = torch.triu(ones, diagonal=1) when n_q == n_kv).
 * dtype: PLI_BF16 / PLI_F16 with head_dim 64 or 128 run the MFMA kernels --
 * attn_fwd_v13 (one generated program per dtype x head_dim x causal x
 * whole / ragged key tiles) where n_kv > 64 (causal: n_q <= n_kv, any
 * diagonal offset), else attn_fwd_v12 / v10; PLI_F32 (and any other
 * head_dim <= 256) the generic fp32-accumulate kernel.  Softmax statistics
 * are fp32 regardless of dtype.  n_kv == 0 gives O = 0.
 */
int pli_flash_attn_fwd(const void* q, const void* k, const void* v, void* o,
                       int batch, int heads, int kv_heads, int n_q, int n_kv,
                       int head_dim, const int64_t* strides, float scale,
                       int causal, int dtype, void* stream);

/*
 * GEMV  y[m] = sum_k W[m, k] * x[k]   (fp32 accumulate, output in dtype).
 * Replaces torch.mv in ch03/gemv_benchmark.py:38 (decode weight GEMV).
 * W row-major with leading dimension ldw (elements, >= k).
 */
int pli_gemv(const void* w, const void* x, void* y, int m, int k, int64_t ldw,
             int dtype, void* stream);

/*
 * GEMM  C[m, n] = A[m, k] * op(B) (+ bias[n])   (fp32 accumulate).
 * trans_b = 0: B is [k, n] row-major (torch.mm, ch03/gemm_benchmark.py:35,
 *              ch05/tiled_matmul.cu:22-61);
 * trans_b = 1: B is [n, k] row-major, i.e. C = A B^T (F.linear,
 *              ch09/tensor_parallel.py:39,67; ch01/attention.py:59-61,71;
 *              x @ weight.T of ch03/batching_benchmark.py:30).
 * bias may be NULL.  A, C row-major with leading dimensions lda, ldc.
 */
int pli_gemm(const void* a, const void* b, void* c, const void* bias, int m,
             int n, int k, int64_t lda, int64_t ldb, int64_t ldc, int trans_b,
             int dtype, void* stream);

/*
 * NT GEMM with an fp32 output: C[m, n] = A[m, k] * B[n, k]^T, A / B bf16 or
 * fp16 (dtype), C fp32 contiguous (ldc = n), fp32 accumulate -- the
 * row-parallel partial of ch09/tensor_parallel.py:66-68 kept in fp32 so the
 * all-reduce sums unrounded partials (RowParallelLinear(reduce_dtype=
 * torch.float32)).  Routes, in the order gemm.hip pli_gemm_f32out checks
 * them: (1) K % 64 == 0, N % 32 == 0, lda % 8 == 0, ldb % 8 == 0, A / B / C
 * 16-byte aligned, M >= 512, N >= 512, at least 128 tiles of 256 x 256 and
 * 256 rows of A and B addressable by a 32-bit offset: gemm_w5 with an fp32
 * epilogue (its persistent walk when M, N are multiples of 256 and K >=
 * 128); (2) the rest of (1)'s alignment class (K % 64 == 0, N % 32 == 0,
 * lda / ldb % 8 == 0, 16-byte aligned A / B / C): the LDS split-K kernel
 * with one slice; (3) everything else: a one-thread-per-output kernel.
 */
int pli_gemm_f32out(const void* a, const void* b, float* c, int m, int n, int k, int64_t lda,
                    int64_t ldb, int dtype, void* stream);

/*
 * pli_gemm with a caller-owned device workspace (16-byte aligned) of at least
 * pli_gemm_workspace_size(m, n, k, trans_b, dtype) bytes (0: none needed, the
 * call is pli_gemm).  Decode-batch / TP-shard NT shapes (16 < m <= 256) then
 * split K over workgroups and sum the fp32 slices in a fixed order (the
 * ch09/tensor_parallel.py:67 row shard at M = 128, ch03/batching_benchmark.py
 * batches).  The workspace is scratch: nothing persists between calls.
 */
size_t pli_gemm_workspace_size(int m, int n, int k, int trans_b, int dtype);
int pli_gemm_ws(const void* a, const void* b, void* c, const void* bias, int m,
                int n, int k, int64_t lda, int64_t ldb, int64_t ldc, int trans_b,
                int dtype, void* workspace, size_t workspace_bytes, void* stream);

/*
 * Fused SwiGLU projection  h[m, n] = silu(x Wg^T)[m, n] * (x Wu^T)[m, n]
 * (fp32 accumulate, silu(g) = g / (1 + e^-g)).
 * Replaces gate_proj -> silu, up_proj, multiply of
 *   ch09/tensor_parallel.py:95-99   TensorParallelMLP.forward (per rank)
 *   ch01/ffn.py:34-39               SwiGLUFFN; ch01/ffn.py:51-57 FusedSwiGLUFFN
 *                                   (gate_up_proj halves: wg = W, wu = W + n*ldw)
 *   ch02/cached_generation.py:119   SwiGLUFFN of the cached model
 * x [m, k] (ldx), wg / wu [n, k] row-major (ldwg, ldwu), h [m, n] (ldh).
 * Neither gate nor up is written to memory.
 */
int pli_gemm_swiglu(const void* x, const void* wg, const void* wu, void* h,
                    int m, int n, int k, int64_t ldx, int64_t ldwg,
                    int64_t ldwu, int64_t ldh, int dtype, void* stream);
/* pli_gemm_swiglu with a caller workspace of pli_gemm_swiglu_workspace_size
 * bytes (0: none needed): decode batches (16 < m <= 256) split K over
 * workgroups for gate and up and apply silu(g) * u in a fixed-order reduce. */
size_t pli_gemm_swiglu_workspace_size(int m, int n, int k, int dtype);
int pli_gemm_swiglu_ws(const void* x, const void* wg, const void* wu, void* h,
                       int m, int n, int k, int64_t ldx, int64_t ldwg,
                       int64_t ldwu, int64_t ldh, int dtype, void* workspace,
                       size_t workspace_bytes, void* stream);

/*
 * HBM calibration kernels of ch05/coalescing.cu:7-20 (fp32):
 *   out[i] = 2 * in[i * stride],  i in [0, n_out).
 * stride == 1 is the coalesced stream (16-byte vector loads), the roofline
 * denominator measured on the device; stride > 1 is the strided contrast.
 */
int pli_scale_copy(const float* in, float* out, int64_t n_out, int stride,
                   void* stream);

/*
 * Roofline calibration (ch03/roofline.py measure_mfma_peak): `blocks`
 * workgroups of 256 threads, one per CU (96 KiB of LDS each) so ONE wave per
 * SIMD, each wave issuing `iters` rounds of back-to-back bf16 MFMAs from
 * registers into independent accumulators, pseudo-random operands; both
 * shapes the same 64x64 output tile per wave and 262,144 FLOP per round
 * (shape 0: 8 x v_mfma_f32_32x32x16_bf16, 1: 16 x v_mfma_f32_16x16x32_bf16).
 * One float per thread goes to out[blocks * 256] so the work is not dead;
 * when `clocks` is non-null, wave w writes clocks[2w] = s_memtime ticks
 * (shader clock) and clocks[2w+1] = s_memrealtime ticks (100 MHz) around its
 * loop.  FLOPs = blocks * 4 * iters * 262144.
 */
int pli_mfma_probe(float* out, uint64_t* clocks, int blocks, int iters, int shape, void* stream);

/*
 * ch05/tiled_matmul.cu:9-20 naive_matmul (the contrast kernel of the ch05
 * demo): C[m][n] = sum_k A[m][k] B[k][n], fp32 row-major, one thread per
 * output element straight from global memory.  Not a production path --
 * pli_gemm with PLI_F32 runs the MFMA tile kernel.
 */
int pli_gemm_naive(const float* a, const float* b, float* c, int m, int n, int k, int64_t lda,
                   int64_t ldb, int64_t ldc, void* stream);

/*
 * Read-only HBM calibration (ch03/roofline.py measure_hbm_read_bandwidth):
 * `blocks` x 256 threads stream `bytes` (16-byte aligned, multiple of 16)
 * with 16-byte non-temporal loads; one XOR word per thread goes to
 * out[blocks * 256].  mode 0: grid-stride (4 loads per lane in flight);
 * mode 1: one contiguous slice per block, 8 loads per lane in flight.
 */
int pli_hbm_read_probe(const void* buf, int64_t bytes, uint32_t* out, int blocks, int mode,
                       void* stream);

/*
 * Row softmax with the single-pass online (max, sum) recurrence of
 * ch06/online_softmax.py:13-25 (== standard_softmax, :5-10), over the last
 * dimension of a contiguous [rows, n] tensor; statistics in fp32.
 */
int pli_softmax_rows(const void* x, void* y, int64_t rows, int n, int dtype,
                     void* stream);

/*
 * ch06/online_softmax.py:28-53 online_softmax_with_output over contiguous
 * x [rows, n] and v [rows, n, dv]:  o[r] = sum_i softmax(x[r])_i v[r, i],
 * d[r] = sum_i exp(x[r, i] - max_r).  o is [rows, dv], d is [rows].
 */
int pli_online_softmax_with_output(const void* x, const void* v, void* o,
                                   void* d, int64_t rows, int n, int dv,
                                   int dtype, void* stream);

/* Decode attention over a KV cache (split-K flash-decoding).
 * Replaces the decode branch of ch02/kv_cache.py:74-101 (GQAWithCache.forward)
 * and ch02/cached_generation.py:58-98 (CachedGQA.forward): repeat_interleave
 * of the cache to Hq heads, matmul, softmax, matmul.
 * Same operand conventions as pli_flash_attn_fwd (strides[12] in elements,
 * q/o [B, Hq, n_q, D]-indexed, k/v [B, Hkv, n_kv, D]-indexed; the cache
 * layout [B, S_max, Hkv, D] is k_b = S_max*Hkv*D, k_h = D, k_n = Hkv*D).
 * causal masks bottom-right (query i sees keys j <= n_kv - n_q + i), the mask
 * of ch02/kv_cache.py:91-95.  The fast path takes bf16/fp16, D in {64, 128}
 * and n_q * Hq/Hkv <= 16 rows per kv head; other shapes run the prefill
 * kernel.  `workspace` (16-byte aligned, fp32 partials) must hold
 * pli_attn_decode_workspace_size(...) bytes; NULL when that is 0. */
size_t pli_attn_decode_workspace_size(int batch, int heads, int kv_heads,
                                      int n_q, int n_kv, int head_dim);
int pli_attn_decode(const void* q, const void* k, const void* v, void* o,
                    int batch, int heads, int kv_heads, int n_q, int n_kv,
                    int head_dim, const int64_t* strides, float scale,
                    int causal, void* workspace, size_t workspace_bytes,
                    int dtype, void* stream);

/*
 * RMSNorm with an optional fused residual add (rows of n elements):
 *   h = x + residual (stored in dtype, as the torch add would; h = x when
 *   residual is NULL), y = h / sqrt(mean(h^2) + eps) * weight, fp32 statistics.
 * Replaces ch02/cached_generation.py:101-109 (RMSNorm.forward) and the
 * residual adds of CachedTransformerBlock.forward (:143-145).  residual and
 * h_out may be NULL; h_out must not alias x or residual.
 */
int pli_rmsnorm(const void* x, const void* residual, const void* weight, void* y,
                void* h_out, int64_t rows, int n, int64_t ldx, int64_t ldr,
                int64_t ldy, int64_t ldh, float eps, int dtype, void* stream);

/*
 * Mixture of experts (ch09/moe_layer.py:18-83: Router softmax/topk/renorm and
 * the per-expert masked loop).
 *
 * pli_moe_route: logits [tokens, experts] (ld_logits) -> per (token, k):
 *   weights (fp32; renormalised over the k when normalize), expert_idx,
 *   pos (row of the expert-sorted activation matrix); gather[row] = token;
 *   offsets[experts + 1] = each expert's row range.  experts <= 64, top_k <= 8.
 *   workspace: int32 [experts + tokens * top_k].
 * pli_gemm_grouped: for every expert e, rows r in [offsets[e], offsets[e+1]):
 *   c[r] = x[gather[r]] W_e^T  (gather NULL = identity), or with wu_ptrs
 *   silu(x W1_e^T) * (x W3_e^T); w_ptrs / wu_ptrs are DEVICE arrays of the
 *   experts' [n, k] weight pointers; rows_bound >= every expert's row count.
 *   bf16/fp16, k % 128 == 0, n % 16 == 0.
 * pli_moe_combine: out[t] = sum_k weights[t, k] * y[pos[t, k]] (fp32 sum in k
 *   order).
 */
int pli_moe_route(const void* logits, int64_t ld_logits, int tokens, int experts,
                  int top_k, int normalize, int dtype, float* weights,
                  int32_t* expert_idx, int32_t* pos, int32_t* gather,
                  int32_t* offsets, int32_t* workspace, void* stream);
int pli_gemm_grouped(const void* x, const int32_t* gather,
                     const void* const* w_ptrs, const void* const* wu_ptrs,
                     void* c, const int32_t* offsets, int experts, int rows_bound,
                     int n, int k, int64_t ldx, int64_t ldw, int64_t ldc,
                     int dtype, void* stream);
int pli_moe_combine(const void* y, int64_t ldy, const int32_t* pos,
                    const float* weights, void* out, int64_t ldo, int tokens,
                    int top_k, int hidden, int dtype, void* stream);

/* Graph-replayable decode (ch08/cuda_graph.py:18-82 captures the decode step;
 * a captured launch cannot take the growing cache length as a host value).
 *
 * pli_kv_append: write n_new tokens of K and V ([B, n_new, Hkv, D]) into the
 * caches at rows *pos_dev .. *pos_dev + n_new - 1 (rows >= capacity are
 * dropped) -- the device-side form of KVCache.update, ch02/kv_cache.py:37-48.
 * strides[12] in elements: {kn_b, kn_h, kn_n, kc_b, kc_h, kc_n, vc_b, vc_h,
 * vc_n, vn_b, vn_h, vn_n}.  bf16/fp16, head_dim % 8 == 0.
 *
 * pli_attn_decode_dev: pli_attn_decode over n_kv = min(*n_kv_dev + n_kv_add,
 * n_kv_max) valid cache rows; the split-K grid and the workspace are sized
 * for n_kv_max (pli_attn_decode_workspace_size(..., n_kv_max, ...)).
 * Fast-path shapes only (else PLI_EUNSUPPORTED). */
int pli_kv_append(const void* k_new, const void* v_new, void* k_cache,
                  void* v_cache, int batch, int n_new, int kv_heads,
                  int head_dim, int capacity, const int64_t* strides,
                  const int32_t* pos_dev, int dtype, void* stream);
/* pli_gemm_multi_nt: the q, k and v projections of a decode step in one
 * launch, k / v written straight into the caches (fuses pli_kv_append).
 * Up to 3 groups share x [m, k] (m <= 128 rows = batch x tokens_per_batch);
 * group g computes x W_g^T ([n_g, k] weights, ldw_g) and stores row
 * r = b * tokens_per_batch + s at
 *   c_g + b * stride_batch_g + (s + *row_offset_g) * stride_token_g (+ col),
 * row_offset_g a device int32 or NULL (= 0); rows >= capacity_g are dropped.
 * bf16/fp16, k % 8 == 0; m > 16 (small-M MFMA kernel) also needs k % 128 == 0,
 * n_g % 16 == 0, strides % 4 == 0 and 8-byte aligned c_g. */
int pli_gemm_multi_nt(const void* x, int64_t ldx, int m, int k,
                      int tokens_per_batch, const void* const* w,
                      void* const* c, const int* n, const int64_t* ldw,
                      const int64_t* stride_batch, const int64_t* stride_token,
                      const int32_t* const* row_offset, const int* capacity,
                      int ngroups, int dtype, void* stream);
/* pli_rms_gemm_nt: a decode-step RMSNorm fused into the projection that
 * consumes it (ch02/cached_generation.py:112-120 RMSNorm -> :58-69 q/k/v,
 * :136-140 gate/up, :180-185 final norm -> lm_head).  Rows: h = a (+ residual)
 * (written to h_out if not NULL), y = h * rsqrt(mean(h^2) + eps) * norm_weight
 * -- bitwise the row pli_rmsnorm writes -- kept on chip; then the groups of
 * pli_gemm_multi_nt on y (w_up non-NULL: every group is SwiGLU,
 * silu(y.w) * (y.w_up), w_up rows with the same ldw).  1 <= m <= 4 rows,
 * k % 8 == 0, k <= 8192, bf16/fp16. */
int pli_rms_gemm_nt(const void* a, int64_t lda, const void* residual, int64_t ldr,
                    const void* norm_weight, float eps, void* h_out, int64_t ldh, int m, int k,
                    int tokens_per_batch, const void* const* w, const void* const* w_up,
                    void* const* c, const int* n, const int64_t* ldw,
                    const int64_t* stride_batch, const int64_t* stride_token,
                    const int32_t* const* row_offset, const int* capacity, int ngroups,
                    int dtype, void* stream);
int pli_attn_decode_dev(const void* q, const void* k, const void* v, void* o,
                        int batch, int heads, int kv_heads, int n_q,
                        int n_kv_max, int head_dim, const int64_t* strides,
                        float scale, int causal, const int32_t* n_kv_dev,
                        int n_kv_add, void* workspace, size_t workspace_bytes,
                        int dtype, void* stream);

/* ------------------------------------------------------------------------
 * Tuning section: the same operations with an explicit kernel choice, for
 * A/B runs (tools/tune.py) and the per-variant parity tests.  Not part of
 * the drop-in surface above -- a caller that binds the reference's
 * interface never needs them.  variant / mode < 0 (or 0 where noted) is the
 * default route; every listed value is parity-tested at the bench sizes
 * (tests/test_gpu_fullsize.py) and on the small edge cases
 * (tests/test_gpu_parity.py, test_gpu_decode.py, test_gpu_moe.py,
 * test_gpu_swiglu.py).
 *
 * pli_flash_attn_fwd_variant: 21 attn_fwd_v2 (round-1 kernel), 50 / 51
 *   attn_fwd_v7 prescaled / exact, 54 / 55 attn_fwd_v10 prescaled / exact,
 *   60 attn_fwd_v10 exact in 4-wave workgroups, 70 / 71 attn_fwd_v12 (one
 *   wave per SIMD, 64 rows per wave; 71 persistent, bitwise equal to 55;
 *   other inputs take 55); 72 = 71 with the defer-max threshold at 0
 *   (tests); 73 / 74 attn_fwd_v12 causal, one block per workgroup /
 *   persistent pair walk; 80 / 81 / 82 attn_fwd_v13 (16x16x32 MFMA, one
 *   generated instruction stream) persistent / one block per workgroup /
 *   80 with the rescale path at every tile (tests) -- 80 is the default
 *   for bf16 and fp16 (attn_fwd_v13h, the f16 MFMA) D = 128 / 64 with Nk a
 *   multiple of 64 from 128, or any Nk > 64 (attn_fwd_v13r / v13hr: the last
 *   key tile fetched from key Nk - 64, its overlap masked in P); 83 / 84 /
 *   85 the causal forms (83 = causal default for any Nq <= Nk and Nk > 64,
 *   ragged Nk on attn_fwd_v13rc / v13hrc; other shapes take 74 / 60);
 *   86 / 87 attn_fwd_pp64 / pp64h (head dim 64, two waves per SIMD,
 *   512-row blocks; causal: pp64c / pp64hc with Nq and Nk - Nq multiples
 *   of 64) / the same with the rescale path at every tile, other shapes
 *   take 80 / 83 (82 / 85); 88 (the default since round 6) = 86 for
 *   non-causal D = 64 where B H ceil(Nq / 512) fills the CUs, else 80 /
 *   83.  Prescaled variants round Q * scale * log2(e) to
 *   the 16-bit input type (2^-9 relative score error in bf16).  The v13
 *   forms, v12 and the exact v7 / v10 bodies (51 / 55 / 60) take any
 *   scale > 0; the prescaled 50 / 54 take scale * log2(e) <= 1 (larger
 *   scales fall back to 21).
 * pli_gemm_w5 schedule (all gemm_w5 routes): W5_SPLIT, DMA spread over both
 *   halves of each 64-deep K step (gemm_w5.hip).
 * pli_gemm_variant / pli_gemm_ws_variant: 0 default; 1 128^2 tile; 2 256^2
 *   one-phase; 3 phased SCHED 0; 4 one-phase + setprio; 5-8 phased SCHED
 *   1/3/5/7; 9-11 grouped one-phase (group_m 4/8/16); 12-15 grouped phased
 *   (8/4/2/16); 20 mid-M; 21 small-M; 22/24 direct-load split-K; 25-29 LDS
 *   split-K (256/512/128 targets, 3-deep ring); 40 gemm_w4v (one wave per
 *   SIMD, K 32 deep); 41 gemm_w5 (K 64 deep), 43 gemm_w5 persistent walk
 *   (M, N multiples of 256) -- 43 is the large-shape default (K >= 128).
 * pli_gemv_variant: 0-16 (rows per wave x 16-B chunks per lane x waves per
 *   block, gemv.hip), -1 default.
 * pli_attn_decode_variant: mode -1 default, 2/9/11/13 load-layout modes
 *   (decode_attn.hip); target_wgs 0 = automatic split.
 * pli_gemm_swiglu_ws_variant: 0 default, 1 split K wherever the split-K
 *   route applies, 2 never split, 3 gemm_w5's SwiGLU tile (the prefill
 *   default), 4 the phased 256 x 128 tile (3 and 4 never split).
 * pli_gemm_grouped_variant: 0 default, 1/2 alternate routes (gemm.hip
 *   grouped_dispatch).
 */
int pli_flash_attn_fwd_variant(const void* q, const void* k, const void* v, void* o, int batch,
                               int heads, int kv_heads, int n_q, int n_kv, int head_dim,
                               const int64_t* strides, float scale, int causal, int dtype,
                               void* stream, int variant);
int pli_gemm_variant(const void* a, const void* b, void* c, const void* bias, int m, int n, int k,
                     int64_t lda, int64_t ldb, int64_t ldc, int trans_b, int dtype, void* stream,
                     int variant);
int pli_gemm_ws_variant(const void* a, const void* b, void* c, const void* bias, int m, int n,
                        int k, int64_t lda, int64_t ldb, int64_t ldc, int trans_b, int dtype,
                        void* workspace, size_t workspace_bytes, void* stream, int variant);
int pli_gemv_variant(const void* w, const void* x, void* y, int m, int k, int64_t ldw, int dtype,
                     void* stream, int variant);
int pli_attn_decode_variant(const void* q, const void* k, const void* v, void* o, int batch,
                            int heads, int kv_heads, int n_q, int n_kv, int head_dim,
                            const int64_t* strides, float scale, int causal, void* workspace,
                            size_t workspace_bytes, int dtype, void* stream, int mode,
                            int target_wgs);
int pli_gemm_swiglu_ws_variant(const void* x, const void* wg, const void* wu, void* h, int m, int n,
                               int k, int64_t ldx, int64_t ldwg, int64_t ldwu, int64_t ldh,
                               int dtype, void* workspace, size_t workspace_bytes, void* stream,
                               int variant);
int pli_gemm_grouped_variant(const void* x, const int32_t* gather, const void* const* w_ptrs,
                             const void* const* wu_ptrs, void* c, const int32_t* offsets,
                             int experts, int rows_bound, int n, int k, int64_t ldx, int64_t ldw,
                             int64_t ldc, int dtype, void* stream, int variant);

#if defined(__GNUC__) || defined(__clang__)
#pragma GCC visibility pop
#endif
#ifdef __cplusplus
}
#endif

#endif /* PLI_H */
