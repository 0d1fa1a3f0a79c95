// Mixture-of-experts routing and combine for gfx950.
//
// Replaces the per-expert Python loop of ch09/moe_layer.py:58-83 (boolean
// masks, x_flat[mask] gathers and masked += per expert and per top-k slot)
// and the router math of :18-33 (softmax, topk, renormalise):
//   pli_moe_route    one wave per token: softmax over the expert logits (fp32),
//                    top-k by wave arg-max, optional renormalisation, and a
//                    per-expert slot from an atomic counter; then an offsets
//                    scan and a scatter that builds, for the grouped GEMMs
//                    (pli_gemm_grouped), the permuted row -> token table and,
//                    for the combine, the (token, k) -> permuted row table.
//   pli_moe_combine  out[t] = sum_k w[t,k] * Y[pos[t,k]], fp32 accumulate in
//                    a fixed k order (deterministic, unlike scatter-add).
#include <cmath>
#include <type_traits>

#include "pli_common.h"

namespace pli {
namespace {

template <typename T>
__device__ __forceinline__ float load_val(const void* p, int64_t i) {
    if constexpr (std::is_same_v<T, float>) return reinterpret_cast<const float*>(p)[i];
    else return elem<T>::to_f32(T{reinterpret_cast<const uint16_t*>(p)[i]});
}

template <typename T>
__global__ __launch_bounds__(256) void moe_route_kernel(const void* __restrict__ logits, int64_t ld,
                                                        int T_, int E, int K, int normalize,
                                                        float* __restrict__ weights,
                                                        int* __restrict__ idx, int* __restrict__ slot,
                                                        int* __restrict__ counts) {
    const int lane = threadIdx.x & 63;
    const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (t >= T_) return;
    float v = lane < E ? load_val<T>(logits, (int64_t)t * ld + lane) : -INFINITY;
    const float m = wave_max(v);
    const float p = lane < E ? __expf(v - m) : 0.f;
    const float prob = p / wave_sum(p);
    bool taken = lane >= E;
    float wsum = 0.f, wk[8];
    int ek[8];
    for (int j = 0; j < K; ++j) {
        // arg-max over lanes not yet taken; ties -> lowest expert index
        float best = taken ? -1.f : prob;
        int bi = taken ? 64 : lane;
        for (int off = 32; off >= 1; off >>= 1) {
            const float ob = __shfl_xor(best, off, 64);
            const int oi = __shfl_xor(bi, off, 64);
            if (ob > best || (ob == best && oi < bi)) {
                best = ob;
                bi = oi;
            }
        }
        wk[j] = best;
        ek[j] = bi;
        wsum += best;
        if (lane == bi) taken = true;
    }
    if (lane < K) {
        float w = 0.f;
        int e = 0;
        for (int j = 0; j < K; ++j)
            if (j == lane) {
                w = wk[j];
                e = ek[j];
            }
        if (normalize) w = w / wsum;
        weights[(int64_t)t * K + lane] = w;
        idx[(int64_t)t * K + lane] = e;
        slot[(int64_t)t * K + lane] = atomicAdd(&counts[e], 1);
    }
}

__global__ void moe_offsets_kernel(const int* __restrict__ counts, int* __restrict__ offsets, int E) {
    if (threadIdx.x == 0) {
        int acc = 0;
        for (int e = 0; e < E; ++e) {
            offsets[e] = acc;
            acc += counts[e];
        }
        offsets[E] = acc;
    }
}

__global__ __launch_bounds__(256) void moe_scatter_kernel(const int* __restrict__ idx,
                                                          const int* __restrict__ slot,
                                                          const int* __restrict__ offsets,
                                                          int* __restrict__ pos,
                                                          int* __restrict__ gather, int TK, int K) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= TK) return;
    const int p = offsets[idx[i]] + slot[i];
    pos[i] = p;
    gather[p] = i / K;
}

template <typename T>
__global__ __launch_bounds__(256) void moe_combine_kernel(const uint16_t* __restrict__ Y, int64_t ldy,
                                                          const int* __restrict__ pos,
                                                          const float* __restrict__ w,
                                                          uint16_t* __restrict__ out, int64_t ldo,
                                                          int K, int H) {
    const int t = blockIdx.x;
    for (int c = threadIdx.x; c < H / 8; c += 256) {
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int j = 0; j < K; ++j) {
            const float wj = w[(int64_t)t * K + j];
            const i32x4 v = *reinterpret_cast<const i32x4*>(Y + (int64_t)pos[(int64_t)t * K + j] * ldy + 8 * c);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t u = (uint32_t)v[q];
                acc[2 * q] = fmaf(wj, elem<T>::to_f32(T{(uint16_t)(u & 0xffff)}), acc[2 * q]);
                acc[2 * q + 1] = fmaf(wj, elem<T>::to_f32(T{(uint16_t)(u >> 16)}), acc[2 * q + 1]);
            }
        }
        *reinterpret_cast<i32x4*>(out + (int64_t)t * ldo + 8 * c) =
            i32x4{(int)pack2<T>(acc[0], acc[1]), (int)pack2<T>(acc[2], acc[3]),
                  (int)pack2<T>(acc[4], acc[5]), (int)pack2<T>(acc[6], acc[7])};
    }
}

}  // namespace
}  // namespace pli

extern "C" int pli_moe_route(const void* logits, int64_t ld_logits, int tokens, int experts,
                             int top_k, int normalize, int dtype, float* weights,
                             int32_t* expert_idx, int32_t* pos, int32_t* gather, int32_t* offsets,
                             int32_t* workspace, void* stream) {
    using namespace pli;
    clear_error();
    // (per-token operands are empty, and may be NULL (pli.h), when tokens == 0;
    // offsets are still written: all zero)
    PLI_REQUIRE(offsets && workspace && (tokens == 0 || (logits && weights && expert_idx && pos && gather)),
                "pli_moe_route: null pointer");
    PLI_REQUIRE(tokens >= 0 && experts > 0 && experts <= 64 && top_k > 0 && top_k <= 8 &&
                    top_k <= experts && ld_logits >= experts,
                "pli_moe_route: bad shape tokens=%d experts=%d (<= 64) top_k=%d (<= 8)", tokens,
                experts, top_k);
    PLI_REQUIRE(dtype == PLI_F32 || dtype == PLI_F16 || dtype == PLI_BF16,
                "pli_moe_route: bad dtype %d", dtype);
    hipStream_t s = (hipStream_t)stream;
    int* counts = workspace;           // [experts]
    int* slot = workspace + experts;   // [tokens * top_k]
    hipError_t err = hipMemsetAsync(counts, 0, sizeof(int) * experts, s);
    if (err != hipSuccess) {
        set_error("pli_moe_route: %s", hipGetErrorString(err));
        return (int)err;
    }
    if (tokens > 0) {
        const dim3 grid((unsigned)cdiv(tokens, 4)), block(256);
        switch (dtype) {
            case PLI_F32:
                hipLaunchKernelGGL(moe_route_kernel<float>, grid, block, 0, s, logits, ld_logits, tokens,
                                   experts, top_k, normalize, weights, expert_idx, slot, counts);
                break;
            case PLI_F16:
                hipLaunchKernelGGL(moe_route_kernel<f16_t>, grid, block, 0, s, logits, ld_logits, tokens,
                                   experts, top_k, normalize, weights, expert_idx, slot, counts);
                break;
            default:
                hipLaunchKernelGGL(moe_route_kernel<bf16_t>, grid, block, 0, s, logits, ld_logits, tokens,
                                   experts, top_k, normalize, weights, expert_idx, slot, counts);
        }
    }
    hipLaunchKernelGGL(moe_offsets_kernel, dim3(1), dim3(64), 0, s, counts, offsets, experts);
    const int tk = tokens * top_k;
    if (tk > 0)
        hipLaunchKernelGGL(moe_scatter_kernel, dim3((unsigned)cdiv(tk, 256)), dim3(256), 0, s,
                           expert_idx, slot, offsets, pos, gather, tk, top_k);
    return launch_status("pli_moe_route");
}

extern "C" int pli_moe_combine(const void* y, int64_t ldy, const int32_t* pos, const float* weights,
                               void* out, int64_t ldo, int tokens, int top_k, int hidden, int dtype,
                               void* stream) {
    using namespace pli;
    clear_error();
    PLI_REQUIRE(tokens >= 0 && top_k > 0 && hidden > 0 && hidden % 8 == 0 && ldy % 8 == 0 &&
                    ldo % 8 == 0 && ldy >= hidden && ldo >= hidden && aligned16(y) && aligned16(out),
                "pli_moe_combine: bad shape / alignment (hidden %% 8 == 0, 16-byte rows)");
    PLI_REQUIRE(dtype == PLI_F16 || dtype == PLI_BF16, "pli_moe_combine: bf16/fp16 only");
    if (tokens == 0) return PLI_OK;  // (empty operands may be NULL, pli.h)
    PLI_REQUIRE(y && pos && weights && out, "pli_moe_combine: null pointer");
    hipStream_t s = (hipStream_t)stream;
    if (dtype == PLI_BF16)
        hipLaunchKernelGGL(moe_combine_kernel<bf16_t>, dim3((unsigned)tokens), dim3(256), 0, s,
                           (const uint16_t*)y, ldy, pos, weights, (uint16_t*)out, ldo, top_k, hidden);
    else
        hipLaunchKernelGGL(moe_combine_kernel<f16_t>, dim3((unsigned)tokens), dim3(256), 0, s,
                           (const uint16_t*)y, ldy, pos, weights, (uint16_t*)out, ldo, top_k, hidden);
    return launch_status("pli_moe_combine");
}
