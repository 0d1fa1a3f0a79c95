// gemm_w6: C = A B (+ bias) for bf16 / fp16, one wave per SIMD, K staged 64
// deep through VGPRs (reference ch03/gemm_benchmark.py:35-49, ch05 / ch09
// F.linear shapes; gfx950).
//
// gemm_w5's tile and LDS images (two 64 KiB slots, 128-B A / NT-B rows,
// 512-B NN-B rows, the same swizzles, the same fragment reads and MFMA
// chains), with the operands staged by global_load_dwordx4 into VGPRs and
// ds_write_b128 instead of LDS-DMA: the w5 no-DMA ablation still ran 15 %
// faster (profiles/r03/gemm/ab_w5_sweep.log), and hipBLASLt's kernel for
// these shapes (MT256x256x64, 4 waves of 128 x 128, 16x16 MFMAs) stages
// through VGPRs.  The swizzle moves from the global source address to the
// LDS write address.
//
// Per step S (128 MFMAs, two k32 halves), staging registers G holding step
// S+1's operand rows (loaded during step S-1):
//   half 0: MFMAs on (S, h0); in their gaps the (S, h1) fragments are read,
//           G is written to slot (S+1) % 2 (free since the barrier of step
//           S-1), then step S+2's rows are loaded into G;
//   lgkmcnt(0) + barrier: slot S+1 written everywhere, slot S's reads done;
//   half 1: MFMAs on (S, h1); in their gaps the (S+1, h0) fragments are read.
// A step's rows have 1.5 halves to arrive before they are written.
// Arithmetic: gemm_256's MFMA chains in k order, so outputs are bitwise those
// of gemm_256 / gemm_w4v / gemm_w5.
#include "gemm_w6.h"

#include <utility>

#include "pli_common.h"
#include "gemm_w4v_asm.h"

// A/B switches (tools/build_ab.sh); the defaults are the product
#ifndef W6_LD_START
#define W6_LD_START 33  // half-0 gap of the first global load (after the writes)
#endif
#ifndef W6_LD_STRIDE
#define W6_LD_STRIDE 2
#endif
#ifndef W6_LD_H1
#define W6_LD_H1 0  // 1: the global loads in half 1 instead
#endif

namespace pli {
namespace {

template <int... I, class Fn>
__device__ __forceinline__ void w6_for(std::integer_sequence<int, I...>, Fn&& fn) {
    (fn(std::integral_constant<int, I>{}), ...);
}
template <int N, class Fn> __device__ __forceinline__ void w6_sfor(Fn&& fn) {
    w6_for(std::make_integer_sequence<int, N>{}, fn);
}

__device__ __forceinline__ void w6_tile(int lb, int tiles_m, int tiles_n, int group_m, int& tm, int& tn) {
    const int width = group_m * tiles_n;
    const int first = (lb / width) * group_m;
    const int rows = min(tiles_m - first, group_m);
    const int r = lb % width;
    tm = first + r % rows;
    tn = r / rows;
}
__device__ __forceinline__ int w6_fnn(int k) { return 2 * ((k & 3) | (((k >> 3) & 1) << 2)); }

template <int OFF> __device__ __forceinline__ void w6_rd128(i32x4& d, uint32_t addr) {
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "n"(OFF));
}
struct W6Pair { i32x2 lo, hi; };
template <int OFF> __device__ __forceinline__ void w6_rdtr(W6Pair& d, uint32_t addr) {
    asm volatile("ds_read_b64_tr_b16 %0, %2 offset:%3\n\tds_read_b64_tr_b16 %1, %2 offset:%4"
                 : "=&v"(d.lo), "=&v"(d.hi) : "v"(addr), "n"(OFF), "n"(OFF + 2048));
}
template <int OFF> __device__ __forceinline__ void w6_wr128(uint32_t addr, const i32x4& v) {
    asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(addr), "v"(v), "n"(OFF) : "memory");
}
__device__ __forceinline__ void w6_ld128(i32x4& d, const uint16_t* base, uint32_t off) {
    asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(d) : "v"(off), "s"(base) : "memory");
}

template <typename T, bool TRANS_B, bool BIAS>
__global__ __launch_bounds__(256, 1) void gemm_w6(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bm,
                                                  uint16_t* __restrict__ C, const uint16_t* __restrict__ bias,
                                                  int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc,
                                                  int tiles_n, int nblocks, int group_m) {
    constexpr int IMG = 32768, SLOT = 2 * IMG;
    using BFrag = std::conditional_t<TRANS_B, i32x4, W6Pair>;
    __shared__ __attribute__((aligned(1024))) char smem[2 * SLOT];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 1, wc = wave & 1;
    int tm, tn;
    w6_tile(xcd_remap(blockIdx.x, nblocks), cdiv(M, 256), tiles_n, group_m, tm, tn);
    const int m0 = tm * 256, n0 = tn * 256;
    const int ks = K / 64;
    const uint32_t lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem;

    // ---- staging plan: wave w moves 8 KiB of each operand image per step,
    // 16 B per lane per load: A / NT-B rows 64w + 8i + (lane >> 3), 16-B chunk
    // lane & 7 (8 full 128-B rows per load); NN-B k-rows 16w + 2i + (lane >>
    // 5), chunk lane & 31 (2 x 512 B).  Rows past M / N re-read the last row.
    uint32_t aoff[8], boff[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int row = 64 * wave + 8 * i + (lane >> 3);
        aoff[i] = (uint32_t)(((int64_t)(min(m0 + row, M - 1) - m0) * lda + 8 * (lane & 7)) * 2);
        if constexpr (TRANS_B) {
            boff[i] = (uint32_t)(((int64_t)(min(n0 + row, N - 1) - n0) * ldb + 8 * (lane & 7)) * 2);
        } else {
            const int kr = 16 * wave + 2 * i + (lane >> 5);
            boff[i] = (uint32_t)(((int64_t)kr * ldb + min(n0 + 8 * (lane & 31), N - 8) - n0) * 2);
        }
    }
    const uint16_t* abase = A + (int64_t)m0 * lda;
    const uint16_t* bbase = TRANS_B ? Bm + (int64_t)n0 * ldb : Bm + n0;
    // LDS write addresses (slot 0): A / NT-B row r, chunk c at c ^ ((r >> 1)
    // & 7) -- loads i and i+2 differ by 16 rows (+2 KiB, same XOR), so two
    // bases; NN-B k-row kr, chunk c at c ^ fnn(kr) -- loads i and i+2 differ
    // by 4 k-rows (+2 KiB, same fnn), four bases
    uint32_t wa[2], wb[TRANS_B ? 2 : 4];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int row = 64 * wave + 8 * i + (lane >> 3);
        const int c = (lane & 7) ^ ((row >> 1) & 7);
        wa[i] = lds0 + (uint32_t)(row * 128 + (c << 4));
        if constexpr (TRANS_B) wb[i] = lds0 + IMG + (uint32_t)(row * 128 + (c << 4));
    }
    if constexpr (!TRANS_B) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {  // loads i = (q & 1) + 4 (q >> 1) (+2)
            const int i = (q & 1) + 4 * (q >> 1);
            const int kr = 16 * wave + 2 * i + (lane >> 5);
            const int c = (lane & 31) ^ w6_fnn(kr);
            wb[q] = lds0 + IMG + (uint32_t)(kr * 512 + (c << 4));
        }
    }

    i32x4 G[16];  // one step's rows of this wave: 0-7 A, 8-15 B
    // load j of K step s (past the last step: a reload of the last step)
    auto gload = [&](auto j_tag, int s) __attribute__((always_inline)) {
        constexpr int j = decltype(j_tag)::value, i = j % 8;
        const int sc = min(s, ks - 1);
        const uint16_t* src = j < 8 ? abase + sc * 64 : (TRANS_B ? bbase + sc * 64 : bbase + (int64_t)sc * 64 * ldb);
        w6_ld128(G[j], src, j < 8 ? aoff[i] : boff[i]);
    };
    // the rows in G have landed (as far as hipcc knows, written here)
    auto gwait = [&]() __attribute__((always_inline)) {
        asm volatile("s_waitcnt vmcnt(0)"
                     : "+v"(G[0]), "+v"(G[1]), "+v"(G[2]), "+v"(G[3]), "+v"(G[4]), "+v"(G[5]), "+v"(G[6]),
                       "+v"(G[7]), "+v"(G[8]), "+v"(G[9]), "+v"(G[10]), "+v"(G[11]), "+v"(G[12]), "+v"(G[13]),
                       "+v"(G[14]), "+v"(G[15])::"memory");
    };
    // write j of G into the slot at byte offset so
    auto gwrite = [&](auto j_tag, uint32_t so) __attribute__((always_inline)) {
        constexpr int j = decltype(j_tag)::value, i = j % 8;
        if constexpr (j < 8) {
            w6_wr128<(i / 2) * 2048>(wa[i & 1] + so, G[j]);
        } else if constexpr (TRANS_B) {
            w6_wr128<(i / 2) * 2048>(wb[i & 1] + so, G[j]);
        } else {
            constexpr int q = (i & 1) + 2 * (i >= 4 ? 1 : 0), extra = ((i % 4) / 2) * 2048;
            w6_wr128<extra>(wb[q] + so, G[j]);
        }
    };

    // ---- fragment read addresses (gemm_w5's)
    const int r16 = lane & 15, h4 = lane >> 4;
    uint32_t a_rd[2], b_rd[TRANS_B ? 2 : 8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int ch = (4 * h + h4) ^ ((r16 >> 1) & 7);
        a_rd[h] = lds0 + (uint32_t)((wr * 128 + r16) * 128 + (ch << 4));
        if constexpr (TRANS_B) b_rd[h] = lds0 + IMG + (uint32_t)((wc * 128 + r16) * 128 + (ch << 4));
    }
    if constexpr (!TRANS_B) {
        const int q = (lane >> 2) & 3, p = lane & 3, kr = 8 * h4 + q;
#pragma unroll
        for (int ni = 0; ni < 8; ++ni) {
            const int c = wc * 16 + 2 * ni + (p >> 1);
            b_rd[ni] = lds0 + IMG + (uint32_t)(kr * 512 + ((c ^ w6_fnn(kr)) << 4) + (p & 1) * 8);
        }
    }

    i32x4 fa[2][8];
    BFrag fb[2][8];
    auto frag_read = [&](auto h_tag, auto i_tag, uint32_t so) __attribute__((always_inline)) {
        constexpr int H = decltype(h_tag)::value, I = decltype(i_tag)::value;
        if constexpr (I < 8) {
            w6_rd128<I * 2048>(fa[H][I], a_rd[H] + so);
        } else if constexpr (TRANS_B) {
            w6_rd128<(I - 8) * 2048>(fb[H][I - 8], b_rd[H] + so);
        } else {
            w6_rdtr<H * 16384>(fb[H][I - 8], b_rd[I - 8] + so);
        }
    };
    auto frag_wait = [&](auto p_tag) __attribute__((always_inline)) {
        constexpr int P = decltype(p_tag)::value;
        if constexpr (TRANS_B) {
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(fa[P][0]), "+v"(fa[P][1]), "+v"(fa[P][2]), "+v"(fa[P][3]), "+v"(fa[P][4]),
                           "+v"(fa[P][5]), "+v"(fa[P][6]), "+v"(fa[P][7]), "+v"(fb[P][0]), "+v"(fb[P][1]),
                           "+v"(fb[P][2]), "+v"(fb[P][3]), "+v"(fb[P][4]), "+v"(fb[P][5]), "+v"(fb[P][6]),
                           "+v"(fb[P][7])::"memory");
        } else {
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(fa[P][0]), "+v"(fa[P][1]), "+v"(fa[P][2]), "+v"(fa[P][3]), "+v"(fa[P][4]),
                           "+v"(fa[P][5]), "+v"(fa[P][6]), "+v"(fa[P][7])::"memory");
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(fb[P][0].lo), "+v"(fb[P][0].hi), "+v"(fb[P][1].lo), "+v"(fb[P][1].hi),
                           "+v"(fb[P][2].lo), "+v"(fb[P][2].hi), "+v"(fb[P][3].lo), "+v"(fb[P][3].hi),
                           "+v"(fb[P][4].lo), "+v"(fb[P][4].hi), "+v"(fb[P][5].lo), "+v"(fb[P][5].hi),
                           "+v"(fb[P][6].lo), "+v"(fb[P][6].hi), "+v"(fb[P][7].lo), "+v"(fb[P][7].hi)::"memory");
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    auto bop = [&](const BFrag& f) __attribute__((always_inline)) {
        if constexpr (TRANS_B) return f;
        else return i32x4{f.lo.x, f.lo.y, f.hi.x, f.hi.y};
    };
    // 64 MFMAs on buffer P; in their gaps (RD) 16 fragment reads of half RH
    // (slot offset rso, one every 2 gaps from gap 0), (WR) the 16 writes of G
    // into slot wso (odd gaps 1-31, after the rows landed), (LD) the 16 loads
    // of step ls into G (after the writes read it)
    auto half = [&](auto p_tag, auto rd_tag, auto rh_tag, uint32_t rso, auto wr_tag, uint32_t wso, auto ld_tag,
                    int ls) __attribute__((always_inline)) {
        constexpr int P = decltype(p_tag)::value, RH = decltype(rh_tag)::value;
        constexpr bool RD = decltype(rd_tag)::value, WR = decltype(wr_tag)::value, LD = decltype(ld_tag)::value;
        if constexpr (WR) gwait();
        w6_sfor<64>([&](auto JJ) {
            constexpr int J = JJ, ni = J / 8, mi = J % 8;
            if constexpr (std::is_same_v<T, bf16_t>) w4v::mfma_bf16<J>(bop(fb[P][ni]), fa[P][mi]);
            else w4v::mfma_f16<J>(bop(fb[P][ni]), fa[P][mi]);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (RD && J % 2 == 0 && J / 2 < 16)
                frag_read(std::integral_constant<int, RH>{}, std::integral_constant<int, J / 2>{}, rso);
            if constexpr (WR && J % 2 == 1 && J / 2 < 16) gwrite(std::integral_constant<int, J / 2>{}, wso);
            // the writes have read G before it is reloaded
            if constexpr (LD && J == W6_LD_START - 1) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            constexpr int D = J - W6_LD_START;
            if constexpr (LD && D >= 0 && D % W6_LD_STRIDE == 0 && D / W6_LD_STRIDE < 16)
                gload(std::integral_constant<int, D / W6_LD_STRIDE>{}, ls);
            __builtin_amdgcn_sched_barrier(0);
        });
    };

    // ---- prologue: accumulators 0; step 0 written, step 1 in G; (0, h0)
    // fragments
    w4v::acc_zero();
    w6_sfor<16>([&](auto J) { gload(J, 0); });
    gwait();
    w6_sfor<16>([&](auto J) { gwrite(J, 0u); });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    w6_sfor<16>([&](auto J) { gload(J, 1); });
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    w6_sfor<16>([&](auto I) { frag_read(std::integral_constant<int, 0>{}, I, 0u); });
    frag_wait(std::integral_constant<int, 0>{});

    using Z = std::integral_constant<int, 0>;
    using O = std::integral_constant<int, 1>;
    auto step = [&](int s, auto more_tag) __attribute__((always_inline)) {
        constexpr bool MORE = decltype(more_tag)::value;  // a step s+1 follows
        const uint32_t so = (uint32_t)(s & 1) * SLOT, sn = (uint32_t)((s + 1) & 1) * SLOT;
        // G (step s+1) -> slot s+1, then step s+2's rows -> G
        half(Z{}, std::true_type{}, O{}, so, std::true_type{}, sn, std::bool_constant<!W6_LD_H1>{}, s + 2);
        frag_wait(O{});  // also: the writes of G landed
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        half(O{}, more_tag, Z{}, sn, std::false_type{}, 0u, std::bool_constant<(bool)W6_LD_H1>{}, s + 2);
        if constexpr (MORE) frag_wait(Z{});
    };
    int s = 0;
    for (; s + 1 < ks; ++s) step(s, std::true_type{});
    step(s, std::false_type{});

    // ---- epilogue (gemm_w5's)
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // dead reloads landed
    __builtin_amdgcn_s_barrier();                                 // every wave is done with the slots
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");              // last MFMA -> accumulator reads
    char* reg = smem + wave * 32768;
    w6_sfor<64>([&](auto JJ) {
        constexpr int J = JJ, ni = J / 8, mi = J % 8;
        f32x4 v;
        w4v::acc_read<J>(v);
        const int n = n0 + 128 * wc + 16 * ni + 4 * h4;
        if constexpr (BIAS) {
            if (n < N) {
                const i32x2 bb = *reinterpret_cast<const i32x2*>(bias + n);
                v[0] += elem<T>::to_f32(T{(uint16_t)(bb.x & 0xffff)});
                v[1] += elem<T>::to_f32(T{(uint16_t)((uint32_t)bb.x >> 16)});
                v[2] += elem<T>::to_f32(T{(uint16_t)(bb.y & 0xffff)});
                v[3] += elem<T>::to_f32(T{(uint16_t)((uint32_t)bb.y >> 16)});
            }
        }
        const i32x2 pk = i32x2{(int)pack2<T>(v[0], v[1]), (int)pack2<T>(v[2], v[3])};
        const int row = 16 * mi + r16, chunk = 2 * ni + (h4 >> 1);
        *reinterpret_cast<i32x2*>(reg + row * 256 + ((chunk ^ r16) << 4) + (h4 & 1) * 8) = pk;
    });
    {
        const int c = lane & 15;
        const int n = n0 + 128 * wc + 8 * c;
#pragma unroll 8
        for (int it = 0; it < 32; ++it) {
            const int row = 4 * it + h4;
            const i32x4 v = *reinterpret_cast<const i32x4*>(reg + row * 256 + ((c ^ (row & 15)) << 4));
            const int m = m0 + 128 * wr + row;
            if (m < M && n < N) *reinterpret_cast<i32x4*>(C + (int64_t)m * ldc + n) = v;
        }
    }
}

}  // namespace

bool gemm_w6_ok(int m, int n, int k, int64_t lda, int64_t ldb, int64_t ldc, int trans_b) {
    (void)m;
    (void)ldc;
    // per-lane load offsets are 32-bit: 256 rows (NN: 64 k-rows) of the operand
    return k >= 64 && k % 64 == 0 && n % 8 == 0 && n >= 8 && lda * 2 * 256 < (1ll << 31) &&
           ldb * 2 * (trans_b ? 256 : 64) < (1ll << 31);
}

int launch_gemm_w6(const void* a, const void* b, void* c, const void* bias, int m, int n, int k, int64_t lda,
                   int64_t ldb, int64_t ldc, int trans_b, int is_bf16, hipStream_t stream, int group_m) {
    PLI_REQUIRE(gemm_w6_ok(m, n, k, lda, ldb, ldc, trans_b), "gemm_w6: shape m=%d n=%d k=%d not supported", m, n,
                k);
    PLI_REQUIRE(group_m >= 1, "gemm_w6: group_m must be >= 1");
    const int tiles_m = cdiv(m, 256), tiles_n = cdiv(n, 256);
    const int64_t nb = (int64_t)tiles_m * tiles_n;
    PLI_REQUIRE(nb < (1ll << 31), "gemm_w6: grid too large");
    const auto* A = (const uint16_t*)a;
    const auto* B = (const uint16_t*)b;
    auto* Cc = (uint16_t*)c;
    const auto* bs = (const uint16_t*)bias;
    const dim3 gr((unsigned)nb), blk(256);
#define W6_LAUNCH(T, TB, BI)                                                                                        \
    hipLaunchKernelGGL((gemm_w6<T, TB, BI>), gr, blk, 0, stream, A, B, Cc, bs, m, n, k, lda, ldb, ldc, tiles_n, \
                       (int)nb, group_m)
    if (is_bf16) {
        if (trans_b) { if (bias) W6_LAUNCH(bf16_t, true, true); else W6_LAUNCH(bf16_t, true, false); }
        else { if (bias) W6_LAUNCH(bf16_t, false, true); else W6_LAUNCH(bf16_t, false, false); }
    } else {
        if (trans_b) { if (bias) W6_LAUNCH(f16_t, true, true); else W6_LAUNCH(f16_t, true, false); }
        else { if (bias) W6_LAUNCH(f16_t, false, true); else W6_LAUNCH(f16_t, false, false); }
    }
#undef W6_LAUNCH
    return launch_status("gemm_w6");
}

}  // namespace pli
