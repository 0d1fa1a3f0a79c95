// gemm_w4v: C = A B (+ bias) for bf16 / fp16, one wave per SIMD (reference
// ch03/gemm_benchmark.py:35-49, ch05 / ch09 F.linear shapes; gfx950).
//
// The structure of attn_fwd_v12 (flash_v12.hip) applied to the GEMM tile:
//   * workgroup = 4 waves (one per SIMD, each owning the whole 512-entry
//     register file), output tile 256 x 256, wave (wr, wc) = 128 x 128 of it;
//   * the wave's C^T lives in the accumulator file, all 256 AGPRs, named
//     literally by the inline-asm MFMAs of gemm_w4v_asm.h (block (ni, mi) of
//     16 x 16 in a[4(8 ni + mi) : +3]); C^T = B^T A^T, so a lane owns one
//     output row and 4 consecutive columns per block (8-byte stores);
//   * v_mfma_f32_16x16x32 (the shape the chip clocks highest under load,
//     MI355X_MICROARCH.md 'DVFS give-back'): 64 MFMAs per 32-deep K step;
//   * K arrives 32 deep per step by LDS-DMA (global_load_lds_dwordx4, 1 KiB
//     per wave-instruction, lane-linear LDS, swizzle on the SOURCE address)
//     into a 5-slot ring of 32 KiB slots (A image + B image), four steps
//     ahead of the MFMAs that consume it: the DMA of step s+4 goes out during
//     step s into the slot of step s-1, whose fragments every wave read
//     during step s-2 -- before the barrier of step s-1;
//   * the next step's fragments (8 A + 8 B reads) are read during the current
//     step's MFMAs, one per gap; one counted vmcnt + one barrier per step.
//
// LDS images (per slot):
//   A, NT-B: [256 rows][32 k] (64-B rows), 16-B chunk c of row r stored at
//            chunk c ^ 3 * ((r >> 3) & 1): each ds_read_b128 lane group
//            ({0-3,12-15,20-27}, ... MI355X_MICROARCH.md LDS table) covers the
//            16 16-B bank slots of a 256-B bank row once.
//   NN-B:    [32 k][256 n] (512-B rows), chunk c of k-row k at c ^ fnn(k)
//            (gemm.hip's g2_fnn): the transposed ds_read_b64_tr_b16 pairs of
//            each 32-lane group land on 16 distinct slot pairs.
// Arithmetic: every output is one chain of MFMAs over K in increasing order,
// 32 k per MFMA -- the order of gemm_256 (variant 2), so outputs are bitwise
// those of that kernel.
#include "gemm_w4v.h"

#include <utility>

#include "pli_common.h"
#include "gemm_w4v_asm.h"

// A/B switches (tools/build_ab.sh); the defaults are the product
#ifndef W4_DMA_START
#define W4_DMA_START 20  // gap of the step's first DMA piece
#endif
#ifndef W4_DMA_STRIDE
#define W4_DMA_STRIDE 5  // gaps between DMA pieces
#endif
#ifndef W4_RD_STRIDE
#define W4_RD_STRIDE 1  // gaps between fragment reads
#endif
// ablations (timing diagnostics only, results wrong): drop one kind of work
#ifndef W4_ABL_DMA
#define W4_ABL_DMA 0
#endif
#ifndef W4_ABL_BAR
#define W4_ABL_BAR 0
#endif
#ifndef W4_ABL_VMW
#define W4_ABL_VMW 0
#endif
#ifndef W4_ABL_RD
#define W4_ABL_RD 0
#endif
#ifndef W4_ABL_EPI
#define W4_ABL_EPI 0
#endif
#ifndef W4_ABL_DMAW0
#define W4_ABL_DMAW0 0  // only wave 0 issues its DMA pieces
#endif
#ifndef W4_ABL_NOB
#define W4_ABL_NOB 0  // no B pieces
#endif
#ifndef W4_ABL_LINES
#define W4_ABL_LINES 0  // A / NT-B pieces as 8 rows x 128 B (wrong data: DMA cost vs cache lines per piece)
#endif
#ifndef W4_EPI_LDS
#define W4_EPI_LDS 1  // epilogue through LDS: 16-B row stores (else 8-B stores from the accumulators)
#endif
#ifndef W4_DMA_IMM
#define W4_DMA_IMM 0  // one M0 write per 4 pieces, pieces 1-3 by instruction offset
#endif

namespace pli {
namespace {

template <int... I, class Fn>
__device__ __forceinline__ void w4_for(std::integer_sequence<int, I...>, Fn&& fn) {
    (fn(std::integral_constant<int, I>{}), ...);
}
template <int N, class Fn> __device__ __forceinline__ void w4_sfor(Fn&& fn) {
    w4_for(std::make_integer_sequence<int, N>{}, fn);
}

// tile order: bands of group_m tile rows swept column by column (gemm.hip
// g2_tile), after the XCD remap
__device__ __forceinline__ void w4_tile(int lb, int tiles_m, int tiles_n, int group_m, int& tm, int& tn) {
    if (group_m <= 0) {
        tm = lb / tiles_n;
        tn = lb % tiles_n;
        return;
    }
    const int width = group_m * tiles_n;
    const int first = (lb / width) * group_m;
    const int rows = min(tiles_m - first, group_m);
    const int r = lb % width;
    tm = first + r % rows;
    tn = r / rows;
}
__device__ __forceinline__ int w4_fnn(int k) { return 2 * ((k & 3) | (((k >> 3) & 1) << 2)); }

template <int OFF> __device__ __forceinline__ void w4_rd128(i32x4& d, uint32_t addr) {
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "n"(OFF));
}
struct W4Pair { i32x2 lo, hi; };
// NN B^T fragment: two transposed reads, k rows +0..3 and +4..7 (2 KiB apart)
__device__ __forceinline__ void w4_rdtr(W4Pair& d, uint32_t addr) {
    asm volatile("ds_read_b64_tr_b16 %0, %2\n\tds_read_b64_tr_b16 %1, %2 offset:2048"
                 : "=&v"(d.lo), "=&v"(d.hi) : "v"(addr));
}

template <typename T, bool TRANS_B, bool BIAS>
__global__ __launch_bounds__(256, 1) void gemm_w4v(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bm,
                                                   uint16_t* __restrict__ C, const uint16_t* __restrict__ bias,
                                                   int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc,
                                                   int tiles_n, int nblocks, int group_m) {
    constexpr int IMG = 16384, SLOT = 2 * IMG, NS = 5;
    using BFrag = std::conditional_t<TRANS_B, i32x4, W4Pair>;
    __shared__ __attribute__((aligned(1024))) char smem[NS * SLOT];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 1, wc = wave & 1;
    int tm, tn;
    w4_tile(xcd_remap(blockIdx.x, nblocks), cdiv(M, 256), tiles_n, group_m, tm, tn);
    const int m0 = tm * 256, n0 = tn * 256;
    const int ks = K / 32;
    const uint32_t lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem;

    // ---- LDS-DMA plan: wave w stages 4 KiB of each operand image per step
    // (4 pieces of 1 KiB): A / NT-B rows 64w .. 64w+63 (16 rows x 64 B per
    // piece), NN-B k-rows 8w .. 8w+7 (2 rows x 512 B per piece).  Per-lane
    // byte offsets from the tile's base; rows past M / N re-read the last row
    // (their outputs are never stored).
    uint32_t aoff[4], boff[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = W4_ABL_LINES ? 64 * wave + 16 * i + (lane >> 3) : 64 * wave + 16 * i + (lane >> 2);
        const int c = W4_ABL_LINES ? (lane & 7) : (lane & 3) ^ (3 * ((row >> 3) & 1));
        aoff[i] = (uint32_t)(((int64_t)(min(m0 + row, M - 1) - m0) * lda + 8 * c) * 2);
        if constexpr (TRANS_B) {
            boff[i] = (uint32_t)(((int64_t)(min(n0 + row, N - 1) - n0) * ldb + 8 * c) * 2);
        } else {
            const int kr = 8 * wave + 2 * i + (lane >> 5);
            const int cn = (lane & 31) ^ w4_fnn(kr);
            boff[i] = (uint32_t)(((int64_t)kr * ldb + min(n0 + 8 * cn, N - 8) - n0) * 2);
        }
    }
    const uint16_t* abase = A + (int64_t)m0 * lda;
    const uint16_t* bbase = TRANS_B ? Bm + (int64_t)n0 * ldb : Bm + n0;
    auto dma1 = [&](const uint16_t* src, uint32_t off, uint32_t lds) __attribute__((always_inline)) {
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(lds), "v"(off), "s"(src)
                     : "memory");
    };
    // DMA piece j (0-3 A, 4-7 B) of K step s (past the last step: a reload of
    // the last step into the dead slot, so every step issues the same count)
    // W4_DMA_IMM: piece i of a group of 4 reaches its LDS kilobyte through
    // the instruction offset i * 1024, which the hardware adds to the global
    // address too -- the scalar base is biased by -i * 1024 bytes instead
    auto dma_next = [&](auto i_tag, const uint16_t* src, uint32_t off) __attribute__((always_inline)) {
        constexpr int i = decltype(i_tag)::value;
        asm volatile("global_load_lds_dwordx4 %0, %1 offset:%2" ::"v"(off),
                     "s"(reinterpret_cast<const char*>(src) - 1024 * i), "n"(1024 * i) : "memory");
    };
    auto dma_piece = [&](auto j_tag, int s) __attribute__((always_inline)) {
        constexpr int j = decltype(j_tag)::value, i = j % 4;
        if (W4_ABL_DMAW0 && wave != 0) return;
        const int sc = min(s, ks - (W4_ABL_LINES ? 2 : 1));  // (ABL_LINES pieces read 64 k: stay in bounds)
        const uint32_t slot = lds0 + (uint32_t)(s % NS) * SLOT + (uint32_t)wave * 4096 + (W4_DMA_IMM ? 0 : i * 1024);
        const uint16_t* src = j < 4 ? abase + sc * 32 : (TRANS_B ? bbase + sc * 32 : bbase + (int64_t)sc * 32 * ldb);
        const uint32_t off = j < 4 ? aoff[i] : boff[i];
        if constexpr (W4_ABL_NOB && j >= 4) return;
        if constexpr (W4_DMA_IMM && i > 0) dma_next(std::integral_constant<int, i>{}, src, off);
        else dma1(src, off, slot + (j < 4 ? 0 : IMG));
    };

    // ---- fragment read addresses (slot 0; + slot * SLOT per step)
    const int r16 = lane & 15, h4 = lane >> 4;
    const uint32_t a_rd = lds0 + (uint32_t)((wr * 128 + r16) * 64 + ((h4 ^ (3 * ((r16 >> 3) & 1))) << 4));
    uint32_t b_rd[TRANS_B ? 1 : 8];
    if constexpr (TRANS_B) {
        b_rd[0] = lds0 + IMG + (uint32_t)((wc * 128 + r16) * 64 + ((h4 ^ (3 * ((r16 >> 3) & 1))) << 4));
    } else {
        const int q = (lane >> 2) & 3, p = lane & 3, kr = 8 * h4 + q;
#pragma unroll
        for (int ni = 0; ni < 8; ++ni) {
            const int c = wc * 16 + 2 * ni + (p >> 1);
            b_rd[ni] = lds0 + IMG + (uint32_t)(kr * 512 + ((c ^ w4_fnn(kr)) << 4) + (p & 1) * 8);
        }
    }

    i32x4 fa[2][8];
    BFrag fb[2][8];
    // fragment read I (0-7 A, 8-15 B) of the step whose slot is at byte
    // offset so, into buffer P
    auto frag_read = [&](auto p_tag, auto i_tag, uint32_t so) __attribute__((always_inline)) {
        constexpr int P = decltype(p_tag)::value, I = decltype(i_tag)::value;
        if constexpr (I < 8) {
            w4_rd128<I * 1024>(fa[P][I], a_rd + so);
        } else if constexpr (TRANS_B) {
            w4_rd128<(I - 8) * 1024>(fb[P][I - 8], b_rd[0] + so);
        } else {
            w4_rdtr(fb[P][I - 8], b_rd[I - 8] + so);
        }
    };
    // the fragments of buffer P have landed (as far as hipcc knows, written here)
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

    // ---- prologue: accumulators 0, K steps 0-3 in flight, step 0's fragments
    w4v::acc_zero();
    w4_sfor<4>([&](auto S) { w4_sfor<8>([&](auto J) { dma_piece(J, S); }); });
    asm volatile("s_waitcnt vmcnt(24)" ::: "memory");  // step 0 (this wave's pieces)
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    w4_sfor<16>([&](auto I) { frag_read(std::integral_constant<int, 0>{}, I, 0u); });
    frag_wait(std::integral_constant<int, 0>{});

    // ---- step s: 64 MFMAs on buffer P; in their gaps (READ) the next step's
    // 16 fragment reads into buffer 1-P, then the 8 DMA pieces of step s+4
    auto step = [&](auto p_tag, auto rd_tag, int s) __attribute__((always_inline)) {
        constexpr int P = decltype(p_tag)::value;
        constexpr bool RD = decltype(rd_tag)::value;
        // step s+1's slot landed: of the pieces issued after it (steps s+2,
        // s+3) 16 may still be in flight
        if (!W4_ABL_VMW) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        if (!W4_ABL_BAR) __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t so = (uint32_t)((s + 1) % NS) * SLOT;
        w4_sfor<64>([&](auto JJ) {
            constexpr int J = JJ, ni = J / 8, mi = J % 8;
            if constexpr (std::is_same_v<T, bf16_t>) w4v::mfma_bf16<J>(bop(fb[P][ni]), fa[P][mi]);
            else w4v::mfma_f16<J>(bop(fb[P][ni]), fa[P][mi]);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (RD && !W4_ABL_RD && J % W4_RD_STRIDE == 0 && J / W4_RD_STRIDE < 16)
                frag_read(std::integral_constant<int, 1 - P>{}, std::integral_constant<int, J / W4_RD_STRIDE>{}, so);
            constexpr int D = J - W4_DMA_START;
            if constexpr (!W4_ABL_DMA && D >= 0 && D % W4_DMA_STRIDE == 0 && D / W4_DMA_STRIDE < 8)
                dma_piece(std::integral_constant<int, D / W4_DMA_STRIDE>{}, s + 4);
            __builtin_amdgcn_sched_barrier(0);
        });
        if constexpr (RD) frag_wait(std::integral_constant<int, 1 - P>{});
    };

    int s = 0;
    for (; s + 2 < ks; s += 2) {
        step(std::integral_constant<int, 0>{}, std::true_type{}, s);
        step(std::integral_constant<int, 1>{}, std::true_type{}, s + 1);
    }
    if (s + 1 < ks) {
        step(std::integral_constant<int, 0>{}, std::true_type{}, s);
        step(std::integral_constant<int, 1>{}, std::false_type{}, s + 1);
    } else {
        step(std::integral_constant<int, 0>{}, std::false_type{}, s);
    }

    // ---- epilogue: accumulator block (ni, mi) holds C[m][n .. n+3] with
    // m = m0 + 128 wr + 16 mi + (lane & 15), n = n0 + 128 wc + 16 ni + 4 (lane >> 4)
    // W4_EPI_LDS: each wave packs its 128 x 128 tile into its own 32 KiB of
    // LDS ([row][256 B], 16-B chunk c of row r at c ^ (r & 15): the 16 rows
    // of a ds_write_b64 lane group hit 16 distinct bank slots) and stores it
    // back as whole 256-B row segments, 16 B per lane: 32 dwordx4 stores per
    // wave instead of 64 dwordx2 (the store tail is issue-bound)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // dead-slot reloads landed
    if constexpr (W4_EPI_LDS) __builtin_amdgcn_s_barrier();  // every wave is done with the ring
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");         // last MFMA -> accumulator reads
    char* reg = smem + wave * 32768;
    w4_sfor<64>([&](auto JJ) {
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
        if constexpr (W4_EPI_LDS) {
            const int row = 16 * mi + r16, chunk = 2 * ni + (h4 >> 1);
            *reinterpret_cast<i32x2*>(reg + row * 256 + ((chunk ^ r16) << 4) + (h4 & 1) * 8) = pk;
        } else {
            const int m = m0 + 128 * wr + 16 * mi + r16;
            if (m < M && n < N && !W4_ABL_EPI) *reinterpret_cast<i32x2*>(C + (int64_t)m * ldc + n) = pk;
        }
    });
    if constexpr (W4_EPI_LDS) {
        // row 4 it + (lane >> 4), chunk lane & 15 (8 columns)
        const int c = lane & 15;
        const int n = n0 + 128 * wc + 8 * c;
#pragma unroll 8
        for (int it = 0; it < 32; ++it) {
            const int row = 4 * it + h4;
            const i32x4 v = *reinterpret_cast<const i32x4*>(reg + row * 256 + ((c ^ (row & 15)) << 4));
            const int m = m0 + 128 * wr + row;
            if (m < M && n < N && !W4_ABL_EPI) *reinterpret_cast<i32x4*>(C + (int64_t)m * ldc + n) = v;
        }
    }
}

}  // namespace

bool gemm_w4v_ok(int m, int n, int k, int64_t lda, int64_t ldb, int64_t ldc, int trans_b) {
    (void)m;
    (void)ldc;
    // per-lane DMA offsets are 32-bit: 256 rows (NN: 32 k-rows) of the operand
    return k >= 32 && k % 32 == 0 && n % 8 == 0 && n >= 8 && lda * 2 * 256 < (1ll << 31) &&
           ldb * 2 * (trans_b ? 256 : 32) < (1ll << 31);
}

int launch_gemm_w4v(const void* a, const void* b, void* c, const void* bias, int m, int n, int k, int64_t lda,
                    int64_t ldb, int64_t ldc, int trans_b, int is_bf16, hipStream_t stream, int group_m) {
    PLI_REQUIRE(gemm_w4v_ok(m, n, k, lda, ldb, ldc, trans_b), "gemm_w4v: shape m=%d n=%d k=%d not supported", m,
                n, k);
    const int tiles_m = cdiv(m, 256), tiles_n = cdiv(n, 256);
    const int64_t nb = (int64_t)tiles_m * tiles_n;
    PLI_REQUIRE(nb < (1ll << 31), "gemm_w4v: grid too large");
    const auto* A = (const uint16_t*)a;
    const auto* B = (const uint16_t*)b;
    auto* Cc = (uint16_t*)c;
    const auto* bs = (const uint16_t*)bias;
    const dim3 gr((unsigned)nb), blk(256);
#define W4V_LAUNCH(T, TB, BI)                                                                                        \
    hipLaunchKernelGGL((gemm_w4v<T, TB, BI>), gr, blk, 0, stream, A, B, Cc, bs, m, n, k, lda, ldb, ldc, tiles_n, \
                       (int)nb, group_m)
    if (is_bf16) {
        if (trans_b) { if (bias) W4V_LAUNCH(bf16_t, true, true); else W4V_LAUNCH(bf16_t, true, false); }
        else { if (bias) W4V_LAUNCH(bf16_t, false, true); else W4V_LAUNCH(bf16_t, false, false); }
    } else {
        if (trans_b) { if (bias) W4V_LAUNCH(f16_t, true, true); else W4V_LAUNCH(f16_t, true, false); }
        else { if (bias) W4V_LAUNCH(f16_t, false, true); else W4V_LAUNCH(f16_t, false, false); }
    }
#undef W4V_LAUNCH
    return launch_status("gemm_w4v");
}

}  // namespace pli
