// gemm_w5: C = A B (+ bias) for bf16 / fp16, one wave per SIMD, K staged 64
// deep (reference ch03/gemm_benchmark.py:35-49, ch05 / ch09 F.linear shapes;
// gfx950).
//
// gemm_w4v's tile (256 x 256, 4 waves of 128 x 128 C^T in the accumulator
// file, v_mfma_f32_16x16x32 named by gemm_w4v_asm.h), with the operands
// staged 64 k deep instead of 32.  The w4v ablation (profiles/r03/gemm/)
// put the LDS-DMA issue first among its costs (NT 8192^3: 1369 TF/s, 1700
// with no DMA), and its cost follows the cache lines a piece touches: the
// same 1 KiB piece as 8 rows x 128 B instead of 16 rows x 64 B ran 1495.
// At 64 k a row of A (and of NT-B) is one 128-B line.
//
// LDS: two 64 KiB slots (A image then B image, 32 KiB each), step S in slot
// S % 2.  Per step (128 MFMAs, two k32 halves; W5_SPLIT, the default):
//   half 0: MFMAs on the (S, h0) fragments; in the first 16 gaps the (S, h1)
//           fragments are read; after gap 24 they are waited for and the
//           workgroup meets (every wave is done reading slot S), and 5 of
//           step S+2's 16 DMA pieces go into slot S in gaps 28-56;
//   s_waitcnt vmcnt(5) + barrier: step S+1's pieces landed everywhere;
//   half 1: MFMAs on (S, h1); in their gaps the (S+1, h0) fragments are read
//           from slot S+1 (every third gap) and the other 11 DMA pieces of
//           step S+2 issue (gaps 1, 7, ... 61).
// (W5_SPLIT 0, round 3: all 16 pieces in half 1 beside the reads, one
// barrier per step; the split is bitwise the same and 0.5-2 % faster,
// profiles/r04/gemm/ab_w5_split.log.)  Past the last step the DMA re-loads
// the last step into the dead slot (no branch in the MFMA stream).
//
// LDS images (per slot):
//   A, NT-B: [256 rows][64 k] (128-B rows), 16-B chunk c of row r at
//            c ^ ((r >> 1) & 7) (gemm_256's swizzle: conflict-free for the
//            16-row x 16-B fragment read); a DMA piece = 8 rows x 128 B.
//   NN-B:    [64 k][256 n] (512-B rows), chunk c of k-row k at c ^ fnn(k)
//            (gemm.hip's g2_fnn), read transposed by ds_read_b64_tr_b16;
//            a piece = 2 k-rows x 512 B.
// Arithmetic: every output is one chain of MFMAs over K in increasing order,
// 32 k per MFMA -- gemm_256's order, so outputs are bitwise those of that
// kernel (and of gemm_w4v).
#include "gemm_w5.h"

#include <utility>

#include "pli_common.h"
#include "gemm_w4v_asm.h"

// A/B switches (tools/build_ab.sh); the defaults are the product
#ifndef W5_DMA_START
#define W5_DMA_START 0  // half-1 gap of the first DMA piece
#endif
#ifndef W5_DMA_STRIDE
#define W5_DMA_STRIDE 4  // gaps between DMA pieces
#endif
#ifndef W5_DMA_IMM
#define W5_DMA_IMM 1  // one M0 write per 4 pieces, pieces 1-3 by instruction offset
#endif
#ifndef W5_RD_STRIDE
#define W5_RD_STRIDE 2  // gaps between fragment reads (with DMA start 0: 0-3 % over stride 1 / start 2, profiles/r03/gemm/ab_w5_ring5.log)
#endif
#ifndef W5_RING5
#define W5_RING5 0  // 5 ring positions of 32 KiB (A and B images apart): A's DMA in half 0, B's in half 1
#endif
#ifndef W5_ABL_DMA
#define W5_ABL_DMA 0  // timing only: no DMA in the loop (results wrong)
#endif
#ifndef W5_ABL_RD
#define W5_ABL_RD 0  // timing only: no fragment reads in the loop (results wrong)
#endif
#ifndef W5_ABL_BAR
#define W5_ABL_BAR 0  // timing only: no barriers in the loop (races; results wrong)
#endif
#ifndef W5_SPLIT
// 1: the (S, h1) fragments are read in half 0's first 16 gaps, a barrier
// after gap 24 frees slot S, and 5 of step S+2's DMA pieces go into half 0's
// later gaps (11 stay in half 1): the pieces spread over 1.6 halves and the
// half-0 ones meet no fragment read
#define W5_SPLIT 1
#endif
// W5_SPLIT placement (A/B knobs): half-0 read stride, barrier gap, DMA
// pieces in half 0 with their first gap and spacing; half-1 read stride,
// first DMA gap and spacing (the remaining 16 - W5S_N0 pieces)
#ifndef W5S_RS0
#define W5S_RS0 1
#endif
#ifndef W5S_BAR
#define W5S_BAR 24
#endif
#ifndef W5S_N0
#define W5S_N0 5
#endif
#ifndef W5S_D0
#define W5S_D0 28
#endif
#ifndef W5S_DS0
#define W5S_DS0 7
#endif
#ifndef W5S_RS1
#define W5S_RS1 3  // placement sweep: profiles/r04/gemm/ab_w5_split_placement.log (s6)
#endif
#ifndef W5S_D1
#define W5S_D1 1
#endif
#ifndef W5S_DS1
#define W5S_DS1 6
#endif

#ifndef W5_Q4
// 1: four meeting points per step (A / B images freed and landed apart, each
// by its own wait + barrier); see w5q below
#define W5_Q4 0
#endif
#ifndef W5Q_RA0
#define W5Q_RA0 0
#endif
#ifndef W5Q_RAS
#define W5Q_RAS 2
#endif
#ifndef W5Q_BA
#define W5Q_BA 20
#endif
#ifndef W5Q_DA0
#define W5Q_DA0 21
#endif
#ifndef W5Q_DAS
#define W5Q_DAS 4
#endif
#ifndef W5Q_RB0
#define W5Q_RB0 23
#endif
#ifndef W5Q_RBS
#define W5Q_RBS 4
#endif
#ifndef W5Q_BB
#define W5Q_BB 54
#endif
#ifndef W5Q_DB0
#define W5Q_DB0 55
#endif
#ifndef W5Q_DBS
#define W5Q_DBS 4
#endif
#ifndef W5Q_VA
#define W5Q_VA 66
#endif
#ifndef W5Q_RC0
#define W5Q_RC0 68
#endif
#ifndef W5Q_RCS
#define W5Q_RCS 2
#endif
#ifndef W5Q_VB
#define W5Q_VB 96
#endif
#ifndef W5Q_RD0
#define W5Q_RD0 97
#endif
#ifndef W5Q_RDS
#define W5Q_RDS 2
#endif

namespace pli {
namespace {


// W5_Q4 schedule of one K step (gap g follows MFMA g of 128; MFMAs 0-63 on
// the (S, h0) fragments, 64-127 on (S, h1)):
//   A(S, h1) reads at RA0 + RAS i; at BA they are waited for and the
//   workgroup meets: slot S's A image is free, and step S+2's A pieces go in
//   at DA0 + DAS i (between them the B(S, h1) reads, RB0 + RBS i); at BB the
//   B reads are waited for, the workgroup meets, and S+2's B pieces go in at
//   DB0 + DBS i.  At VA this wave's A(S+1) pieces have landed (vmcnt: the 8
//   B(S+1) pieces and the S+2 pieces issued so far may be in flight), the
//   workgroup meets, and A(S+1, h0) is read at RC0 + RCS i; at VB the same
//   for B(S+1), read at RD0 + RDS i.  Each image gets its own free / landed
//   point, so a piece has >= 140 gaps from issue to use.
namespace w5q {
constexpr int RA0 = W5Q_RA0, RAS = W5Q_RAS, BA = W5Q_BA, DA0 = W5Q_DA0, DAS = W5Q_DAS, RB0 = W5Q_RB0,
              RBS = W5Q_RBS, BB = W5Q_BB, DB0 = W5Q_DB0, DBS = W5Q_DBS, VA = W5Q_VA, RC0 = W5Q_RC0,
              RCS = W5Q_RCS, VB = W5Q_VB, RD0 = W5Q_RD0, RDS = W5Q_RDS;
constexpr int dma_gap(int j) { return j < 8 ? DA0 + DAS * j : DB0 + DBS * (j - 8); }
constexpr int dma_at(int g) {
    for (int j = 0; j < 16; ++j)
        if (dma_gap(j) == g) return j;
    return -1;
}
constexpr int issued_before(int g) {
    int n = 0;
    for (int j = 0; j < 16; ++j) n += dma_gap(j) < g;
    return n;
}
// read at gap g: 0-7 A(S, h1), 8-15 B(S, h1), 16-23 A(S+1, h0), 24-31 B(S+1, h0)
constexpr int read_gap(int r) {
    return r < 8 ? RA0 + RAS * r : r < 16 ? RB0 + RBS * (r - 8) : r < 24 ? RC0 + RCS * (r - 16) : RD0 + RDS * (r - 24);
}
constexpr int read_at(int g) {
    for (int r = 0; r < 32; ++r)
        if (read_gap(r) == g) return r;
    return -1;
}
constexpr bool valid() {
    for (int g = 0; g < 128; ++g) {
        int nr = 0, nd = 0;
        for (int r = 0; r < 32; ++r) nr += read_gap(r) == g;
        for (int j = 0; j < 16; ++j) nd += dma_gap(j) == g;
        if (nr > 1 || nd > 1) return false;
    }
    for (int r = 0; r < 8; ++r)
        if (read_gap(r) >= BA || read_gap(8 + r) >= BB || read_gap(16 + r) <= VA || read_gap(16 + r) < 64 ||
            read_gap(24 + r) <= VB || read_gap(24 + r) > 127)
            return false;
    for (int j = 0; j < 8; ++j)
        if (dma_gap(j) <= BA || dma_gap(8 + j) <= BB || dma_gap(8 + j) > 127) return false;
    return BA < BB && BB < 64 && VA < VB && issued_before(VB) == 16 && issued_before(VA) >= 8;
}
static_assert(!W5_Q4 || valid(), "W5_Q4 schedule: overlapping or misordered events");
}  // namespace w5q

template <int... I, class Fn>
__device__ __forceinline__ void w5_for(std::integer_sequence<int, I...>, Fn&& fn) {
    (fn(std::integral_constant<int, I>{}), ...);
}
template <int N, class Fn> __device__ __forceinline__ void w5_sfor(Fn&& fn) {
    w5_for(std::make_integer_sequence<int, N>{}, fn);
}

__device__ __forceinline__ void w5_tile(int lb, int tiles_m, int tiles_n, int group_m, int& tm, int& tn) {
    const int width = group_m * tiles_n;
    const int first = (lb / width) * group_m;
    const int rows = min(tiles_m - first, group_m);
    const int r = lb % width;
    tm = first + r % rows;
    tn = r / rows;
}
__device__ __forceinline__ int w5_fnn(int k) { return 2 * ((k & 3) | (((k >> 3) & 1) << 2)); }

template <int OFF> __device__ __forceinline__ void w5_rd128(i32x4& d, uint32_t addr) {
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "n"(OFF));
}
struct W5Pair { i32x2 lo, hi; };
// NN B^T fragment: two transposed reads, k rows +0..3 and +4..7 (2 KiB apart)
template <int OFF> __device__ __forceinline__ void w5_rdtr(W5Pair& d, uint32_t addr) {
    asm volatile("ds_read_b64_tr_b16 %0, %2 offset:%3\n\tds_read_b64_tr_b16 %1, %2 offset:%4"
                 : "=&v"(d.lo), "=&v"(d.hi) : "v"(addr), "n"(OFF), "n"(OFF + 2048));
}

// PERSIST (variant 43; M and N multiples of 256): one workgroup per CU walks
// the tiles L, L + G, ... (G = gridDim.x, a multiple of 8: one XCD per walk);
// the K stream continues across tiles (the last two steps of a tile DMA the
// next tile's steps 0 and 1 into the ring, the slot parity follows a global
// step count), and the epilogue stages through a separate 32 KiB region
// (8 KiB per wave, four passes of 32 rows) so the ring keeps the next tile's
// first steps.
// F32OUT (pli_gemm_f32out, the row-parallel fp32 partial): C is float
// [M][ldc], stored straight from the accumulators (16 B per lane), no bias.
// SWIGLU (pli_gemm_swiglu prefill; NT, no bias, one tile per workgroup):
// C[m][n] = silu(A Bg^T) * (A Bu^T) on a 256 x 128 output tile -- the B image's
// rows 0-127 are gate rows n0 .. n0+127 (Bm), rows 128-255 the same up rows
// (Bu), so wave (wr, 1) holds the up values of wave (wr, 0)'s gate block; it
// hands them over through LDS (fp32) and wave (wr, 0) stores silu(g) * u.
template <typename T, bool TRANS_B, bool BIAS, bool PERSIST = false, bool F32OUT = false, bool SWIGLU = false>
__global__ __launch_bounds__(256, 1) void gemm_w5(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bm,
                                                  void* __restrict__ Cv, const uint16_t* __restrict__ bias,
                                                  int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc,
                                                  int tiles_n, int nblocks, int group_m,
                                                  const uint16_t* __restrict__ Bu = nullptr, int64_t ldbu = 0) {
    constexpr int IMG = 32768, SLOT = 2 * IMG;
    using BFrag = std::conditional_t<TRANS_B, i32x4, W5Pair>;
    static_assert(!(F32OUT && BIAS), "the fp32-output form has no bias");
    static_assert(!SWIGLU || (TRANS_B && !BIAS && !PERSIST && !F32OUT), "the SwiGLU form is NT, one tile");
    constexpr int TN = SWIGLU ? 128 : 256;  // output columns per tile
    uint16_t* C = reinterpret_cast<uint16_t*>(Cv);
    static_assert(!(PERSIST && W5_RING5), "the persistent form uses the two-slot ring");
    constexpr int EPI = 2 * SLOT;  // PERSIST: epilogue staging, 8 KiB per wave
    __shared__ __attribute__((aligned(1024))) char smem[W5_RING5 ? 5 * IMG : (PERSIST ? 2 * SLOT + 32768 : 2 * SLOT)];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 1, wc = wave & 1;
    int tm, tn;
    int L = blockIdx.x;
    w5_tile(xcd_remap(L, nblocks), cdiv(M, 256), tiles_n, group_m, tm, tn);
    int m0 = tm * 256, n0 = tn * TN;
    const int ks = K / 64;
    const uint32_t lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem;

    // ---- LDS-DMA plan: wave w stages 8 KiB of each operand image per step
    // (8 pieces of 1 KiB): A / NT-B rows 64w .. 64w+63 (8 rows x 128 B per
    // piece), NN-B k-rows 16w .. 16w+15 (2 x 512 B per piece).  Per-lane byte
    // offsets from the tile's base; rows past M / N re-read the last row
    // (their outputs are never stored).
    uint32_t aoff[8], boff[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int row = 64 * wave + 8 * i + (lane >> 3);
        const int c = (lane & 7) ^ ((row >> 1) & 7);
        aoff[i] = (uint32_t)(((int64_t)(min(m0 + row, M - 1) - m0) * lda + 8 * c) * 2);
        if constexpr (SWIGLU) {  // waves 0-1: gate rows, waves 2-3: the same up rows
            const int rb = row & 127;
            boff[i] = (uint32_t)(((int64_t)(min(n0 + rb, N - 1) - n0) * (wave < 2 ? ldb : ldbu) + 8 * c) * 2);
        } else if constexpr (TRANS_B) {
            boff[i] = (uint32_t)(((int64_t)(min(n0 + row, N - 1) - n0) * ldb + 8 * c) * 2);
        } else {
            const int kr = 16 * wave + 2 * i + (lane >> 5);
            const int cn = (lane & 31) ^ w5_fnn(kr);
            boff[i] = (uint32_t)(((int64_t)kr * ldb + min(n0 + 8 * cn, N - 8) - n0) * 2);
        }
    }
    // (PERSIST: M, N multiples of 256, so no row is clamped and the offsets
    // above hold for every tile; only the bases move)
    const uint16_t* abase = A + (int64_t)m0 * lda;
    const uint16_t* bbase = SWIGLU ? (wave < 2 ? Bm + (int64_t)n0 * ldb : Bu + (int64_t)n0 * ldbu)
                            : TRANS_B ? Bm + (int64_t)n0 * ldb : Bm + n0;
    const uint16_t *nabase = abase, *nbbase = bbase;  // PERSIST: the next tile's
    bool has_next = false;
    int gs = 0;  // PERSIST: global step count of this tile's step 0 (slot parity)
    auto dma1 = [&](const uint16_t* src, uint32_t off, uint32_t lds) __attribute__((always_inline)) {
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(lds), "v"(off), "s"(src)
                     : "memory");
    };
    // W5_DMA_IMM: piece i of a group of 4 reaches its LDS kilobyte through
    // the instruction offset (i % 4) * 1024, which the hardware adds to the
    // global address too -- the scalar base is biased by that much instead
    auto dma_next = [&](auto i_tag, const uint16_t* src, uint32_t off) __attribute__((always_inline)) {
        constexpr int i = decltype(i_tag)::value;
        asm volatile("global_load_lds_dwordx4 %0, %1 offset:%2" ::"v"(off),
                     "s"(reinterpret_cast<const char*>(src) - 1024 * i), "n"(1024 * i) : "memory");
    };
    // LDS byte offset of step s's A (x = 0) or B (x = 1) image: slot s % 2,
    // or (W5_RING5) ring position (2s + x) % 5
    auto img_off = [&](int s, int x) __attribute__((always_inline)) {
        return W5_RING5 ? (uint32_t)((2 * s + x) % 5) * IMG : (uint32_t)((gs + s) & 1) * SLOT + (uint32_t)x * IMG;
    };
    // DMA piece j (0-7 A, 8-15 B) of K step s into its image (past the last
    // step: a reload of the last step)
    auto dma_piece = [&](auto j_tag, int s) __attribute__((always_inline)) {
        constexpr int j = decltype(j_tag)::value, i = j % 8;
        const uint32_t slot = lds0 + img_off(s, j < 8 ? 0 : 1) + (uint32_t)wave * 8192 +
                              (uint32_t)(W5_DMA_IMM ? (i / 4) * 4096 : i * 1024);
        // past the last step: PERSIST with a next tile, that tile's step
        // s - ks; else a reload of the last step
        const uint16_t *ab = abase, *bb = bbase;
        int sc = min(s, ks - 1);
        if constexpr (PERSIST) {
            if (s >= ks && has_next) {  // (ks >= 2: the launcher's condition)
                ab = nabase;
                bb = nbbase;
                sc = min(s - ks, ks - 1);
            }
        }
        const uint32_t off = j < 8 ? aoff[i] : boff[i];
        const uint16_t* src = j < 8 ? ab + sc * 64 : (TRANS_B ? bb + sc * 64 : bb + (int64_t)sc * 64 * ldb);
        if constexpr (W5_DMA_IMM && i % 4 > 0) dma_next(std::integral_constant<int, i % 4>{}, src, off);
        else dma1(src, off, slot);
    };

    // ---- fragment read addresses (slot 0, half 0; + slot * SLOT, halves by
    // address (A / NT-B: the chunk XOR) or offset (NN-B: +16 KiB))
    const int r16 = lane & 15, h4 = lane >> 4;
    uint32_t a_rd[2], b_rd[TRANS_B ? 2 : 8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int ch = (4 * h + h4) ^ ((r16 >> 1) & 7);
        a_rd[h] = lds0 + (uint32_t)((wr * 128 + r16) * 128 + (ch << 4));
        if constexpr (TRANS_B) b_rd[h] = lds0 + (uint32_t)((wc * 128 + r16) * 128 + (ch << 4));
    }
    if constexpr (!TRANS_B) {
        const int q = (lane >> 2) & 3, p = lane & 3, kr = 8 * h4 + q;
#pragma unroll
        for (int ni = 0; ni < 8; ++ni) {
            const int c = wc * 16 + 2 * ni + (p >> 1);
            b_rd[ni] = lds0 + (uint32_t)(kr * 512 + ((c ^ w5_fnn(kr)) << 4) + (p & 1) * 8);
        }
    }

    i32x4 fa[2][8];
    BFrag fb[2][8];
    // fragment read I (0-7 A, 8-15 B) of half H of the step whose A and B
    // images sit at byte offsets sa, sb, into buffer P (= H)
    auto frag_read = [&](auto h_tag, auto i_tag, uint32_t sa, uint32_t sb) __attribute__((always_inline)) {
        constexpr int H = decltype(h_tag)::value, I = decltype(i_tag)::value;
        if constexpr (I < 8) {
            w5_rd128<I * 2048>(fa[H][I], a_rd[H] + sa);
        } else if constexpr (TRANS_B) {
            w5_rd128<(I - 8) * 2048>(fb[H][I - 8], b_rd[H] + sb);
        } else {
            w5_rdtr<H * 16384>(fb[H][I - 8], b_rd[I - 8] + sb);
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
    // 64 MFMAs on buffer P, with fragment reads (RD: 16, half RH into buffer
    // RH, image offsets rsa / rsb) and DMA pieces J0 .. J0+NJ-1 of step ds in
    // their gaps
    constexpr int DSTART = W5_RING5 ? 2 : W5_DMA_START, DSTRIDE = W5_RING5 ? 8 : W5_DMA_STRIDE;
    // RS: gaps between fragment reads, DS0 / DSTR: first gap and spacing of
    // the DMA pieces, BAR: the gap after which the reads are waited for and
    // the workgroup meets (-1: none)
    auto half_x = [&](auto p_tag, auto rd_tag, auto rh_tag, uint32_t rsa, uint32_t rsb, auto j0_tag, auto nj_tag,
                      int ds, auto rs_tag, auto ds0_tag, auto dstr_tag, auto bar_tag) __attribute__((always_inline)) {
        constexpr int P = decltype(p_tag)::value, RH = decltype(rh_tag)::value;
        constexpr bool RD = decltype(rd_tag)::value;
        constexpr int J0 = decltype(j0_tag)::value, NJ = decltype(nj_tag)::value;
        constexpr int RS = decltype(rs_tag)::value, DS0 = decltype(ds0_tag)::value;
        constexpr int DSTR = decltype(dstr_tag)::value, BAR = decltype(bar_tag)::value;
        w5_sfor<64>([&](auto JJ) {
            constexpr int J = JJ, ni = J / 8, mi = J % 8;
            if constexpr (std::is_same_v<T, bf16_t>) w4v::mfma_bf16<J>(bop(fb[P][ni]), fa[P][mi]);
            else w4v::mfma_f16<J>(bop(fb[P][ni]), fa[P][mi]);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (!W5_ABL_RD && RD && J % RS == 0 && J / RS < 16)
                frag_read(std::integral_constant<int, RH>{}, std::integral_constant<int, J / RS>{}, rsa, rsb);
            if constexpr (J == BAR) {
                frag_wait(std::integral_constant<int, RH>{});
                if constexpr (!W5_ABL_BAR) __builtin_amdgcn_s_barrier();
                __builtin_amdgcn_sched_barrier(0);
            }
            constexpr int D = J - DS0;
            if constexpr (!W5_ABL_DMA && D >= 0 && D % DSTR == 0 && D / DSTR < NJ)
                dma_piece(std::integral_constant<int, J0 + D / DSTR>{}, ds);
            __builtin_amdgcn_sched_barrier(0);
        });
    };
    auto half = [&](auto p_tag, auto rd_tag, auto rh_tag, uint32_t rsa, uint32_t rsb, auto j0_tag, auto nj_tag, int ds)
        __attribute__((always_inline)) {
        half_x(p_tag, rd_tag, rh_tag, rsa, rsb, j0_tag, nj_tag, ds, std::integral_constant<int, W5_RD_STRIDE>{},
               std::integral_constant<int, DSTART>{}, std::integral_constant<int, DSTRIDE>{},
               std::integral_constant<int, -1>{});
    };

    // ---- prologue: accumulators 0, steps 0 and 1 in flight, (0, h0) fragments
    // PERSIST: the next tile of this walk (its bases, for the stream's DMA)
    auto next_tile = [&]() __attribute__((always_inline)) {
        has_next = L + (int)gridDim.x < nblocks;
        if (has_next) {
            int tm2, tn2;
            w5_tile(xcd_remap(L + (int)gridDim.x, nblocks), cdiv(M, 256), tiles_n, group_m, tm2, tn2);
            nabase = A + (int64_t)(tm2 * 256) * lda;
            nbbase = TRANS_B ? Bm + (int64_t)(tn2 * 256) * ldb : Bm + tn2 * 256;
        }
    };
    if constexpr (PERSIST) next_tile();
    w4v::acc_zero();
    w5_sfor<16>([&](auto J) { dma_piece(J, 0); });
    w5_sfor<16>([&](auto J) { dma_piece(J, 1); });
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // step 0 (this wave's pieces)
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    w5_sfor<16>([&](auto I) { frag_read(std::integral_constant<int, 0>{}, I, img_off(0, 0), img_off(0, 1)); });
    frag_wait(std::integral_constant<int, 0>{});

    using Z = std::integral_constant<int, 0>;
    using O = std::integral_constant<int, 1>;
    auto frag_wait_x = [&](auto p_tag, auto b_tag) __attribute__((always_inline)) {
        constexpr int P = decltype(p_tag)::value;
        constexpr bool Bop = decltype(b_tag)::value;
        if constexpr (!Bop) {
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(fa[P][0]), "+v"(fa[P][1]), "+v"(fa[P][2]), "+v"(fa[P][3]), "+v"(fa[P][4]),
                           "+v"(fa[P][5]), "+v"(fa[P][6]), "+v"(fa[P][7])::"memory");
        } else if constexpr (TRANS_B) {
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(fb[P][0]), "+v"(fb[P][1]), "+v"(fb[P][2]), "+v"(fb[P][3]), "+v"(fb[P][4]),
                           "+v"(fb[P][5]), "+v"(fb[P][6]), "+v"(fb[P][7])::"memory");
        } else {
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(fb[P][0].lo), "+v"(fb[P][0].hi), "+v"(fb[P][1].lo), "+v"(fb[P][1].hi),
                           "+v"(fb[P][2].lo), "+v"(fb[P][2].hi), "+v"(fb[P][3].lo), "+v"(fb[P][3].hi),
                           "+v"(fb[P][4].lo), "+v"(fb[P][4].hi), "+v"(fb[P][5].lo), "+v"(fb[P][5].hi),
                           "+v"(fb[P][6].lo), "+v"(fb[P][6].hi), "+v"(fb[P][7].lo), "+v"(fb[P][7].hi)::"memory");
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    // W5_Q4: one K step, 128 MFMAs with the w5q events in their gaps
    auto step_q4 = [&](int s, auto more_tag) __attribute__((always_inline)) {
        constexpr bool MORE = decltype(more_tag)::value;
        const uint32_t sa0 = img_off(s, 0), sb0 = img_off(s, 1), sa1 = img_off(s + 1, 0), sb1 = img_off(s + 1, 1);
        w5_sfor<128>([&](auto JJ) {
            constexpr int J = JJ, P = J / 64, JL = J % 64, ni = JL / 8, mi = JL % 8;
            if constexpr (std::is_same_v<T, bf16_t>) w4v::mfma_bf16<JL>(bop(fb[P][ni]), fa[P][mi]);
            else w4v::mfma_f16<JL>(bop(fb[P][ni]), fa[P][mi]);
            __builtin_amdgcn_sched_barrier(0);
            constexpr int r = w5q::read_at(J);
            if constexpr (!W5_ABL_RD && r >= 0 && r < 16)
                frag_read(std::integral_constant<int, 1>{}, std::integral_constant<int, r>{}, sa0, sb0);
            if constexpr (!W5_ABL_RD && r >= 16 && MORE)
                frag_read(std::integral_constant<int, 0>{}, std::integral_constant<int, r - 16>{}, sa1, sb1);
            if constexpr (J == w5q::BA || J == w5q::BB) {
                frag_wait_x(std::integral_constant<int, 1>{}, std::bool_constant<J == w5q::BB>{});
                if constexpr (!W5_ABL_BAR) __builtin_amdgcn_s_barrier();
                __builtin_amdgcn_sched_barrier(0);
            }
            if constexpr (J == w5q::VA || J == w5q::VB) {
                // this wave's A (VA) / B (VB) pieces of step s+1 landed
                constexpr int n = (J == w5q::VA ? 8 : 0) + w5q::issued_before(J);
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(n) : "memory");
                if constexpr (!W5_ABL_BAR) __builtin_amdgcn_s_barrier();
                __builtin_amdgcn_sched_barrier(0);
            }
            constexpr int d = w5q::dma_at(J);
            if constexpr (!W5_ABL_DMA && d >= 0) dma_piece(std::integral_constant<int, d>{}, s + 2);
            __builtin_amdgcn_sched_barrier(0);
        });
        if constexpr (MORE) frag_wait(Z{});
    };
    auto step = [&](int s, auto more_tag) __attribute__((always_inline)) {
        constexpr bool MORE = decltype(more_tag)::value;  // a step s+1 follows
        if constexpr (W5_Q4) {
            step_q4(s, more_tag);
            return;
        }
        using N0 = std::integral_constant<int, 0>;
        using N8 = std::integral_constant<int, 8>;
        using N16 = std::integral_constant<int, 16>;
        // W5_RING5: step s+2's A pieces in half 0 (into B(s-1)'s dead ring
        // position), its B pieces in half 1 (into A(s)'s); else all 16 in half 1
        if constexpr (W5_SPLIT) {
            using I = std::integral_constant<int, 1>;
            (void)I{};
            half_x(Z{}, std::true_type{}, O{}, img_off(s, 0), img_off(s, 1), N0{},
                   std::integral_constant<int, W5S_N0>{}, s + 2, std::integral_constant<int, W5S_RS0>{},
                   std::integral_constant<int, W5S_D0>{}, std::integral_constant<int, W5S_DS0>{},
                   std::integral_constant<int, W5S_BAR>{});
            // step s+1 landed (W5S_N0 of s+2's pieces in flight)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(W5S_N0) : "memory");
            if constexpr (!W5_ABL_BAR) __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
            half_x(O{}, more_tag, Z{}, img_off(s + 1, 0), img_off(s + 1, 1), std::integral_constant<int, W5S_N0>{},
                   std::integral_constant<int, 16 - W5S_N0>{}, s + 2, std::integral_constant<int, W5S_RS1>{},
                   std::integral_constant<int, W5S_D1>{}, std::integral_constant<int, W5S_DS1>{},
                   std::integral_constant<int, -1>{});
            if constexpr (MORE) frag_wait(Z{});
            return;
        }
        if constexpr (W5_RING5)
            half(Z{}, std::true_type{}, O{}, img_off(s, 0), img_off(s, 1), N0{}, N8{}, s + 2);
        else
            half(Z{}, std::true_type{}, O{}, img_off(s, 0), img_off(s, 1), N0{}, N0{}, s + 2);
        frag_wait(O{});
        // step s+1 landed (this wave's pieces; RING5: step s+2's A pieces,
        // issued in half 0, may stay in flight)
        if constexpr (W5_RING5) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (W5_RING5)
            half(O{}, more_tag, Z{}, img_off(s + 1, 0), img_off(s + 1, 1), N8{}, N8{}, s + 2);
        else
            half(O{}, more_tag, Z{}, img_off(s + 1, 0), img_off(s + 1, 1), N0{}, N16{}, s + 2);
        if constexpr (MORE) frag_wait(Z{});
    };
    // accumulator block J = (ni, mi) -> packed bf16 / fp16 (bias added):
    // C[m][n .. n+3], m = m0 + 128 wr + 16 mi + (lane & 15), n = n0 + 128 wc +
    // 16 ni + 4 (lane >> 4)
    auto acc_pack = [&](auto j_tag) __attribute__((always_inline)) {
        constexpr int J = decltype(j_tag)::value, ni = J / 8;
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
        return i32x2{(int)pack2<T>(v[0], v[1]), (int)pack2<T>(v[2], v[3])};
    };
    // F32OUT: every accumulator block straight to C (float), 16 B per lane
    auto store_f32 = [&]() __attribute__((always_inline)) {
        asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");  // last MFMA -> accumulator reads
        float* Cf = reinterpret_cast<float*>(Cv);
        w5_sfor<64>([&](auto JJ) {
            constexpr int J = JJ, ni = J / 8, mi = J % 8;
            f32x4 v;
            w4v::acc_read<J>(v);
            const int m = m0 + 128 * wr + 16 * mi + r16, n = n0 + 128 * wc + 16 * ni + 4 * h4;
            if (m < M && n < N) *reinterpret_cast<f32x4*>(Cf + (int64_t)m * ldc + n) = v;
        });
    };
    for (;;) {
        int s = 0;
        for (; s + 1 < ks; ++s) step(s, std::true_type{});
        step(s, std::false_type{});

        if constexpr (SWIGLU) {
            // up (waves wc = 1) -> LDS as fp32, lane-private [block][lane];
            // gate waves read their lane's up values and store silu(g) * u
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // dead-slot reloads landed
            __builtin_amdgcn_s_barrier();                     // every wave is done with the ring
            asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");  // last MFMA -> accumulator reads
            f32x4* up = reinterpret_cast<f32x4*>(smem + wr * 65536);
            if (wc == 1) {
                w5_sfor<64>([&](auto JJ) {
                    f32x4 v;
                    w4v::acc_read<JJ>(v);
                    up[JJ * 64 + lane] = v;
                });
            }
            __syncthreads();
            if (wc == 0) {
                w5_sfor<64>([&](auto JJ) {
                    constexpr int J = JJ, ni = J / 8, mi = J % 8;
                    f32x4 g;
                    w4v::acc_read<J>(g);
                    const f32x4 u = up[J * 64 + lane];
                    f32x4 h;
#pragma unroll
                    for (int r = 0; r < 4; ++r) h[r] = g[r] / (1.f + __expf(-g[r])) * u[r];  // gemm.hip silu_mul
                    const int m = m0 + 128 * wr + 16 * mi + r16, n = n0 + 16 * ni + 4 * h4;
                    if (m < M && n < N)
                        *reinterpret_cast<i32x2*>(C + (int64_t)m * ldc + n) =
                            i32x2{(int)pack2<T>(h[0], h[1]), (int)pack2<T>(h[2], h[3])};
                });
            }
            break;
        } else if constexpr (F32OUT && !PERSIST) {
            store_f32();
            // the last step's dead-slot reloads land before the LDS is released
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            break;
        } else if constexpr (!PERSIST) {
            // ---- epilogue (gemm_w4v's): each wave packs its 128 x 128 tile
            // into its own 32 KiB of LDS ([row][256 B], chunk c of row r at
            // c ^ (r & 15)) and stores whole 256-B row segments, 16 B per lane
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // dead-slot reloads landed
            __builtin_amdgcn_s_barrier();                     // every wave is done with the ring
            asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");  // last MFMA -> accumulator reads
            char* reg = smem + wave * 32768;
            w5_sfor<64>([&](auto JJ) {
                constexpr int J = JJ, ni = J / 8, mi = J % 8;
                const i32x2 pk = acc_pack(JJ);
                const int row = 16 * mi + r16, chunk = 2 * ni + (h4 >> 1);
                *reinterpret_cast<i32x2*>(reg + row * 256 + ((chunk ^ r16) << 4) + (h4 & 1) * 8) = pk;
            });
            const int c = lane & 15;
            const int n = n0 + 128 * wc + 8 * c;
#pragma unroll 8
            for (int it = 0; it < 32; ++it) {
                const int row = 4 * it + h4;
                const i32x4 v = *reinterpret_cast<const i32x4*>(reg + row * 256 + ((c ^ (row & 15)) << 4));
                const int m = m0 + 128 * wr + row;
                if (m < M && n < N) *reinterpret_cast<i32x4*>(C + (int64_t)m * ldc + n) = v;
            }
            break;
        } else {
            if constexpr (F32OUT) {
                store_f32();  // 64 stores per wave (M, N multiples of 256)
            } else {
            // ---- epilogue through this wave's 8 KiB of the staging region,
            // four passes of 32 rows (accumulator rows mi = 2p, 2p + 1); the
            // ring keeps the next tile's steps 0 and 1.  M, N multiples of
            // 256: every store is in bounds, 32 per wave.
            asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");  // last MFMA -> accumulator reads
            char* reg = smem + EPI + wave * 8192;
            const int c = lane & 15;
            const int n = n0 + 128 * wc + 8 * c;
            w5_sfor<4>([&](auto PP) {
                constexpr int pss = PP;
                w5_sfor<16>([&](auto II) {
                    constexpr int ni = II / 2, mi = 2 * pss + II % 2;
                    const i32x2 pk = acc_pack(std::integral_constant<int, 8 * ni + mi>{});
                    const int row = 16 * (II % 2) + r16, chunk = 2 * ni + (h4 >> 1);
                    *reinterpret_cast<i32x2*>(reg + row * 256 + ((chunk ^ r16) << 4) + (h4 & 1) * 8) = pk;
                });
#pragma unroll
                for (int it = 0; it < 8; ++it) {
                    const int row = 4 * it + h4;
                    const i32x4 v = *reinterpret_cast<const i32x4*>(reg + row * 256 + ((c ^ (row & 15)) << 4));
                    const int m = m0 + 128 * wr + 32 * pss + row;
                    *reinterpret_cast<i32x4*>(C + (int64_t)m * ldc + n) = v;
                }
            });
            }
            if (!has_next) break;
            // ---- next tile: its steps 0 and 1 are in the ring (DMA'd by
            // this tile's last two steps)
            gs += ks;
            L += (int)gridDim.x;
            w5_tile(xcd_remap(L, nblocks), cdiv(M, 256), tiles_n, group_m, tm, tn);
            m0 = tm * 256;
            n0 = tn * 256;
            abase = nabase;
            bbase = nbbase;
            next_tile();
            w4v::acc_zero();
            // step 0 landed: younger than its pieces are step 1's 16 and the
            // epilogue's 32 stores (F32OUT: 64 stores, more than vmcnt holds:
            // vmcnt(63) still retires the oldest 16 + 16 + 1)
            if constexpr (F32OUT) asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
            w5_sfor<16>([&](auto I) { frag_read(std::integral_constant<int, 0>{}, I, img_off(0, 0), img_off(0, 1)); });
            frag_wait(std::integral_constant<int, 0>{});
        }
    }
    // the last (reload) pieces land before the LDS is released
    if constexpr (PERSIST) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

int launch_gemm_w5_swiglu(const void* x, const void* wg, const void* wu, void* h, int m, int n, int k, int64_t ldx,
                          int64_t ldwg, int64_t ldwu, int64_t ldh, int is_bf16, hipStream_t stream) {
    PLI_REQUIRE(k >= 64 && k % 64 == 0 && n % 8 == 0 && ldx * 2 * 256 < (1ll << 31) &&
                    ldwg * 2 * 128 < (1ll << 31) && ldwu * 2 * 128 < (1ll << 31),
                "gemm_w5 swiglu: shape m=%d n=%d k=%d not supported", m, n, k);
    const int tiles_n = cdiv(n, 128);
    const int64_t nb = (int64_t)cdiv(m, 256) * tiles_n;
    PLI_REQUIRE(nb < (1ll << 31), "gemm_w5 swiglu: grid too large");
    const auto* X = (const uint16_t*)x;
    const auto* G = (const uint16_t*)wg;
    const auto* U = (const uint16_t*)wu;
    if (is_bf16)
        hipLaunchKernelGGL((gemm_w5<bf16_t, true, false, false, false, true>), dim3((unsigned)nb), dim3(256), 0,
                           stream, X, G, h, nullptr, m, n, k, ldx, ldwg, ldh, tiles_n, (int)nb, 4, U, ldwu);
    else
        hipLaunchKernelGGL((gemm_w5<f16_t, true, false, false, false, true>), dim3((unsigned)nb), dim3(256), 0,
                           stream, X, G, h, nullptr, m, n, k, ldx, ldwg, ldh, tiles_n, (int)nb, 4, U, ldwu);
    return launch_status("gemm_w5<swiglu>");
}

bool gemm_w5_ok(int m, int n, int k, int64_t lda, int64_t ldb, int64_t ldc, int trans_b) {
    (void)m;
    (void)ldc;
    // per-lane DMA offsets are 32-bit: 256 rows (NN: 64 k-rows) of the operand
    return k >= 64 && k % 64 == 0 && n % 8 == 0 && n >= 8 && lda * 2 * 256 < (1ll << 31) &&
           ldb * 2 * (trans_b ? 256 : 64) < (1ll << 31);
}

int launch_gemm_w5(const void* a, const void* b, void* c, const void* bias, int m, int n, int k, int64_t lda,
                   int64_t ldb, int64_t ldc, int trans_b, int is_bf16, hipStream_t stream, int group_m,
                   bool persistent, bool f32out) {
    PLI_REQUIRE(!f32out || (trans_b && bias == nullptr), "gemm_w5: fp32 output is NT without bias");
    PLI_REQUIRE(gemm_w5_ok(m, n, k, lda, ldb, ldc, trans_b), "gemm_w5: shape m=%d n=%d k=%d not supported", m, n,
                k);
#ifdef W5_GROUP_M
    group_m = W5_GROUP_M;  // A/B builds only
#endif
    PLI_REQUIRE(group_m >= 1, "gemm_w5: group_m must be >= 1");
    const int tiles_m = cdiv(m, 256), tiles_n = cdiv(n, 256);
    const int64_t nb = (int64_t)tiles_m * tiles_n;
    PLI_REQUIRE(nb < (1ll << 31), "gemm_w5: grid too large");
    const auto* A = (const uint16_t*)a;
    const auto* B = (const uint16_t*)b;
    auto* Cc = (uint16_t*)c;
    const auto* bs = (const uint16_t*)bias;
    // persistent (variant 43): one workgroup per CU of the stream's device,
    // a multiple of 8 (each walk stays on one XCD); M, N multiples of 256
    PLI_REQUIRE(!persistent || (m % 256 == 0 && n % 256 == 0), "gemm_w5 persistent: M, N must be multiples of 256");
    // the stream prefetches two steps past a tile, i.e. the next tile's
    // steps 0 and 1: one-step tiles (K = 64) take the one-tile form
    if (k < 128) persistent = false;
    int grid = (int)nb;
    if (persistent) {
        const int g = cu_count(stream) / 8 * 8;
        if (g >= 8 && nb > g) grid = g;
    }
    const dim3 gr((unsigned)grid), blk(256);
#define W5_LAUNCH(T, TB, BI)                                                                                         \
    do {                                                                                                             \
        if (f32out) {                                                                                                \
            if (persistent)                                                                                          \
                hipLaunchKernelGGL((gemm_w5<T, true, false, true, true>), gr, blk, 0, stream, A, B, c, nullptr, m, n, \
                                   k, lda, ldb, ldc, tiles_n, (int)nb, group_m);                                    \
            else                                                                                                     \
                hipLaunchKernelGGL((gemm_w5<T, true, false, false, true>), gr, blk, 0, stream, A, B, c, nullptr, m,  \
                                   n, k, lda, ldb, ldc, tiles_n, (int)nb, group_m);                                 \
        } else if (persistent)                                                                                       \
            hipLaunchKernelGGL((gemm_w5<T, TB, BI, true>), gr, blk, 0, stream, A, B, Cc, bs, m, n, k, lda, ldb, ldc, \
                               tiles_n, (int)nb, group_m);                                                           \
        else                                                                                                         \
            hipLaunchKernelGGL((gemm_w5<T, TB, BI, false>), gr, blk, 0, stream, A, B, Cc, bs, m, n, k, lda, ldb,     \
                               ldc, tiles_n, (int)nb, group_m);                                                      \
    } while (0)
    if (is_bf16) {
        if (trans_b) { if (bias) W5_LAUNCH(bf16_t, true, true); else W5_LAUNCH(bf16_t, true, false); }
        else { if (bias) W5_LAUNCH(bf16_t, false, true); else W5_LAUNCH(bf16_t, false, false); }
    } else {
        if (trans_b) { if (bias) W5_LAUNCH(f16_t, true, true); else W5_LAUNCH(f16_t, true, false); }
        else { if (bias) W5_LAUNCH(f16_t, false, true); else W5_LAUNCH(f16_t, false, false); }
    }
#undef W5_LAUNCH
    return launch_status("gemm_w5");
}

}  // namespace pli
