// GEMM for gfx950 (MI355X): C = A op(B) (+ bias), fp32 accumulate.
//
// Replaces torch.mm of ch03/gemm_benchmark.py:35 (NN), the 16x16 shared-memory
// tiled_matmul of ch05/tiled_matmul.cu:22-61, and F.linear of
// ch09/tensor_parallel.py:39,67 / ch01/attention.py:59-71 (NT, + bias).
//
// MFMA kernel (bf16 / fp16): 128x128 output tile, BK = 64, 4 waves in 2x2,
// each wave a 64x64 sub-tile of 2x2 v_mfma_f32_32x32x16 blocks.  The MFMA is
// issued as C^T = op(B)^T A^T so the accumulator keeps the output ROW on the
// lane and 4 consecutive columns per register quad: the epilogue writes 8-byte
// row segments with the bias added in registers.
//   A tile  [128 m][64 k]   128-B rows, XOR-swizzled, fragments by ds_read_b128
//   B tile  NT: [128 n][64 k] same image as A
//           NN: [64 k][128 n] 256-B rows; the K-strided operand fragment comes
//               from two ds_read_b64_tr_b16 (gfx950 transposed LDS read), so
//               torch.mm's row-major B needs no transpose pass in HBM.
// Tiles are register-staged into double-buffered LDS (loads for k-tile t+1 in
// flight under the MFMAs of tile t), one barrier per k-tile; blocks are
// remapped so each XCD sweeps a contiguous band of output tiles (L2 reuse of
// the A row-panel / B column-panel).
//
// Generic kernel (fp32, ragged or unaligned shapes): 64x64 LDS-tiled VALU
// kernel, 4x4 outputs per thread, fp32 accumulate.
#include <type_traits>

#include "gemm_f32.h"
#include "gemm_w4v.h"
#include "gemm_w5.h"
#include "pli_common.h"

namespace pli {
namespace {

constexpr int BM = 128, BN = 128, BK = 64;

// 128-byte rows (64 x 16-bit): chunk ^= g((row>>1)&7)
__device__ __forceinline__ int off128(int row, int ch) {
    const int i = (row >> 1) & 7;
    const int g = ((i & 1) << 2) | (i >> 1);
    return row * 128 + ((ch ^ g) << 4);
}
// 256-byte rows (128 x 16-bit): chunk ^= ((row&3)<<2 | (row>>2)&3)
__device__ __forceinline__ int off256(int row, int ch) {
    const int f = ((row & 3) << 2) | ((row >> 2) & 3);
    return row * 256 + ((ch ^ f) << 4);
}

__device__ __forceinline__ float silu_mul(float g, float u) {
    return g / (1.f + __expf(-g)) * u;
}

// SWIGLU (NT only): C[m, n] = silu(A Bg^T)[m, n] * (A Bu^T)[m, n].  The B tile's
// first 64 rows are Bg rows nb..nb+63 and its last 64 the same rows of Bu, so
// waves wn = 0 hold gate and wn = 1 up accumulators for the same (m, n) at the
// same lane/register; the up waves hand theirs over through LDS.
template <typename T, bool TRANS_B, bool BIAS, bool SWIGLU = false>
__global__ __launch_bounds__(256, 2) void gemm_mfma(const uint16_t* __restrict__ A,
                                                    const uint16_t* __restrict__ Bm,
                                                    uint16_t* __restrict__ C,
                                                    const uint16_t* __restrict__ bias, int M, int N,
                                                    int K, int64_t lda, int64_t ldb, int64_t ldc,
                                                    int tiles_n, int nblocks,
                                                    const uint16_t* __restrict__ Bu = nullptr,
                                                    int64_t ldbu = 0) {
    static_assert(!SWIGLU || TRANS_B, "SwiGLU GEMM takes weights as [n][k]");
    constexpr int TILE = BM * BK * 2;  // 16 KiB per operand tile
    __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h32 = lane >> 5, l32 = lane & 31;
    const int wm = wave >> 1, wn = wave & 1;  // 2x2 waves, 64x64 each

    const int lb = xcd_remap(blockIdx.x, nblocks);
    const int m0 = (lb / tiles_n) * BM, n0 = (lb % tiles_n) * (SWIGLU ? BN / 2 : BN);
    const int ktiles = cdiv(K, BK);

    // staging: 1024 chunks of 16 B per operand tile, 4 per thread
    i32x4 ast[4], bst[4];
    auto load_tile = [&](int kt) {
        const int k0 = kt * BK;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int c = tid + 256 * i;
            {   // A: row = c/8 (m), chunk c%8 (k)
                const int r = c >> 3, ch = c & 7;
                const int mm = min(m0 + r, M - 1), kk = k0 + ch * 8;
                const i32x4 x = *reinterpret_cast<const i32x4*>(A + (int64_t)mm * lda + min(kk, K - 8));
                ast[i] = (m0 + r < M && kk < K) ? x : i32x4{0, 0, 0, 0};
            }
            if constexpr (SWIGLU) {  // rows 0..63 gate, 64..127 up, both n0 + (r & 63)
                const int r = c >> 3, ch = c & 7, rn = n0 + (r & 63);
                const int nn = min(rn, N - 1), kk = k0 + ch * 8;
                const uint16_t* src = r < 64 ? Bm + (int64_t)nn * ldb : Bu + (int64_t)nn * ldbu;
                const i32x4 x = *reinterpret_cast<const i32x4*>(src + min(kk, K - 8));
                bst[i] = (rn < N && kk < K) ? x : i32x4{0, 0, 0, 0};
            } else if constexpr (TRANS_B) {  // B [N][K]: row = n
                const int r = c >> 3, ch = c & 7;
                const int nn = min(n0 + r, N - 1), kk = k0 + ch * 8;
                const i32x4 x = *reinterpret_cast<const i32x4*>(Bm + (int64_t)nn * ldb + min(kk, K - 8));
                bst[i] = (n0 + r < N && kk < K) ? x : i32x4{0, 0, 0, 0};
            } else {  // B [K][N]: row = k (16 chunks of n)
                const int r = c >> 4, ch = c & 15;
                const int kk = min(k0 + r, K - 1), nn = n0 + ch * 8;
                const i32x4 x = *reinterpret_cast<const i32x4*>(Bm + (int64_t)kk * ldb + min(nn, N - 8));
                bst[i] = (k0 + r < K && nn < N) ? x : i32x4{0, 0, 0, 0};
            }
        }
    };
    auto store_tile = [&](int buf) {
        char* as = smem + buf * 2 * TILE;
        char* bs = as + TILE;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int c = tid + 256 * i;
            lds_write_b128(as, off128(c >> 3, c & 7), ast[i]);
            if constexpr (TRANS_B)
                lds_write_b128(bs, off128(c >> 3, c & 7), bst[i]);
            else
                lds_write_b128(bs, off256(c >> 4, c & 15), bst[i]);
        }
    };

    f32x16 acc[2][2];  // [n-block][m-block] of C^T
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int g = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;

    load_tile(0);
    store_tile(0);
    __syncthreads();
    for (int kt = 0; kt < ktiles; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < ktiles) load_tile(kt + 1);
        const char* as = smem + buf * 2 * TILE;
        const char* bs = as + TILE;
#pragma unroll
        for (int kk = 0; kk < BK / 16; ++kk) {
            i32x4 af[2], bf[2];
#pragma unroll
            for (int mi = 0; mi < 2; ++mi)
                af[mi] = lds_read_b128(as, off128(wm * 64 + mi * 32 + l32, 2 * kk + h32));
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) {
                if constexpr (TRANS_B) {
                    bf[ni] = lds_read_b128(bs, off128(wn * 64 + ni * 32 + l32, 2 * kk + h32));
                } else {
                    // rows k = 16kk + 8h32 + {0..3} and {4..7}; cols n = 32-block + lane
                    const int row = 16 * kk + 8 * h32 + qq;
                    const int ch = (wn * 64 + ni * 32) / 8 + 2 * (g & 1) + (pp >> 1);
                    const i32x2 lo = lds_read_tr16(bs, off256(row, ch) + 8 * (pp & 1));
                    const i32x2 hi = lds_read_tr16(bs, off256(row + 4, ch) + 8 * (pp & 1));
                    bf[ni] = i32x4{lo.x, lo.y, hi.x, hi.y};
                }
            }
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
#pragma unroll
                for (int mi = 0; mi < 2; ++mi)
                    acc[ni][mi] = mfma32x32x16<T>(bf[ni], af[mi], acc[ni][mi]);
        }
        if (kt + 1 < ktiles) store_tile(buf ^ 1);
        __syncthreads();
    }

    if constexpr (SWIGLU) {
        // up waves park their accumulators; gate waves combine and store
        float* xu = reinterpret_cast<float*>(smem) + wm * (2 * 2 * 16 * 64);
        if (wn == 1) {
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
#pragma unroll
                for (int mi = 0; mi < 2; ++mi)
#pragma unroll
                    for (int r = 0; r < 16; ++r) xu[((ni * 2 + mi) * 16 + r) * 64 + lane] = acc[ni][mi][r];
        }
        __syncthreads();
        if (wn == 1) return;
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) {
            const int m = m0 + wm * 64 + mi * 32 + l32;
            if (m >= M) continue;
            uint16_t* crow = C + (int64_t)m * ldc;
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int n = n0 + ni * 32 + 8 * i + 4 * h32;
                    if (n >= N) continue;
                    float v[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        v[j] = silu_mul(acc[ni][mi][4 * i + j],
                                        xu[((ni * 2 + mi) * 16 + 4 * i + j) * 64 + lane]);
                    *reinterpret_cast<i32x2*>(crow + n) =
                        i32x2{(int)pack2<T>(v[0], v[1]), (int)pack2<T>(v[2], v[3])};
                }
        }
        return;
    }
    // epilogue: acc[ni][mi][r] = C[m = m0+wm*64+mi*32+l32][n = n0+wn*64+ni*32+(r&3)+8(r>>2)+4h32]
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
        const int m = m0 + wm * 64 + mi * 32 + l32;
        if (m >= M) continue;
        uint16_t* crow = C + (int64_t)m * ldc;
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int n = n0 + wn * 64 + ni * 32 + 8 * i + 4 * h32;
                if (n >= N) continue;  // N % 8 == 0 on this path: whole quads
                float v0 = acc[ni][mi][4 * i], v1 = acc[ni][mi][4 * i + 1];
                float v2 = acc[ni][mi][4 * i + 2], v3 = acc[ni][mi][4 * i + 3];
                if constexpr (BIAS) {
                    v0 += elem<T>::to_f32(T{bias[n]});
                    v1 += elem<T>::to_f32(T{bias[n + 1]});
                    v2 += elem<T>::to_f32(T{bias[n + 2]});
                    v3 += elem<T>::to_f32(T{bias[n + 3]});
                }
                *reinterpret_cast<i32x2*>(crow + n) =
                    i32x2{(int)pack2<T>(v0, v1), (int)pack2<T>(v2, v3)};
            }
    }
}

// ---------------------------------------------------------------------------
// 256x256 tile, 8 waves (2 in M x 4 in N, 128x64 outputs each), BK = 64, on
// v_mfma_f32_16x16x32 (C^T = B^T A^T, so a lane owns an output row and 4
// consecutive columns per accumulator).  Operand tiles arrive by LDS-DMA
// (global_load_lds_dwordx4, 1 KiB per wave-instruction, lane-linear): the
// swizzles below are applied on the SOURCE address.  K-tile t+1 is in flight
// (second LDS buffer, 2 x 64 KiB) while t is computed; vmcnt(0) + barrier
// per K-tile.  One block per CU; 256 blocks at 4096^2.
//   A, NT B: [256 rows][64 k] (128-B rows), chunk ^= (row >> 1) & 7 --
//            conflict-free for the 16x16x32 fragment read (16 rows x 16 B
//            per lane group).
//   NN B:    [64 k][256 n] (512-B rows), fragment = two ds_read_b64_tr_b16,
//            chunk ^= 2 * ((k & 3) | ((k >> 3) & 1) << 2) -- each half-wave's
//            8 rows x 32 B land on 64 distinct banks.
constexpr int G2M = 256, G2N = 256, G2K = 64;

__device__ __forceinline__ int g2_off_rows(int row, int c) {  // 128-B rows
    return row * 128 + ((c ^ ((row >> 1) & 7)) << 4);
}
__device__ __forceinline__ int g2_fnn(int k) { return 2 * ((k & 3) | (((k >> 3) & 1) << 2)); }

// Logical tile index -> output tile.  group_m == 0: row-major.  Otherwise
// bands of group_m tile rows are swept column by column, so the ~32 blocks an
// XCD runs at once (consecutive indices after xcd_remap) cover a
// group_m x (32 / group_m) patch: group_m A panels and 32 / group_m B panels
// per K-step instead of 1 A panel and 32 B panels.
__device__ __forceinline__ void g2_tile(int lb, int tiles_m, int tiles_n, int group_m, int& tm,
                                        int& tn) {
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

template <typename T, bool TRANS_B, bool BIAS, bool PRIO = false>
__global__ __launch_bounds__(512, 2) void gemm_256(const uint16_t* __restrict__ A,
                                                   const uint16_t* __restrict__ Bm,
                                                   uint16_t* __restrict__ C,
                                                   const uint16_t* __restrict__ bias, int M, int N,
                                                   int K, int64_t lda, int64_t ldb, int64_t ldc,
                                                   int tiles_n, int nblocks, int group_m) {
    constexpr int TA = G2M * G2K * 2;  // 32 KiB
    constexpr int TB = G2N * G2K * 2;  // 32 KiB
    constexpr int BUF = TA + TB;
    __shared__ __attribute__((aligned(16))) char smem[2 * BUF];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 2, wc = wave & 3;
    const int l16 = lane & 15, g = lane >> 4;
    const int lb = xcd_remap(blockIdx.x, nblocks);
    int tmi, tni;
    g2_tile(lb, cdiv(M, G2M), tiles_n, group_m, tmi, tni);
    const int m0 = tmi * G2M, n0 = tni * G2N;
    const int ktiles = K / G2K;

    // DMA plan: 32 pieces of 1 KiB per operand tile, 4 per wave each.
    auto dma = [&](int kt, int buf) {
        char* as = smem + buf * BUF;
        char* bs = as + TA;
        const int k0 = kt * G2K;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int piece = wave * 4 + i;          // rows 8*piece .. +7
            const int row = piece * 8 + (lane >> 3), slot = lane & 7;
            const int c = slot ^ ((row >> 1) & 7);
            const int mm = min(m0 + row, M - 1);
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void*)(A + (int64_t)mm * lda + k0 + 8 * c),
                (__attribute__((address_space(3))) void*)(as + piece * 1024), 16, 0, 0);
            if constexpr (TRANS_B) {
                const int nn = min(n0 + row, N - 1);
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void*)(Bm + (int64_t)nn * ldb + k0 + 8 * c),
                    (__attribute__((address_space(3))) void*)(bs + piece * 1024), 16, 0, 0);
            } else {
                // [64 k][256 n]: piece = rows 2*piece, 2*piece+1 (512 B each)
                const int kr = piece * 2 + (lane >> 5), sl = lane & 31;
                const int cn = sl ^ g2_fnn(kr);
                const int ncol = min(n0 + 8 * cn, N - 8);
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void*)(Bm + (int64_t)(k0 + kr) * ldb + ncol),
                    (__attribute__((address_space(3))) void*)(bs + piece * 1024), 16, 0, 0);
            }
        }
    };

    f32x4 acc[4][8];  // [n-frag][m-frag] of C^T
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int qq = l16 >> 2, pp = lane & 3;
    dma(0, 0);
    __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) lgkmcnt(0) expcnt(0)
    __syncthreads();
    for (int kt = 0; kt < ktiles; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < ktiles) dma(kt + 1, buf ^ 1);
        const char* as = smem + buf * BUF;
        const char* bs = as + TA;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            i32x4 af[8], bf[4];
#pragma unroll
            for (int mi = 0; mi < 8; ++mi)
                af[mi] = lds_read_b128(as, g2_off_rows(wr * 128 + mi * 16 + l16, 4 * s + g));
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) {
                if constexpr (TRANS_B) {
                    bf[ni] = lds_read_b128(bs, g2_off_rows(wc * 64 + ni * 16 + l16, 4 * s + g));
                } else {
                    // k rows 32s + 8g + qq (+4), n cols wc*64 + ni*16 + 4pp
                    const int kr = 32 * s + 8 * g + qq;
                    const int nc = wc * 64 + ni * 16 + 4 * pp;  // element column
                    const int c = nc >> 3, within = (nc & 7) * 2;
                    const i32x2 lo = lds_read_tr16(bs, kr * 512 + ((c ^ g2_fnn(kr)) << 4) + within);
                    const i32x2 hi = lds_read_tr16(bs, (kr + 4) * 512 + ((c ^ g2_fnn(kr + 4)) << 4) + within);
                    bf[ni] = i32x4{lo.x, lo.y, hi.x, hi.y};
                }
            }
            if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int ni = 0; ni < 4; ++ni)
#pragma unroll
                for (int mi = 0; mi < 8; ++mi) acc[ni][mi] = mfma16x16x32<T>(bf[ni], af[mi], acc[ni][mi]);
            if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
        }
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
    }

    // epilogue: acc[ni][mi][r] = C[m0 + wr*128 + mi*16 + l16][n0 + wc*64 + ni*16 + 4g + r]
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
        const int m = m0 + wr * 128 + mi * 16 + l16;
        if (m >= M) continue;
        uint16_t* crow = C + (int64_t)m * ldc;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
            const int n = n0 + wc * 64 + ni * 16 + 4 * g;
            if (n >= N) continue;
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                v[r] = acc[ni][mi][r];
                if constexpr (BIAS) v[r] += elem<T>::to_f32(T{bias[n + r]});
            }
            *reinterpret_cast<i32x2*>(crow + n) = i32x2{(int)pack2<T>(v[0], v[1]), (int)pack2<T>(v[2], v[3])};
        }
    }
}

// ---------------------------------------------------------------------------
// gemm_256p: the 256x256 tile with a phased pipeline (4 phases per K-tile,
// 16 MFMAs each; after the guide's 8-phase template, schedule derived here).
// Each half-tile (A rows 0-127 "At", 128-255 "Ab", B rows/cols likewise "Bt",
// "Bb"; 16 KiB) is one LDS-DMA unit.  A wave owns 64 rows of each A half and
// 32 columns of each B half, so phase p reads only:
//   P1: At + Bt fragments  -> C(At, Bt)      P2: Bb -> C(At, Bb)
//   P3: Ab -> C(Ab, Bb)                       P4: (registers) -> C(Ab, Bt)
// One half-tile is DMA'd per phase, 5-6 phases ahead of its first read:
//   P1(t): Bb(t+1)  P2(t): Ab(t+1)  P3(t): At(t+2)  P4(t): Bt(t+2)
// into buffer kt & 1; every restage is >= 2 phases after the last read of the
// old contents, so one barrier per phase orders it.  A half read in phase p is
// retired by a counted vmcnt in phase p-1 before that phase's barrier
// (vmcnt(8): the 4 half-tiles issued after it may stay in flight; vmcnt(0)
// once the issue stream has run out).  All LDS in one __shared__ array, raw
// s_barrier, sched_barrier at the phase edges so hipcc keeps the order.
//
// SCHED bits (A/B; 0 = the schedule above):
//  1: the guide's two barriers per phase with waves 4-7 (wr = 1) one barrier
//     behind: a phase is {reads + DMA issue} barrier {MFMAs} barrier, so the
//     two waves on each SIMD alternate a read segment with an MFMA segment.
//     With the stagger, all reads of phase p are retired by the barrier that
//     ends the lagging half's MFMA segment of phase p; the restage points
//     above are >= 2 phases later and the counted waits stay one phase
//     ahead of the first read, so the same issue plan is race-free.
//  2: s_setprio(1) around each MFMA cluster
//  4: the phase's fragment reads issued before its DMA (template order)
// SWIGLU (NT): C[m, n] = silu(A Bg^T) * (A Bu^T) on a 256 x 128 output tile:
// the Bt half-tile holds Bg rows n0..n0+127 and Bb the same rows of Bu, so a
// lane's acc[ni] (gate) and acc[ni + 2] (up) are the same (m, n).
//
// The tile body is shared by the dense kernel (gemm_256p) and the grouped MoE
// kernel (gemm_256g): output rows m0 .. min(m0 + 256, mend) - 1, A row r read
// from A[amap ? amap[r] : r] (the per-lane source rows are loaded once before
// the first DMA: a gather load inside the pipeline would make hipcc drain the
// LDS-DMA queue with vmcnt(0) at its use).
constexpr int G2P_LDS = 2 * 4 * 16384;

template <typename T, bool TRANS_B, bool BIAS, int SCHED, bool SWIGLU>
__device__ __forceinline__ void g256p_body(char* __restrict__ smem, const uint16_t* __restrict__ A,
                                           int64_t lda, const int* __restrict__ amap, int m0,
                                           int mend, const uint16_t* __restrict__ Bm, int64_t ldb,
                                           const uint16_t* __restrict__ Bu, int64_t ldbu, int n0,
                                           int N, int K, uint16_t* __restrict__ C, int64_t ldc,
                                           const uint16_t* __restrict__ bias) {
    static_assert(!SWIGLU || (TRANS_B && !BIAS), "SwiGLU tile: NT, no bias");
    constexpr int HT = 16384, BUF = 4 * HT;
    constexpr int AT = 0, AB = 1, BT = 2, BB = 3;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 2, wc = wave & 3;
    const int l16 = lane & 15, g = lane >> 4, qq = l16 >> 2, pp = lane & 3;
    const int M = mend;
    const int ktiles = K / G2K;
    // source rows of this lane's A pieces: [half AT/AB][piece i]
    int arow[2][2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int r = min(m0 + 128 * h + (wave * 2 + i) * 8 + (lane >> 3), mend - 1);
            arow[h][i] = amap ? amap[r] : r;
        }

    auto issue = [&](int half, int kt) {
        if (kt >= ktiles) return;
        char* dst = smem + (kt & 1) * BUF + half * HT;
        const int k0 = kt * G2K;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int piece = wave * 2 + i;
            if (half == AT || half == AB || TRANS_B) {
                const int row = piece * 8 + (lane >> 3), slot = lane & 7;
                const int c = slot ^ ((row >> 1) & 7);
                const uint16_t* src;
                if (half == AT || half == AB)
                    src = A + (int64_t)arow[half == AB ? 1 : 0][i] * lda;
                else if constexpr (SWIGLU)
                    src = half == BB ? Bu + (int64_t)min(n0 + row, N - 1) * ldbu
                                     : Bm + (int64_t)min(n0 + row, N - 1) * ldb;
                else
                    src = Bm + (int64_t)min(n0 + (half == BB ? 128 : 0) + row, N - 1) * ldb;
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void*)(src + k0 + 8 * c),
                    (__attribute__((address_space(3))) void*)(dst + piece * 1024), 16, 0, 0);
            } else {  // NN B half: [64 k][128 n], 256-B rows, 4 rows per piece
                const int row = piece * 4 + (lane >> 4), slot = lane & 15;
                const int c = slot ^ g2_fnn(row);
                const int ncol = min(n0 + (half == BB ? 128 : 0) + 8 * c, N - 8);
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void*)(Bm + (int64_t)(k0 + row) * ldb + ncol),
                    (__attribute__((address_space(3))) void*)(dst + piece * 1024), 16, 0, 0);
            }
        }
    };
    auto read_a = [&](const char* half, int mi, int s) {
        return lds_read_b128(half, g2_off_rows(wr * 64 + mi * 16 + l16, 4 * s + g));
    };
    auto read_b = [&](const char* half, int ni, int s) {
        if constexpr (TRANS_B) {
            return lds_read_b128(half, g2_off_rows(wc * 32 + ni * 16 + l16, 4 * s + g));
        } else {
            const int kr = 32 * s + 8 * g + qq;
            const int nc = wc * 32 + ni * 16 + 4 * pp;
            const int c = nc >> 3, within = (nc & 7) * 2;
            const i32x2 lo = lds_read_tr16(half, kr * 256 + ((c ^ g2_fnn(kr)) << 4) + within);
            const i32x2 hi = lds_read_tr16(half, (kr + 4) * 256 + ((c ^ g2_fnn(kr + 4)) << 4) + within);
            return i32x4{lo.x, lo.y, hi.x, hi.y};
        }
    };
    auto wait_vm = [&](bool drain) {
        if (drain) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    };
    auto sync = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr ((SCHED & 2) != 0) __builtin_amdgcn_s_setprio(1);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto sync_end = [&]() {  // end of a phase's MFMA cluster
        if constexpr ((SCHED & 3) != 0) {
            __builtin_amdgcn_sched_barrier(0);
            if constexpr ((SCHED & 2) != 0) __builtin_amdgcn_s_setprio(0);
            if constexpr ((SCHED & 1) != 0) __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    constexpr bool kReadFirst = (SCHED & 4) != 0;

    f32x4 acc[4][8];  // [n-frag: 0,1 = Bt, 2,3 = Bb][m-frag: 0-3 = At, 4-7 = Ab]
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // prologue: K-tile 0 complete-able, At/Bt of K-tile 1 in flight
    issue(AT, 0);
    issue(BT, 0);
    issue(BB, 0);
    issue(AB, 0);
    issue(AT, 1);
    issue(BT, 1);
    wait_vm(ktiles < 2);  // retires At(0), Bt(0)
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    if constexpr ((SCHED & 1) != 0) {
        if (wr == 1) __builtin_amdgcn_s_barrier();  // the lagging half
    }
    __builtin_amdgcn_sched_barrier(0);

    i32x4 fat[4][2], fab[4][2], fbt[2][2], fbb[2][2];
    for (int kt = 0; kt < ktiles; ++kt) {
        const char* base = smem + (kt & 1) * BUF;
        const bool drain = kt + 2 >= ktiles;
        // ---- P1: At + Bt -> C(At, Bt)
        if constexpr (!kReadFirst) issue(BB, kt + 1);
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) fbt[ni][s2] = read_b(base + BT * HT, ni, s2);
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) fat[mi][s2] = read_a(base + AT * HT, mi, s2);
        if constexpr (kReadFirst) issue(BB, kt + 1);
        wait_vm(drain);  // retires Bb(kt), read in P2
        sync();
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
                    acc[ni][mi] = mfma16x16x32<T>(fbt[ni][s2], fat[mi][s2], acc[ni][mi]);
        sync_end();
        // ---- P2: Bb -> C(At, Bb)
        if constexpr (!kReadFirst) issue(AB, kt + 1);
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) fbb[ni][s2] = read_b(base + BB * HT, ni, s2);
        if constexpr (kReadFirst) issue(AB, kt + 1);
        wait_vm(drain);  // retires Ab(kt), read in P3
        sync();
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
                    acc[2 + ni][mi] = mfma16x16x32<T>(fbb[ni][s2], fat[mi][s2], acc[2 + ni][mi]);
        sync_end();
        // ---- P3: Ab -> C(Ab, Bb)
        if constexpr (!kReadFirst) issue(AT, kt + 2);
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) fab[mi][s2] = read_a(base + AB * HT, mi, s2);
        if constexpr (kReadFirst) issue(AT, kt + 2);
        sync();
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
                    acc[2 + ni][4 + mi] = mfma16x16x32<T>(fbb[ni][s2], fab[mi][s2], acc[2 + ni][4 + mi]);
        sync_end();
        // ---- P4: registers -> C(Ab, Bt)
        issue(BT, kt + 2);
        wait_vm(drain);  // retires At(kt+1), Bt(kt+1), read in the next P1
        sync();
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
                    acc[ni][4 + mi] = mfma16x16x32<T>(fbt[ni][s2], fab[mi][s2], acc[ni][4 + mi]);
        sync_end();
    }
    if constexpr ((SCHED & 1) != 0) {
        if (wr == 0) __builtin_amdgcn_s_barrier();  // equal barrier counts
    }

    // epilogue: acc[ni][mi][r] = C[m][n], m = m0 + (mi>>2)*128 + wr*64 + (mi&3)*16 + l16,
    //                                     n = n0 + (ni>>1)*128 + wc*32 + (ni&1)*16 + 4g + r
    if constexpr (SWIGLU) {  // gate acc[ni], up acc[ni + 2] of column n0 + wc*32 + ni*16 + 4g + r
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) {
            const int m = m0 + (mi >> 2) * 128 + wr * 64 + (mi & 3) * 16 + l16;
            if (m >= M) continue;
            uint16_t* crow = C + (int64_t)m * ldc;
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) {
                const int n = n0 + wc * 32 + ni * 16 + 4 * g;
                if (n >= N) continue;
                float v[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = silu_mul(acc[ni][mi][r], acc[ni + 2][mi][r]);
                *reinterpret_cast<i32x2*>(crow + n) = i32x2{(int)pack2<T>(v[0], v[1]), (int)pack2<T>(v[2], v[3])};
            }
        }
        return;
    }
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
        const int m = m0 + (mi >> 2) * 128 + wr * 64 + (mi & 3) * 16 + l16;
        if (m >= M) continue;
        uint16_t* crow = C + (int64_t)m * ldc;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
            const int n = n0 + (ni >> 1) * 128 + wc * 32 + (ni & 1) * 16 + 4 * g;
            if (n >= N) continue;
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                v[r] = acc[ni][mi][r];
                if constexpr (BIAS) v[r] += elem<T>::to_f32(T{bias[n + r]});
            }
            *reinterpret_cast<i32x2*>(crow + n) = i32x2{(int)pack2<T>(v[0], v[1]), (int)pack2<T>(v[2], v[3])};
        }
    }
}


template <typename T, bool TRANS_B, bool BIAS, int SCHED = 0, bool SWIGLU = false>
__global__ __launch_bounds__(512, 2) void gemm_256p(const uint16_t* __restrict__ A,
                                                    const uint16_t* __restrict__ Bm,
                                                    uint16_t* __restrict__ C,
                                                    const uint16_t* __restrict__ bias, int M, int N,
                                                    int K, int64_t lda, int64_t ldb, int64_t ldc,
                                                    int tiles_n, int nblocks, int group_m,
                                                    const uint16_t* __restrict__ Bu, int64_t ldbu) {
    constexpr int TN = SWIGLU ? 128 : G2N;  // output columns per tile
    __shared__ __attribute__((aligned(16))) char smem[G2P_LDS];
    const int lb = xcd_remap(blockIdx.x, nblocks);
    int tmi, tni;
    g2_tile(lb, cdiv(M, G2M), tiles_n, group_m, tmi, tni);
    g256p_body<T, TRANS_B, BIAS, SCHED, SWIGLU>(smem, A, lda, nullptr, tmi * G2M, M, Bm, ldb, Bu,
                                                ldbu, tni * TN, N, K, C, ldc, bias);
}

// Grouped MoE GEMM on the phased tile: expert e owns the expert-sorted rows
// offsets[e] .. offsets[e+1]-1 (device table, pli_moe_route); its rows are cut
// into 256-row slots, slot s of the launch (slots_bound = cdiv(rows, 256) + E,
// an upper bound) is found by a scalar scan of the offsets, and blocks past
// the real slot count exit before any barrier.  A rows are read through
// `gather` (row -> token of x; NULL: A is already expert-sorted), B is expert
// e's weight (W[e], for SWIGLU gate W[e] / up Wu[e]), C rows are the sorted rows.
template <typename T, bool SWIGLU>
__global__ __launch_bounds__(512, 2) void gemm_256g(const uint16_t* __restrict__ X, int64_t ldx,
                                                    const int* __restrict__ gather,
                                                    const uint16_t* const* __restrict__ W,
                                                    const uint16_t* const* __restrict__ Wu,
                                                    int64_t ldw, uint16_t* __restrict__ C,
                                                    int64_t ldc, const int* __restrict__ offsets,
                                                    int E, int N, int K, int slots, int tiles_n,
                                                    int nblocks) {
    constexpr int TN = SWIGLU ? 128 : G2N;
    __shared__ __attribute__((aligned(16))) char smem[G2P_LDS];
    const int lb = xcd_remap(blockIdx.x, nblocks);
    int slot, tni;
    g2_tile(lb, slots, tiles_n, 4, slot, tni);
    int e = -1, rbeg = 0, rend = 0, acc = 0;
    for (int j = 0; j < E; ++j) {
        const int b0 = offsets[j], b1 = offsets[j + 1];
        const int nt = (b1 - b0 + G2M - 1) / G2M;
        if (slot < acc + nt) {
            e = j;
            rbeg = b0 + (slot - acc) * G2M;
            rend = b1;
            break;
        }
        acc += nt;
    }
    if (e < 0) return;  // whole block: before any barrier
    g256p_body<T, true, false, 7, SWIGLU>(smem, X, ldx, gather, rbeg, rend, W[e], ldw,
                                          SWIGLU ? Wu[e] : nullptr, ldw, tni * TN, N, K, C, ldc,
                                          nullptr);
}

// ---------------------------------------------------------------------------
// Generic LDS-tiled kernel (any dtype, any shape/stride), fp32 accumulate.
constexpr int GT = 64, GKT = 16;

// SWIGLU (NT): the 64-column B tile is 32 gate + 32 up columns of the same
// 32 outputs, so thread columns j = 0/2 and 1/3 pair up in registers.
template <typename T, bool TRANS_B, bool SWIGLU = false>
__global__ __launch_bounds__(256) void gemm_generic(const T* __restrict__ A, const T* __restrict__ Bm,
                                                    T* __restrict__ C, const T* __restrict__ bias,
                                                    int M, int N, int K, int64_t lda, int64_t ldb,
                                                    int64_t ldc, const T* __restrict__ Bu = nullptr,
                                                    int64_t ldbu = 0) {
    __shared__ float As[GKT][GT + 4];
    __shared__ float Bs[GKT][GT + 4];
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    const int m0 = blockIdx.y * GT, n0 = blockIdx.x * (SWIGLU ? GT / 2 : GT);
    float acc[4][4] = {};
    for (int k0 = 0; k0 < K; k0 += GKT) {
        for (int i = tid; i < GT * GKT; i += 256) {
            {   // A[m][k] -> As[k][m]
                const int r = i / GKT, kk = i % GKT;
                const int m = m0 + r, kx = k0 + kk;
                As[kk][r] = (m < M && kx < K) ? elem<T>::to_f32(A[(int64_t)m * lda + kx]) : 0.f;
            }
            if constexpr (SWIGLU) {  // cols 0..31 gate, 32..63 up of outputs n0 + (r & 31)
                const int r = i / GKT, kk = i % GKT;
                const int n = n0 + (r & 31), kx = k0 + kk;
                const T* src = r < 32 ? Bm + (int64_t)n * ldb : Bu + (int64_t)n * ldbu;
                Bs[kk][r] = (n < N && kx < K) ? elem<T>::to_f32(src[kx]) : 0.f;
            } else if constexpr (TRANS_B) {  // B[n][k] -> Bs[k][n]
                const int r = i / GKT, kk = i % GKT;
                const int n = n0 + r, kx = k0 + kk;
                Bs[kk][r] = (n < N && kx < K) ? elem<T>::to_f32(Bm[(int64_t)n * ldb + kx]) : 0.f;
            } else {  // B[k][n] -> Bs[k][n]
                const int kk = i / GT, r = i % GT;
                const int n = n0 + r, kx = k0 + kk;
                Bs[kk][r] = (n < N && kx < K) ? elem<T>::to_f32(Bm[(int64_t)kx * ldb + n]) : 0.f;
            }
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < GKT; ++kk) {
            float a[4], b[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = As[kk][ty + 16 * i];
#pragma unroll
            for (int j = 0; j < 4; ++j) b[j] = Bs[kk][tx + 16 * j];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a[i], b[j], acc[i][j]);
        }
        __syncthreads();
    }
    if constexpr (SWIGLU) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int m = m0 + ty + 16 * i;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int n = n0 + tx + 16 * j;
                if (m < M && n < N)
                    C[(int64_t)m * ldc + n] = elem<T>::from_f32(silu_mul(acc[i][j], acc[i][j + 2]));
            }
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = m0 + ty + 16 * i;
        if (m >= M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = n0 + tx + 16 * j;
            if (n >= N) continue;
            float vv = acc[i][j];
            if (bias) vv += elem<T>::to_f32(bias[n]);
            C[(int64_t)m * ldc + n] = elem<T>::from_f32(vv);
        }
    }
}

// ---------------------------------------------------------------------------
// Skinny NT path for decode batches (x @ W^T with M <= 16 rows of X,
// ch03/batching_benchmark.py:25-39): HBM-bound on W like the GEMV.  One W row
// per wave, each lane streams 16-byte W chunks (non-temporal, read once) and
// dots them with the matching chunk of every X row (X is tiny and stays in
// L1/L2); NB fp32 accumulators per lane, one shuffle reduction per output.
// SWIGLU: the wave streams row n of both Wg (W) and Wu and writes
// silu(x.wg) * (x.wu): one pass over the two weight rows, no gate/up tensors.
template <typename T, int NB, int CPL, bool SWIGLU = false>
__global__ __launch_bounds__(128) void gemm_skinny_nt(const uint16_t* __restrict__ X,
                                                      const uint16_t* __restrict__ W,
                                                      uint16_t* __restrict__ C,
                                                      const uint16_t* __restrict__ bias, int M,
                                                      int N, int nchunks, int64_t ldx, int64_t ldw,
                                                      int64_t ldc,
                                                      const uint16_t* __restrict__ Wu = nullptr,
                                                      int64_t ldwu = 0) {
    constexpr int NW = SWIGLU ? 2 : 1;  // weight rows per output
    const int lane = threadIdx.x & 63;
    const int n = blockIdx.x * 2 + (threadIdx.x >> 6);
    if (n >= N) return;
    const uint16_t* wrow[NW];
    wrow[0] = W + (int64_t)n * ldw;
    if constexpr (SWIGLU) wrow[NW - 1] = Wu + (int64_t)n * ldwu;
    float acc[NW][NB];
#pragma unroll
    for (int w = 0; w < NW; ++w)
#pragma unroll
        for (int bb = 0; bb < NB; ++bb) acc[w][bb] = 0.f;
    for (int c0 = 0; c0 < nchunks; c0 += 64 * CPL) {
        i32x4 wv[NW][CPL];
#pragma unroll
        for (int w = 0; w < NW; ++w)
#pragma unroll
            for (int u = 0; u < CPL; ++u) {
                const int cc = min(c0 + lane + 64 * u, nchunks - 1);
                wv[w][u] = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(wrow[w] + cc * 8));
            }
#pragma unroll
        for (int u = 0; u < CPL; ++u) {
            const int cc = c0 + lane + 64 * u;
            if (cc < nchunks) {
#pragma unroll
                for (int bb = 0; bb < NB; ++bb) {
                    if (bb < M) {
                        const i32x4 xv = *reinterpret_cast<const i32x4*>(X + bb * ldx + cc * 8);
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int xi = xv[i];
                            const float x0 = elem<T>::to_f32(T{(uint16_t)(xi & 0xffff)});
                            const float x1 = elem<T>::to_f32(T{(uint16_t)((uint32_t)xi >> 16)});
#pragma unroll
                            for (int w = 0; w < NW; ++w) {
                                const int wi = wv[w][u][i];
                                const float w0 = elem<T>::to_f32(T{(uint16_t)(wi & 0xffff)});
                                const float w1 = elem<T>::to_f32(T{(uint16_t)((uint32_t)wi >> 16)});
                                acc[w][bb] = fmaf(w1, x1, fmaf(w0, x0, acc[w][bb]));
                            }
                        }
                    }
                }
            }
        }
    }
    const float bn = (!SWIGLU && bias) ? elem<T>::to_f32(T{bias[n]}) : 0.f;
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) {
        if (bb < M) {
            float r = wave_sum(acc[0][bb]);
            if constexpr (SWIGLU) r = silu_mul(r, wave_sum(acc[NW - 1][bb]));
            if (lane == 0) C[bb * ldc + n] = __builtin_bit_cast(uint16_t, elem<T>::from_f32(r + bn));
        }
    }
}

// Multi-output skinny NT GEMM for the decode step: up to 3 weight matrices
// (e.g. the q, k and v projections) against the same M <= 16 rows of X in
// ONE launch, each output with its own row addressing so the k / v rows can
// be written straight into a [B, S_max, Hkv, D] cache at a device-resident
// position: row r = b * S + s of group g goes to
//   c + b * stride_batch + (s + *row_offset) * stride_token   (+ column n),
// and is dropped when s + *row_offset >= capacity.  One wave per output
// column, as gemm_skinny_nt; waves are assigned to groups by column range.
struct MultiGroup {
    const uint16_t* w;
    uint16_t* c;
    int n;
    int64_t ldw, stride_batch, stride_token;
    const int* row_offset;
    int capacity;
};
struct MultiArgs {
    MultiGroup g[3];
    int ngroups;
};

template <typename T, int NB, int CPL = 8>
__global__ __launch_bounds__(128) void gemm_skinny_multi(const uint16_t* __restrict__ X, int M,
                                                         int S, int nchunks, int64_t ldx,
                                                         MultiArgs args) {
    const int lane = threadIdx.x & 63;
    int n = blockIdx.x * 2 + (threadIdx.x >> 6);
    int gi = 0;
    while (gi < args.ngroups && n >= args.g[gi].n) n -= args.g[gi++].n;
    if (gi >= args.ngroups) return;
    const MultiGroup& G = args.g[gi];
    const uint16_t* wrow = G.w + (int64_t)n * G.ldw;
    float acc[NB];
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) acc[bb] = 0.f;
    for (int c0 = 0; c0 < nchunks; c0 += 64 * CPL) {
        i32x4 wv[CPL];
#pragma unroll
        for (int u = 0; u < CPL; ++u) {
            const int cc = min(c0 + lane + 64 * u, nchunks - 1);
            wv[u] = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(wrow + cc * 8));
        }
#pragma unroll
        for (int u = 0; u < CPL; ++u) {
            const int cc = c0 + lane + 64 * u;
            if (cc < nchunks) {
#pragma unroll
                for (int bb = 0; bb < NB; ++bb) {
                    if (bb < M) {
                        const i32x4 xv = *reinterpret_cast<const i32x4*>(X + bb * ldx + cc * 8);
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int wi = wv[u][i], xi = xv[i];
                            const float w0 = elem<T>::to_f32(T{(uint16_t)(wi & 0xffff)});
                            const float w1 = elem<T>::to_f32(T{(uint16_t)((uint32_t)wi >> 16)});
                            const float x0 = elem<T>::to_f32(T{(uint16_t)(xi & 0xffff)});
                            const float x1 = elem<T>::to_f32(T{(uint16_t)((uint32_t)xi >> 16)});
                            acc[bb] = fmaf(w1, x1, fmaf(w0, x0, acc[bb]));
                        }
                    }
                }
            }
        }
    }
    const int off = G.row_offset ? *G.row_offset : 0;
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) {
        if (bb < M) {
            const float r = wave_sum(acc[bb]);
            const int b = bb / S, srow = bb % S + off;
            if (lane == 0 && srow < G.capacity)
                G.c[b * G.stride_batch + (int64_t)srow * G.stride_token + n] =
                    __builtin_bit_cast(uint16_t, elem<T>::from_f32(r));
        }
    }
}

template <typename T>
int launch_skinny(const void* a, const void* b, void* c, const void* bias, int M, int N, int K,
                  int64_t lda, int64_t ldb, int64_t ldc, hipStream_t s) {
    const dim3 grid(cdiv(N, 2)), block(128);
    const int nch = K / 8;
#define PLI_SKINNY(NB, CPL)                                                                   \
    hipLaunchKernelGGL((gemm_skinny_nt<T, NB, CPL>), grid, block, 0, s, (const uint16_t*)a,   \
                       (const uint16_t*)b, (uint16_t*)c, (const uint16_t*)bias, M, N, nch, lda, \
                       ldb, ldc)
    // M <= 4 with K <= 8192: every load of a row in one batch (CPL = chunks per
    // lane rounded up to 4, at least 8), so a wave waits on HBM once.  With
    // CPL 8, a 5632-column row takes two round trips. That row is the decode
    // step's down projection, where CPL 12 cuts 9.1 us to 8.3 us per launch.
    // K <= 1024 / 2048 (<= 128 / 256 chunks): CPL 2 / 4, all 64 lanes carry the
    // row (the same per-lane chunk order as CPL 8, whose upper part would be
    // masked off, so bitwise the same result).
#define PLI_SKINNY_CPL(NB)                    \
    if (nch <= 128) PLI_SKINNY(NB, 2);        \
    else if (nch <= 256) PLI_SKINNY(NB, 4);   \
    else if (nch <= 512) PLI_SKINNY(NB, 8);   \
    else if (nch <= 768) PLI_SKINNY(NB, 12);  \
    else if (nch <= 1024) PLI_SKINNY(NB, 16); \
    else PLI_SKINNY(NB, 8);
    if (M <= 1) { PLI_SKINNY_CPL(1) }
    else if (M <= 2) { PLI_SKINNY_CPL(2) }
    else if (M <= 4) { PLI_SKINNY_CPL(4) }
    else if (M <= 8) PLI_SKINNY(8, 8);
    else PLI_SKINNY(16, 8);
#undef PLI_SKINNY_CPL
#undef PLI_SKINNY
    return launch_status("gemm_skinny_nt");
}

// ---------------------------------------------------------------------------
// Small-M NT path (16 < M <= 128 decode batches / short prefill chunks):
// C^T[16 W rows][M] = W[16 rows, K] . X^T on v_mfma_f32_16x16x32.  One
// workgroup per 16 W rows (N/16 workgroups: 256 at N=4096, one per CU), K
// split over its 4 waves; W fragments (16 rows x 64 B per wave-instruction)
// are streamed from HBM exactly once and feed NBG MFMAs (one per 16 batch
// rows), X fragments come from L2.  Partial C^T tiles are summed through LDS.
// SWIGLU: each wave streams the 16 rows of Wg (W) AND of Wu over its K range
// into two accumulators per batch group; the epilogue writes silu(g) * u.
// MULTI (pli_gemm_multi_nt at 16 < m <= 128): the columns are the
// concatenated groups of `margs` (each a multiple of 16 wide, so a workgroup's
// 16 columns lie in one group) and row r = b * mtok + s of group g is stored
// at c_g + b * stride_batch + (s + *row_offset) * stride_token, as
// gemm_skinny_multi does: the packed q/k/v GEMM writes k / v straight into
// the caches.
template <typename T, int NBG, bool BIAS, bool SWIGLU = false, bool MULTI = false>
__global__ __launch_bounds__(256) void gemm_smallm_nt(const uint16_t* __restrict__ X,
                                                      const uint16_t* __restrict__ W,
                                                      uint16_t* __restrict__ C,
                                                      const uint16_t* __restrict__ bias, int M,
                                                      int N, int K, int64_t ldx, int64_t ldw,
                                                      int64_t ldc,
                                                      const uint16_t* __restrict__ Wu = nullptr,
                                                      int64_t ldwu = 0, MultiArgs margs = {},
                                                      int mtok = 1) {
    constexpr int NW = SWIGLU ? 2 : 1;     // weight matrices streamed
    constexpr int U = SWIGLU ? 4 : 8;      // k-steps issued ahead per wave (8 KiB of W in flight)
    __shared__ __attribute__((aligned(16))) float part[4][NBG][NW][4][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int n0 = blockIdx.x * 16;
    int gsel = 0;
    if constexpr (MULTI) {  // the host sizes the grid to the groups' total width
        while (gsel < margs.ngroups - 1 && n0 >= margs.g[gsel].n) n0 -= margs.g[gsel++].n;
        W = margs.g[gsel].w;
        ldw = margs.g[gsel].ldw;
        N = margs.g[gsel].n;
    }
    const int r16 = lane & 15, kq = 8 * (lane >> 4);
    const int kw = K / 4;  // this wave's K range
    const uint16_t* wp[NW];
    wp[0] = W + (int64_t)min(n0 + r16, N - 1) * ldw + wave * kw + kq;
    if constexpr (SWIGLU) wp[NW - 1] = Wu + (int64_t)min(n0 + r16, N - 1) * ldwu + wave * kw + kq;
    const uint16_t* xp[NBG];
#pragma unroll
    for (int gi = 0; gi < NBG; ++gi)
        xp[gi] = X + (int64_t)min(gi * 16 + r16, M - 1) * ldx + wave * kw + kq;
    f32x4 acc[NW][NBG];
#pragma unroll
    for (int w = 0; w < NW; ++w)
#pragma unroll
        for (int gi = 0; gi < NBG; ++gi) acc[w][gi] = f32x4{0.f, 0.f, 0.f, 0.f};
    int k0 = 0;
    for (; k0 + 32 * U <= kw; k0 += 32 * U) {
        i32x4 wf[NW][U], xf[U][NBG];
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int w = 0; w < NW; ++w)
                wf[w][u] = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(wp[w] + k0 + 32 * u));
#pragma unroll
            for (int gi = 0; gi < NBG; ++gi)
                xf[u][gi] = *reinterpret_cast<const i32x4*>(xp[gi] + k0 + 32 * u);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int w = 0; w < NW; ++w)
#pragma unroll
                for (int gi = 0; gi < NBG; ++gi)
                    acc[w][gi] = mfma16x16x32<T>(wf[w][u], xf[u][gi], acc[w][gi]);
    }
    for (; k0 < kw; k0 += 32) {  // remainder k-steps (kw % 32 == 0)
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const i32x4 wf = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(wp[w] + k0));
#pragma unroll
            for (int gi = 0; gi < NBG; ++gi)
                acc[w][gi] = mfma16x16x32<T>(wf, *reinterpret_cast<const i32x4*>(xp[gi] + k0), acc[w][gi]);
        }
    }
#pragma unroll
    for (int w = 0; w < NW; ++w)
#pragma unroll
        for (int gi = 0; gi < NBG; ++gi)
#pragma unroll
            for (int r = 0; r < 4; ++r) part[wave][gi][w][r][lane] = acc[w][gi][r];
    __syncthreads();
    // wave w reduces batch groups gi = w, w+4, ...; lane (col = batch, rows 4q..4q+3 = W rows)
    for (int gi = wave; gi < NBG; gi += 4) {
        const int bt = gi * 16 + r16;
        const int nr = n0 + 4 * (lane >> 4);
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            v[r] = part[0][gi][0][r][lane] + part[1][gi][0][r][lane] + part[2][gi][0][r][lane] +
                   part[3][gi][0][r][lane];
            if constexpr (SWIGLU)
                v[r] = silu_mul(v[r], part[0][gi][NW - 1][r][lane] + part[1][gi][NW - 1][r][lane] +
                                          part[2][gi][NW - 1][r][lane] + part[3][gi][NW - 1][r][lane]);
        }
        if constexpr (MULTI) {
            const MultiGroup& G = margs.g[gsel];
            const int b = bt / mtok, srow = bt % mtok + (G.row_offset ? *G.row_offset : 0);
            if (bt < M && nr < N && srow < G.capacity)
                *reinterpret_cast<i32x2*>(G.c + b * G.stride_batch + (int64_t)srow * G.stride_token + nr) =
                    i32x2{(int)pack2<T>(v[0], v[1]), (int)pack2<T>(v[2], v[3])};
        } else if (bt < M && nr < N) {
            if constexpr (BIAS) {
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] += elem<T>::to_f32(T{bias[nr + r]});
            }
            *reinterpret_cast<i32x2*>(C + (int64_t)bt * ldc + nr) =
                i32x2{(int)pack2<T>(v[0], v[1]), (int)pack2<T>(v[2], v[3])};
        }
    }
}

// Grouped (MoE expert) form of the small-M kernel: workgroup = (expert e,
// 16 output columns).  Expert e owns rows offsets[e] .. offsets[e+1]-1 of the
// permuted activation matrix; its X rows are read through `gather` (token
// index per permuted row, or identity when null), its weights through the
// device pointer table `w_ptrs[e]` (the reference keeps one nn.Linear per
// expert, ch09/moe_layer.py:36-45), and the rows are processed 16*NBG at a
// time (NBG sized on the host from the row bound, so decode batches run
// NBG = 1).  SWIGLU: w_ptrs / wu_ptrs are W1 / W3 and the output is
// silu(x W1^T) * (x W3^T).
template <typename T, int NBG, bool SWIGLU>
__global__ __launch_bounds__(256) void gemm_grouped_nt(
    const uint16_t* __restrict__ X, const int* __restrict__ gather,
    const uint16_t* const* __restrict__ w_ptrs, const uint16_t* const* __restrict__ wu_ptrs,
    uint16_t* __restrict__ C, const int* __restrict__ offsets, int N, int K, int64_t ldx,
    int64_t ldw, int64_t ldc, int nblk) {
    constexpr int NW = SWIGLU ? 2 : 1;
    constexpr int U = SWIGLU ? 4 : 8;
    __shared__ __attribute__((aligned(16))) float part[4][NBG][NW][4][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int e = blockIdx.x / nblk, n0 = (blockIdx.x % nblk) * 16;
    const int r0 = offsets[e], Me = offsets[e + 1] - r0;
    if (Me <= 0) return;
    const int r16 = lane & 15, kq = 8 * (lane >> 4);
    const int kw = K / 4;
    const uint16_t* wp[NW];
    wp[0] = w_ptrs[e] + (int64_t)min(n0 + r16, N - 1) * ldw + wave * kw + kq;
    if constexpr (SWIGLU) wp[NW - 1] = wu_ptrs[e] + (int64_t)min(n0 + r16, N - 1) * ldw + wave * kw + kq;
    for (int c0 = 0; c0 < Me; c0 += 16 * NBG) {
        const int M = min(16 * NBG, Me - c0);
        const uint16_t* xp[NBG];
#pragma unroll
        for (int gi = 0; gi < NBG; ++gi) {
            const int pr = r0 + c0 + min(gi * 16 + r16, M - 1);
            const int tok = gather ? gather[pr] : pr;
            xp[gi] = X + (int64_t)tok * ldx + wave * kw + kq;
        }
        f32x4 acc[NW][NBG];
#pragma unroll
        for (int w = 0; w < NW; ++w)
#pragma unroll
            for (int gi = 0; gi < NBG; ++gi) acc[w][gi] = f32x4{0.f, 0.f, 0.f, 0.f};
        int k0 = 0;
        for (; k0 + 32 * U <= kw; k0 += 32 * U) {
            i32x4 wf[NW][U], xf[U][NBG];
#pragma unroll
            for (int u = 0; u < U; ++u) {
#pragma unroll
                for (int w = 0; w < NW; ++w)
                    wf[w][u] = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(wp[w] + k0 + 32 * u));
#pragma unroll
                for (int gi = 0; gi < NBG; ++gi)
                    xf[u][gi] = *reinterpret_cast<const i32x4*>(xp[gi] + k0 + 32 * u);
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int w = 0; w < NW; ++w)
#pragma unroll
                    for (int gi = 0; gi < NBG; ++gi)
                        acc[w][gi] = mfma16x16x32<T>(wf[w][u], xf[u][gi], acc[w][gi]);
        }
        for (; k0 < kw; k0 += 32) {
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                const i32x4 wf = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(wp[w] + k0));
#pragma unroll
                for (int gi = 0; gi < NBG; ++gi)
                    acc[w][gi] = mfma16x16x32<T>(wf, *reinterpret_cast<const i32x4*>(xp[gi] + k0), acc[w][gi]);
            }
        }
        __syncthreads();  // part[] of the previous chunk fully consumed
#pragma unroll
        for (int w = 0; w < NW; ++w)
#pragma unroll
            for (int gi = 0; gi < NBG; ++gi)
#pragma unroll
                for (int r = 0; r < 4; ++r) part[wave][gi][w][r][lane] = acc[w][gi][r];
        __syncthreads();
        for (int gi = wave; gi < NBG; gi += 4) {
            const int bt = gi * 16 + r16;
            const int nr = n0 + 4 * (lane >> 4);
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                v[r] = part[0][gi][0][r][lane] + part[1][gi][0][r][lane] + part[2][gi][0][r][lane] +
                       part[3][gi][0][r][lane];
                if constexpr (SWIGLU)
                    v[r] = silu_mul(v[r], part[0][gi][NW - 1][r][lane] + part[1][gi][NW - 1][r][lane] +
                                              part[2][gi][NW - 1][r][lane] + part[3][gi][NW - 1][r][lane]);
            }
            if (bt < M && nr < N)
                *reinterpret_cast<i32x2*>(C + (int64_t)(r0 + c0 + bt) * ldc + nr) =
                    i32x2{(int)pack2<T>(v[0], v[1]), (int)pack2<T>(v[2], v[3])};
        }
    }
}

template <typename T>
int launch_smallm(const void* a, const void* b, void* c, const void* bias, int M, int N, int K,
                  int64_t lda, int64_t ldb, int64_t ldc, hipStream_t s) {
    const dim3 grid(cdiv(N, 16)), block(256);
#define PLI_SMALLM(G)                                                                          \
    do {                                                                                       \
        if (bias)                                                                              \
            hipLaunchKernelGGL((gemm_smallm_nt<T, G, true>), grid, block, 0, s,                \
                               (const uint16_t*)a, (const uint16_t*)b, (uint16_t*)c,           \
                               (const uint16_t*)bias, M, N, K, lda, ldb, ldc);                 \
        else                                                                                   \
            hipLaunchKernelGGL((gemm_smallm_nt<T, G, false>), grid, block, 0, s,               \
                               (const uint16_t*)a, (const uint16_t*)b, (uint16_t*)c,           \
                               (const uint16_t*)bias, M, N, K, lda, ldb, ldc);                 \
    } while (0)
    if (M <= 16) PLI_SMALLM(1);
    else if (M <= 32) PLI_SMALLM(2);
    else if (M <= 64) PLI_SMALLM(4);
    else PLI_SMALLM(8);
#undef PLI_SMALLM
    return launch_status("gemm_smallm_nt");
}

// ---------------------------------------------------------------------------
// Mid-M NT path (batched decode / TP shards at M ~ 32-256: the ch09 row shard
// at M = 128): C^T[32 W rows][<= 128 X rows] per workgroup on
// v_mfma_f32_32x32x16.  The workgroup's 32 weight rows are streamed from HBM
// exactly once (non-temporal), split over the 4 waves in K; every lane loads
// its MFMA fragments straight from global memory (W row n0 + l%32, X row
// m + l%32, 16 B at k + 8(l/32)), two 64-k steps in flight per wave, and the
// four K partials are summed through LDS.  N/32 workgroups (256 at N = 8192):
// X (the small operand) is re-read from L2 once per workgroup, half the L2
// traffic of the 16-row small-M kernel, which is what bounds that kernel at
// M = 128.  grid.y walks 128-row slabs of X for M > 128.
template <typename T, int MC, bool BIAS>
__global__ __launch_bounds__(256) void gemm_midm_nt(const uint16_t* __restrict__ X,
                                                    const uint16_t* __restrict__ W,
                                                    uint16_t* __restrict__ C,
                                                    const uint16_t* __restrict__ bias, int M,
                                                    int N, int K, int64_t ldx, int64_t ldw,
                                                    int64_t ldc) {
    __shared__ __attribute__((aligned(16))) float part[4][MC][16][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int l32 = lane & 31, h32 = lane >> 5;
    const int n0 = blockIdx.x * 32, m0 = blockIdx.y * 128;
    const int kw = K / 4;  // this wave's K range: [wave * kw, (wave + 1) * kw)
    const uint16_t* wp = W + (int64_t)min(n0 + l32, N - 1) * ldw + wave * kw + 8 * h32;
    const uint16_t* xp[MC];
#pragma unroll
    for (int mc = 0; mc < MC; ++mc)
        xp[mc] = X + (int64_t)min(m0 + 32 * mc + l32, M - 1) * ldx + wave * kw + 8 * h32;
    f32x16 acc[MC];
#pragma unroll
    for (int mc = 0; mc < MC; ++mc)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[mc][e] = 0.f;

    i32x4 wf[2][4], xf[2][MC][4];
    auto load = [&](int b, int k0) {
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
            wf[b][s2] = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(wp + k0 + 16 * s2));
#pragma unroll
            for (int mc = 0; mc < MC; ++mc)
                xf[b][mc][s2] = *reinterpret_cast<const i32x4*>(xp[mc] + k0 + 16 * s2);
        }
    };
    auto compute = [&](int b) {
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
            for (int mc = 0; mc < MC; ++mc)
                acc[mc] = mfma32x32x16<T>(wf[b][s2], xf[b][mc][s2], acc[mc]);
    };
    const int steps = kw / 64;  // host guarantees K % 256 == 0, steps >= 1
    load(0, 0);
    int st = 0;
    for (; st + 2 <= steps; st += 2) {
        load(1, (st + 1) * 64);
        compute(0);
        if (st + 2 < steps) load(0, (st + 2) * 64);
        compute(1);
    }
    if (st < steps) compute(0);

    // acc[mc][r] = C[m][n]: m = m0 + 32 mc + l32, n = n0 + 8 (r >> 2) + 4 h32 + (r & 3)
#pragma unroll
    for (int mc = 0; mc < MC; ++mc)
#pragma unroll
        for (int r = 0; r < 16; ++r) part[wave][mc][r][lane] = acc[mc][r];
    __syncthreads();
    for (int mc = wave; mc < MC; mc += 4) {
        const int m = m0 + 32 * mc + l32;
        if (m >= M) continue;
        uint16_t* crow = C + (int64_t)m * ldc;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int n = n0 + 8 * q + 4 * h32;
            if (n >= N) continue;
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 4 * q + r;
                v[r] = part[0][mc][i][lane] + part[1][mc][i][lane] + part[2][mc][i][lane] +
                       part[3][mc][i][lane];
                if constexpr (BIAS) v[r] += elem<T>::to_f32(T{bias[n + r]});
            }
            *reinterpret_cast<i32x2*>(crow + n) = i32x2{(int)pack2<T>(v[0], v[1]), (int)pack2<T>(v[2], v[3])};
        }
    }
}

template <typename T>
int launch_midm(const void* a, const void* b, void* c, const void* bias, int M, int N, int K,
                int64_t lda, int64_t ldb, int64_t ldc, hipStream_t s) {
    const dim3 grid(cdiv(N, 32), cdiv(M, 128)), block(256);
    const int mc = cdiv(min(M, 128), 32);
#define PLI_MIDM(MCC)                                                                          \
    do {                                                                                       \
        if (bias)                                                                              \
            hipLaunchKernelGGL((gemm_midm_nt<T, MCC, true>), grid, block, 0, s,                \
                               (const uint16_t*)a, (const uint16_t*)b, (uint16_t*)c,           \
                               (const uint16_t*)bias, M, N, K, lda, ldb, ldc);                 \
        else                                                                                   \
            hipLaunchKernelGGL((gemm_midm_nt<T, MCC, false>), grid, block, 0, s,               \
                               (const uint16_t*)a, (const uint16_t*)b, (uint16_t*)c,           \
                               (const uint16_t*)bias, M, N, K, lda, ldb, ldc);                 \
    } while (0)
    if (mc == 1) PLI_MIDM(1);
    else if (mc == 2) PLI_MIDM(2);
    else if (mc == 3) PLI_MIDM(3);
    else PLI_MIDM(4);
#undef PLI_MIDM
    return launch_status("gemm_midm_nt");
}

// ---------------------------------------------------------------------------
// Split-K mid-M NT path (caller workspace; pli_gemm_ws): workgroup = (128
// weight rows, one K slice, one 128-row slab of X).  Wave w streams weight
// rows n0 + 32 w .. +31 over the slice (non-temporal, exactly once) and all
// MC 32-row chunks of X; the four waves load the SAME X fragments, so X is
// fetched from L2 once per workgroup and shared through the CU's L1 -- a
// quarter of the X traffic of gemm_midm_nt, which is what bounds the M ~ 128
// shapes.  KS slices fill the chip (N/128 x KS ~ 256 workgroups); each slice
// writes an fp32 partial C tile (16-B stores) to ws[ks][m][n] and
// gemm_splitk_reduce sums them in fixed order (deterministic) into C (+ bias).
// KS == 1 writes C directly.
template <typename T, int MC, bool PARTIAL, bool BIAS>
__global__ __launch_bounds__(256) void gemm_splitk_nt(const uint16_t* __restrict__ X,
                                                      const uint16_t* __restrict__ W,
                                                      uint16_t* __restrict__ C,
                                                      float* __restrict__ ws,
                                                      const uint16_t* __restrict__ bias, int M,
                                                      int N, int K, int kslice, int64_t ldx,
                                                      int64_t ldw, int64_t ldc) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int l32 = lane & 31, h32 = lane >> 5;
    const int nw = blockIdx.x * 128 + wave * 32;  // this wave's first weight row
    const int ks = blockIdx.y, m0 = blockIdx.z * 128;
    const int kb = ks * kslice;
    const uint16_t* wp = W + (int64_t)min(nw + l32, N - 1) * ldw + kb + 8 * h32;
    const uint16_t* xp[MC];
#pragma unroll
    for (int mc = 0; mc < MC; ++mc)
        xp[mc] = X + (int64_t)min(m0 + 32 * mc + l32, M - 1) * ldx + kb + 8 * h32;
    f32x16 acc[MC];
#pragma unroll
    for (int mc = 0; mc < MC; ++mc)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[mc][e] = 0.f;

    i32x4 wf[2][4], xf[2][MC][4];
    auto load = [&](int b, int k0) {
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
            wf[b][s2] = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(wp + k0 + 16 * s2));
#pragma unroll
            for (int mc = 0; mc < MC; ++mc)
                xf[b][mc][s2] = *reinterpret_cast<const i32x4*>(xp[mc] + k0 + 16 * s2);
        }
    };
    auto compute = [&](int b) {
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
            for (int mc = 0; mc < MC; ++mc)
                acc[mc] = mfma32x32x16<T>(wf[b][s2], xf[b][mc][s2], acc[mc]);
    };
    const int steps = kslice / 64;  // host: kslice % 64 == 0, >= 64
    load(0, 0);
    int st = 0;
    for (; st + 2 <= steps; st += 2) {
        load(1, (st + 1) * 64);
        compute(0);
        if (st + 2 < steps) load(0, (st + 2) * 64);
        compute(1);
    }
    if (st < steps) compute(0);

    // acc[mc][4q + r] = C[m][n]: m = m0 + 32 mc + l32, n = nw + 8 q + 4 h32 + r
    if (nw >= N) return;
#pragma unroll
    for (int mc = 0; mc < MC; ++mc) {
        const int m = m0 + 32 * mc + l32;
        if (m >= M) continue;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int n = nw + 8 * q + 4 * h32;
            if constexpr (PARTIAL) {
                *reinterpret_cast<f32x4*>(ws + ((int64_t)ks * M + m) * N + n) =
                    f32x4{acc[mc][4 * q], acc[mc][4 * q + 1], acc[mc][4 * q + 2], acc[mc][4 * q + 3]};
            } else {
                float v[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v[r] = acc[mc][4 * q + r];
                    if constexpr (BIAS) v[r] += elem<T>::to_f32(T{bias[n + r]});
                }
                *reinterpret_cast<i32x2*>(C + (int64_t)m * ldc + n) =
                    i32x2{(int)pack2<T>(v[0], v[1]), (int)pack2<T>(v[2], v[3])};
            }
        }
    }
}

// C[m][n] = sum_ks ws[ks][m][n] (+ bias): 8 consecutive n per thread
template <typename T, bool BIAS>
__global__ __launch_bounds__(256) void gemm_splitk_reduce(const float* __restrict__ ws,
                                                          uint16_t* __restrict__ C,
                                                          const uint16_t* __restrict__ bias,
                                                          int M, int N, int KS, int64_t ldc) {
    const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
    const int64_t MN = (int64_t)M * N;
    if (i >= MN) return;
    const int m = (int)(i / N), n = (int)(i % N);
    float v[8];
    {
        const f32x4 a = *reinterpret_cast<const f32x4*>(ws + i);
        const f32x4 b = *reinterpret_cast<const f32x4*>(ws + i + 4);
#pragma unroll
        for (int r = 0; r < 4; ++r) { v[r] = a[r]; v[4 + r] = b[r]; }
    }
    for (int ks = 1; ks < KS; ++ks) {
        const f32x4 a = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(ws + ks * MN + i));
        const f32x4 b = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(ws + ks * MN + i + 4));
#pragma unroll
        for (int r = 0; r < 4; ++r) { v[r] += a[r]; v[4 + r] += b[r]; }
    }
    if constexpr (BIAS) {
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] += elem<T>::to_f32(T{bias[n + r]});
    }
    *reinterpret_cast<i32x4*>(C + (int64_t)m * ldc + n) =
        i32x4{(int)pack2<T>(v[0], v[1]), (int)pack2<T>(v[2], v[3]), (int)pack2<T>(v[4], v[5]),
              (int)pack2<T>(v[6], v[7])};
}

// LDS-staged form of gemm_splitk_nt (variant 25): each 64-k step of the
// workgroup's 128 weight rows and MC*32 X rows arrives by LDS-DMA as whole
// 128-B row segments (1 KiB = 8 rows per wave-instruction, chunk XOR-swizzled
// on the source address, g2_off_rows), double-buffered, and the MFMA
// fragments come back by ds_read_b128 -- the direct-load kernel touches 32
// half-lines per load instruction, which caps it far below HBM rate.
// W2 (SwiGLU, PARTIAL only): grid.y = 2 x the slices, slices y >= nks2 read
// the up weights W2 and write partial planes nks2 .. 2 nks2 - 1.
template <typename T, int MC, bool PARTIAL, bool BIAS, int NB = 2>
__global__ __launch_bounds__(256) void gemm_splitk_lds_nt(const uint16_t* __restrict__ X,
                                                          const uint16_t* __restrict__ W,
                                                          uint16_t* __restrict__ C,
                                                          float* __restrict__ ws,
                                                          const uint16_t* __restrict__ bias, int M,
                                                          int N, int K, int kslice, int64_t ldx,
                                                          int64_t ldw, int64_t ldc,
                                                          const uint16_t* __restrict__ W2 = nullptr,
                                                          int64_t ldw2 = 0, int nks2 = 0) {
    constexpr int WIMG = 128 * 128, XIMG = MC * 32 * 128, BUF = WIMG + XIMG;
    __shared__ __attribute__((aligned(1024))) char smem[NB * BUF];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int l32 = lane & 31, h32 = lane >> 5;
    const int n0 = blockIdx.x * 128, nw = n0 + wave * 32;
    const int ks = blockIdx.y, m0 = blockIdx.z * 128;  // ks = output plane
    const bool up = W2 != nullptr && ks >= nks2;
    if (up) {
        W = W2;
        ldw = ldw2;
    }
    const int kb = (up ? ks - nks2 : ks) * kslice;
    // DMA pieces of this wave: W rows 32 w + 8 i + (lane >> 3), i < 4; X rows
    // 8 j + (lane >> 3) for pieces j = w, w + 4, .. < 4 MC
    const int prow = lane >> 3, slot = lane & 7;
    const uint16_t* wsrc[4];
    int wdst[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = wave * 32 + 8 * i + prow;
        wsrc[i] = W + (int64_t)min(n0 + row, N - 1) * ldw + kb + 8 * (slot ^ ((row >> 1) & 7));
        wdst[i] = (wave * 4 + i) * 1024;
    }
    const uint16_t* xsrc[MC];
    int xdst[MC];
#pragma unroll
    for (int j = 0; j < MC; ++j) {
        const int piece = wave + 4 * j, row = 8 * piece + prow;
        xsrc[j] = X + (int64_t)min(m0 + row, M - 1) * ldx + kb + 8 * (slot ^ ((row >> 1) & 7));
        xdst[j] = WIMG + piece * 1024;
    }
    auto issue = [&](int buf, int k0) {
        char* base = smem + buf * BUF;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(wsrc[i] + k0),
                                             (__attribute__((address_space(3))) void*)(base + wdst[i]), 16, 0, 0);
#pragma unroll
        for (int j = 0; j < MC; ++j)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(xsrc[j] + k0),
                                             (__attribute__((address_space(3))) void*)(base + xdst[j]), 16, 0, 0);
    };
    f32x16 acc[MC];
#pragma unroll
    for (int mc = 0; mc < MC; ++mc)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[mc][e] = 0.f;

    const int steps = kslice / 64;
    auto mma_step = [&](const char* base) {
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
            const i32x4 wfr = lds_read_b128(base, g2_off_rows(wave * 32 + l32, 2 * s2 + h32));
#pragma unroll
            for (int mc = 0; mc < MC; ++mc) {
                const i32x4 xfr = lds_read_b128(base + WIMG, g2_off_rows(mc * 32 + l32, 2 * s2 + h32));
                acc[mc] = mfma32x32x16<T>(wfr, xfr, acc[mc]);
            }
        }
    };
    if constexpr (NB == 3) {
        // 3-deep ring, one barrier per step: wait for step st, barrier (every
        // wave is also done with step st-1, whose buffer the next issue refills),
        // issue step st+2, compute step st
        issue(0, 0);
        if (steps > 1) issue(1, 64);
        for (int st = 0; st < steps; ++st) {
            if (st + 1 < steps) {
                if constexpr (MC == 1) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
                else if constexpr (MC == 2) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
                else if constexpr (MC == 3) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __syncthreads();
            if (st + 2 < steps) issue((st + 2) % 3, (st + 2) * 64);
            mma_step(smem + (st % 3) * BUF);
        }
    } else {
    issue(0, 0);
    for (int st = 0; st < steps; ++st) {
        const int buf = st & 1;
        if (st + 1 < steps) {
            issue(buf ^ 1, (st + 1) * 64);
            if constexpr (MC == 1) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
            else if constexpr (MC == 2) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
            else if constexpr (MC == 3) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();  // every wave's pieces of step st have landed
        mma_step(smem + buf * BUF);
        __syncthreads();  // buffer buf is refilled by the DMA issued next step
    }
    }

    if (nw >= N) return;
#pragma unroll
    for (int mc = 0; mc < MC; ++mc) {
        const int m = m0 + 32 * mc + l32;
        if (m >= M) continue;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int n = nw + 8 * q + 4 * h32;
            if constexpr (PARTIAL) {
                *reinterpret_cast<f32x4*>(ws + ((int64_t)ks * M + m) * N + n) =
                    f32x4{acc[mc][4 * q], acc[mc][4 * q + 1], acc[mc][4 * q + 2], acc[mc][4 * q + 3]};
            } else {
                float v[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v[r] = acc[mc][4 * q + r];
                    if constexpr (BIAS) v[r] += elem<T>::to_f32(T{bias[n + r]});
                }
                *reinterpret_cast<i32x2*>(C + (int64_t)m * ldc + n) =
                    i32x2{(int)pack2<T>(v[0], v[1]), (int)pack2<T>(v[2], v[3])};
            }
        }
    }
}

// h[m][n] = silu(sum_s g_s) * (sum_s u_s) over the 2 x KS partial planes of
// the SwiGLU split-K launch (gate planes 0..KS-1, up planes KS..2KS-1)
template <typename T>
__global__ __launch_bounds__(256) void gemm_splitk_reduce_swiglu(const float* __restrict__ ws,
                                                                 uint16_t* __restrict__ H, int M,
                                                                 int N, int KS, int64_t ldh) {
    const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
    const int64_t MN = (int64_t)M * N;
    if (i >= MN) return;
    const int m = (int)(i / N), n = (int)(i % N);
    float g[8], u[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) g[r] = u[r] = 0.f;
    for (int ks = 0; ks < KS; ++ks) {
        const f32x4 g0 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(ws + ks * MN + i));
        const f32x4 g1 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(ws + ks * MN + i + 4));
        const f32x4 u0 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(ws + (KS + ks) * MN + i));
        const f32x4 u1 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(ws + (KS + ks) * MN + i + 4));
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            g[r] += g0[r]; g[4 + r] += g1[r];
            u[r] += u0[r]; u[4 + r] += u1[r];
        }
    }
    float v[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = silu_mul(g[r], u[r]);
    *reinterpret_cast<i32x4*>(H + (int64_t)m * ldh + n) =
        i32x4{(int)pack2<T>(v[0], v[1]), (int)pack2<T>(v[2], v[3]), (int)pack2<T>(v[4], v[5]),
              (int)pack2<T>(v[6], v[7])};
}

// Grouped (MoE) form of the LDS-staged kernel for decode-sized routing
// (rows_bound <= 1024): workgroup = (output tile, 128-row slab of expert e's
// rows, expert e).  Expert e's weights come from the device pointer table;
// its X rows through `gather` (per-lane LDS-DMA source rows); one K pass (the
// experts x tiles already fill the chip).  SW (W1/W3): the W image is 64 gate
// rows (waves 0-1) + the same 64 up rows (waves 2-3); the up waves hand their
// accumulators over through LDS and waves 0-1 write silu(g) * u, so neither
// activation reaches HBM.  Slabs past an expert's rows exit before any barrier.
template <typename T, int MC, bool SW>
__global__ __launch_bounds__(256) void gemm_grouped_lds_nt(
    const uint16_t* __restrict__ X, int64_t ldx, const int32_t* __restrict__ gather,
    const uint16_t* const* __restrict__ wtab, const uint16_t* const* __restrict__ wutab,
    int64_t ldw, uint16_t* __restrict__ C, int64_t ldc, const int32_t* __restrict__ offsets, int N,
    int K) {
    constexpr int WIMG = 128 * 128, XIMG = MC * 32 * 128, BUF = WIMG + XIMG;
    constexpr int TN = SW ? 64 : 128;  // output columns per workgroup
    __shared__ __attribute__((aligned(1024))) char smem[2 * BUF];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int l32 = lane & 31, h32 = lane >> 5;
    const int e = blockIdx.z;
    const int r0 = offsets[e] + blockIdx.y * 128, r1 = offsets[e + 1];
    if (r0 >= r1) return;  // uniform over the workgroup
    const int n0 = blockIdx.x * TN;
    const uint16_t* We = wtab[e];
    const uint16_t* Wue = SW ? wutab[e] : nullptr;
    const int prow = lane >> 3, slot = lane & 7;
    const uint16_t* wsrc[4];
    int wdst[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = wave * 32 + 8 * i + prow;  // W image row
        const uint16_t* base = We;
        int nr = n0 + row;
        if constexpr (SW) {
            if (row >= 64) { base = Wue; nr = n0 + row - 64; }
        }
        wsrc[i] = base + (int64_t)min(nr, N - 1) * ldw + 8 * (slot ^ ((row >> 1) & 7));
        wdst[i] = (wave * 4 + i) * 1024;
    }
    const uint16_t* xsrc[MC];
    int xdst[MC];
#pragma unroll
    for (int j = 0; j < MC; ++j) {
        const int piece = wave + 4 * j, row = 8 * piece + prow;
        const int r = min(r0 + row, r1 - 1);
        const int src = gather ? gather[r] : r;
        xsrc[j] = X + (int64_t)src * ldx + 8 * (slot ^ ((row >> 1) & 7));
        xdst[j] = WIMG + piece * 1024;
    }
    auto issue = [&](int buf, int k0) {
        char* b = smem + buf * BUF;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(wsrc[i] + k0),
                                             (__attribute__((address_space(3))) void*)(b + wdst[i]), 16, 0, 0);
#pragma unroll
        for (int j = 0; j < MC; ++j)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(xsrc[j] + k0),
                                             (__attribute__((address_space(3))) void*)(b + xdst[j]), 16, 0, 0);
    };
    f32x16 acc[MC];
#pragma unroll
    for (int mc = 0; mc < MC; ++mc)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[mc][q] = 0.f;
    const int steps = K / 64;
    issue(0, 0);
    for (int st = 0; st < steps; ++st) {
        const int buf = st & 1;
        if (st + 1 < steps) {
            issue(buf ^ 1, (st + 1) * 64);
            if constexpr (MC == 1) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
            else if constexpr (MC == 2) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
            else if constexpr (MC == 3) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        const char* b = smem + buf * BUF;
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
            const i32x4 wfr = lds_read_b128(b, g2_off_rows(wave * 32 + l32, 2 * s2 + h32));
#pragma unroll
            for (int mc = 0; mc < MC; ++mc) {
                const i32x4 xfr = lds_read_b128(b + WIMG, g2_off_rows(mc * 32 + l32, 2 * s2 + h32));
                acc[mc] = mfma32x32x16<T>(wfr, xfr, acc[mc]);
            }
        }
        __syncthreads();
    }
    // acc[mc][4q + r]: row r0 + 32 mc + l32, column (image row) 32 w' + 8 q + 4 h32 + r
    if constexpr (SW) {
        float* part = reinterpret_cast<float*>(smem);  // [2 waves][MC][16][64], after the last barrier
        if (wave >= 2) {
#pragma unroll
            for (int mc = 0; mc < MC; ++mc)
#pragma unroll
                for (int q = 0; q < 16; ++q) part[(((wave - 2) * MC + mc) * 16 + q) * 64 + lane] = acc[mc][q];
        }
        __syncthreads();
        if (wave >= 2) return;
    }
    const int nw = n0 + wave * 32;
    if (nw >= N) return;
#pragma unroll
    for (int mc = 0; mc < MC; ++mc) {
        const int m = r0 + 32 * mc + l32;
        if (m >= r1) continue;
        uint16_t* crow = C + (int64_t)m * ldc;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int n = nw + 8 * q + 4 * h32;
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                v[r] = acc[mc][4 * q + r];
                if constexpr (SW) {
                    const float* part = reinterpret_cast<const float*>(smem);
                    v[r] = silu_mul(v[r], part[((wave * MC + mc) * 16 + 4 * q + r) * 64 + lane]);
                }
            }
            *reinterpret_cast<i32x2*>(crow + n) = i32x2{(int)pack2<T>(v[0], v[1]), (int)pack2<T>(v[2], v[3])};
        }
    }
}

// K slices for the split-K mid-M path: the largest power of two with
// cdiv(N,128) * cdiv(M,128) * KS <= target workgroups, slices of >= 256 and a
// multiple of 64.  0: the path does not apply.
inline int splitk_slices(int M, int N, int K, int target, int max_m = 256) {
    if (M <= 16 || M > max_m || N % 32 != 0 || K % 64 != 0 || K < 64) return 0;
    const int64_t tiles = (int64_t)cdiv(N, 128) * cdiv(M, 128);
    int ks = 1;
    while (tiles * ks * 2 <= target && K % (ks * 2 * 64) == 0 && K / (ks * 2) >= 256) ks *= 2;
    return ks;
}

template <typename T>
int launch_splitk(const void* a, const void* b, void* c, const void* bias, int M, int N, int K,
                  int64_t lda, int64_t ldb, int64_t ldc, int ks, float* ws, hipStream_t s,
                  bool lds = false, bool nb3 = false, bool f32out = false) {
    const dim3 grid(cdiv(N, 128), ks, cdiv(M, 128)), block(256);
    const int mc = cdiv(min(M, 128), 32);
    const int kslice = K / ks;
#define PLI_SK(MCC, PA, BI)                                                                     \
    do {                                                                                        \
        if (lds && nb3)                                                                         \
            hipLaunchKernelGGL((gemm_splitk_lds_nt<T, MCC, PA, BI, 3>), grid, block, 0, s,        \
                               (const uint16_t*)a, (const uint16_t*)b, (uint16_t*)c, ws,        \
                               (const uint16_t*)bias, M, N, K, kslice, lda, ldb, ldc);          \
        else if (lds)                                                                           \
            hipLaunchKernelGGL((gemm_splitk_lds_nt<T, MCC, PA, BI>), grid, block, 0, s,           \
                               (const uint16_t*)a, (const uint16_t*)b, (uint16_t*)c, ws,        \
                               (const uint16_t*)bias, M, N, K, kslice, lda, ldb, ldc);          \
        else                                                                                    \
            hipLaunchKernelGGL((gemm_splitk_nt<T, MCC, PA, BI>), grid, block, 0, s,               \
                               (const uint16_t*)a, (const uint16_t*)b, (uint16_t*)c, ws,        \
                               (const uint16_t*)bias, M, N, K, kslice, lda, ldb, ldc);          \
    } while (0)
#define PLI_SK_MC(PA, BI)                   \
    do {                                    \
        if (mc == 1) PLI_SK(1, PA, BI);     \
        else if (mc == 2) PLI_SK(2, PA, BI); \
        else if (mc == 3) PLI_SK(3, PA, BI); \
        else PLI_SK(4, PA, BI);             \
    } while (0)
    if (f32out) {  // one slice, the fp32 plane is the product (pli_gemm_f32out)
        PLI_SK_MC(true, false);
        return launch_status("gemm_splitk_lds_nt");
    }
    const char* name = lds ? "gemm_splitk_lds_nt" : "gemm_splitk_nt";
    if (ks > 1) {
        PLI_SK_MC(true, false);
        const int rc = launch_status(name);
        if (rc) return rc;
        const int64_t groups = ((int64_t)M * N) / 8;
        const dim3 rgrid((unsigned)cdiv((int)((groups + 255) / 256 * 256), 256));
        if (bias)
            hipLaunchKernelGGL((gemm_splitk_reduce<T, true>), rgrid, dim3(256), 0, s, ws, (uint16_t*)c,
                               (const uint16_t*)bias, M, N, ks, ldc);
        else
            hipLaunchKernelGGL((gemm_splitk_reduce<T, false>), rgrid, dim3(256), 0, s, ws, (uint16_t*)c,
                               (const uint16_t*)bias, M, N, ks, ldc);
        return launch_status("gemm_splitk_reduce");
    }
    if (bias) PLI_SK_MC(false, true);
    else PLI_SK_MC(false, false);
#undef PLI_SK_MC
#undef PLI_SK
    return launch_status(name);
}

template <typename T>
int launch_splitk_swiglu(const void* x, const void* wg, const void* wu, void* h, int M, int N,
                         int K, int64_t ldx, int64_t ldwg, int64_t ldwu, int64_t ldh, int ks,
                         float* ws, hipStream_t s) {
    const dim3 grid(cdiv(N, 128), 2 * ks, cdiv(M, 128)), block(256);
    const int mc = cdiv(min(M, 128), 32);
    const int kslice = K / ks;
#define PLI_SKS(MCC)                                                                              \
    hipLaunchKernelGGL((gemm_splitk_lds_nt<T, MCC, true, false>), grid, block, 0, s,               \
                       (const uint16_t*)x, (const uint16_t*)wg, (uint16_t*)h, ws, nullptr, M, N, K, \
                       kslice, ldx, ldwg, ldh, (const uint16_t*)wu, ldwu, ks)
    if (mc == 1) PLI_SKS(1);
    else if (mc == 2) PLI_SKS(2);
    else if (mc == 3) PLI_SKS(3);
    else PLI_SKS(4);
#undef PLI_SKS
    const int rc = launch_status("gemm_splitk_nt<swiglu>");
    if (rc) return rc;
    const int64_t groups = ((int64_t)M * N) / 8;
    hipLaunchKernelGGL((gemm_splitk_reduce_swiglu<T>), dim3((unsigned)((groups + 255) / 256)),
                       dim3(256), 0, s, ws, (uint16_t*)h, M, N, ks, ldh);
    return launch_status("gemm_splitk_reduce_swiglu");
}

template <typename T>
int launch_mfma(const void* a, const void* b, void* c, const void* bias, int M, int N, int K,
                int64_t lda, int64_t ldb, int64_t ldc, int trans_b, hipStream_t s) {
    const int tm = cdiv(M, BM), tn = cdiv(N, BN);
    const int64_t nb = (int64_t)tm * tn;
    PLI_REQUIRE(nb < (1ll << 31), "pli_gemm: grid too large");
    const dim3 grid((unsigned)nb), block(256);
#define PLI_GEMM_LAUNCH(TB, BI)                                                               \
    hipLaunchKernelGGL((gemm_mfma<T, TB, BI>), grid, block, 0, s, (const uint16_t*)a,          \
                       (const uint16_t*)b, (uint16_t*)c, (const uint16_t*)bias, M, N, K, lda, \
                       ldb, ldc, tn, (int)nb)
    if (trans_b) {
        if (bias) PLI_GEMM_LAUNCH(true, true); else PLI_GEMM_LAUNCH(true, false);
    } else {
        if (bias) PLI_GEMM_LAUNCH(false, true); else PLI_GEMM_LAUNCH(false, false);
    }
#undef PLI_GEMM_LAUNCH
    return launch_status("gemm_mfma");
}

template <typename T, bool TB, bool BI>
void launch_256p(int sched, dim3 grid, dim3 block, hipStream_t s, const void* a, const void* b,
                 void* c, const void* bias, int M, int N, int K, int64_t lda, int64_t ldb,
                 int64_t ldc, int tn, int nb, int group_m) {
#define PLI_G256P(SC)                                                                           \
    hipLaunchKernelGGL((gemm_256p<T, TB, BI, SC>), grid, block, 0, s, (const uint16_t*)a,       \
                       (const uint16_t*)b, (uint16_t*)c, (const uint16_t*)bias, M, N, K, lda, ldb, \
                       ldc, tn, nb, group_m, nullptr, 0)
    switch (sched) {
        case 1: PLI_G256P(1); break;
        case 3: PLI_G256P(3); break;
        case 5: PLI_G256P(5); break;
        case 7: PLI_G256P(7); break;
        default: PLI_G256P(0);
    }
#undef PLI_G256P
}

template <typename T>
int launch_256(const void* a, const void* b, void* c, const void* bias, int M, int N, int K,
               int64_t lda, int64_t ldb, int64_t ldc, int trans_b, hipStream_t s, int phased,
               bool prio = false, int group_m = 0) {
    // phased: -1 = gemm_256 (one phase per K-tile), else gemm_256p's SCHED bits
    const int tm = cdiv(M, G2M), tn = cdiv(N, G2N);
    const int64_t nb = (int64_t)tm * tn;
    PLI_REQUIRE(nb < (1ll << 31), "pli_gemm: grid too large");
    const dim3 grid((unsigned)nb), block(512);
#define PLI_G256(TB, BI)                                                                          \
    do {                                                                                          \
        if (phased >= 0)                                                                          \
            launch_256p<T, TB, BI>(phased, grid, block, s, a, b, c, bias, M, N, K, lda, ldb, ldc, \
                                   tn, (int)nb, group_m);                                         \
        else if (prio)                                                                            \
            hipLaunchKernelGGL((gemm_256<T, TB, BI, true>), grid, block, 0, s, (const uint16_t*)a, \
                               (const uint16_t*)b, (uint16_t*)c, (const uint16_t*)bias, M, N, K,  \
                               lda, ldb, ldc, tn, (int)nb, group_m);                              \
        else                                                                                      \
            hipLaunchKernelGGL((gemm_256<T, TB, BI>), grid, block, 0, s, (const uint16_t*)a,      \
                               (const uint16_t*)b, (uint16_t*)c, (const uint16_t*)bias, M, N, K,  \
                               lda, ldb, ldc, tn, (int)nb, group_m);                              \
    } while (0)
    if (trans_b) {
        if (bias) PLI_G256(true, true); else PLI_G256(true, false);
    } else {
        if (bias) PLI_G256(false, true); else PLI_G256(false, false);
    }
#undef PLI_G256
    return launch_status("gemm_256");
}

template <typename T>
int launch_generic(const void* a, const void* b, void* c, const void* bias, int M, int N, int K,
                   int64_t lda, int64_t ldb, int64_t ldc, int trans_b, hipStream_t s) {
    const dim3 grid(cdiv(N, GT), cdiv(M, GT)), block(256);
    if (trans_b)
        hipLaunchKernelGGL((gemm_generic<T, true>), grid, block, 0, s, (const T*)a, (const T*)b,
                           (T*)c, (const T*)bias, M, N, K, lda, ldb, ldc);
    else
        hipLaunchKernelGGL((gemm_generic<T, false>), grid, block, 0, s, (const T*)a, (const T*)b,
                           (T*)c, (const T*)bias, M, N, K, lda, ldb, ldc);
    return launch_status("gemm_generic");
}

inline bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// ---- fused SwiGLU launches: h = silu(x Wg^T) * (x Wu^T)
template <typename T>
int launch_swiglu(const void* x, const void* wg, const void* wu, void* h, int M, int N, int K,
                  int64_t ldx, int64_t ldwg, int64_t ldwu, int64_t ldh, bool vec, hipStream_t s,
                  int variant = 0) {
    const auto* X = (const uint16_t*)x;
    const auto* G = (const uint16_t*)wg;
    const auto* U = (const uint16_t*)wu;
    auto* Hh = (uint16_t*)h;
    if constexpr (!std::is_same_v<T, float>) {
    if (vec && (M == 1 || (M <= 16 && !(K % 128 == 0 && N % 16 == 0)))) {
        const dim3 grid(cdiv(N, 2)), block(128);
#define PLI_SKINNY_SW(NB)                                                                         \
    hipLaunchKernelGGL((gemm_skinny_nt<T, NB, 4, true>), grid, block, 0, s, X, G, Hh, nullptr, M, \
                       N, K / 8, ldx, ldwg, ldh, U, ldwu)
        if (M <= 1) PLI_SKINNY_SW(1);
        else if (M <= 2) PLI_SKINNY_SW(2);
        else if (M <= 4) PLI_SKINNY_SW(4);
        else if (M <= 8) PLI_SKINNY_SW(8);
        else PLI_SKINNY_SW(16);
#undef PLI_SKINNY_SW
        return launch_status("gemm_skinny_nt<swiglu>");
    }
    if (vec && M <= 128 && K % 128 == 0 && N % 16 == 0) {
        const dim3 grid(cdiv(N, 16)), block(256);
#define PLI_SMALLM_SW(NBG)                                                                        \
    hipLaunchKernelGGL((gemm_smallm_nt<T, NBG, false, true>), grid, block, 0, s, X, G, Hh,       \
                       nullptr, M, N, K, ldx, ldwg, ldh, U, ldwu)
        if (M <= 16) PLI_SMALLM_SW(1);
        else if (M <= 32) PLI_SMALLM_SW(2);
        else if (M <= 64) PLI_SMALLM_SW(4);
        else PLI_SMALLM_SW(8);
#undef PLI_SMALLM_SW
        return launch_status("gemm_smallm_nt<swiglu>");
    }
    // gemm_w5's SwiGLU form (one wave per SIMD, K 64 deep), the prefill
    // default since round 4: bitwise the phased tile's output and faster on
    // every measured shape (4096 x 14336 x 4096 1371 vs 1303 TF/s, 16384 x
    // 14336 x 4096 1359 vs 1309, 4096 x 1792 x 4096 1305 vs 1185, 2048 x 5632
    // x 2048 940 vs 922; profiles/r04/swiglu_w5.log).  Variant 3 forces it
    // (ragged M / N are masked in its epilogue), 4 forces the phased tile.
    if (vec && variant != 4 && (variant == 3 || (M >= G2M && N >= 256)) && K % 64 == 0 &&
        (variant == 3 || (int64_t)cdiv(M, G2M) * cdiv(N, 128) >= 96) && ldx * 2 * 256 < (1ll << 31) &&
        ldwg * 2 * 128 < (1ll << 31) && ldwu * 2 * 128 < (1ll << 31))
        return launch_gemm_w5_swiglu(x, wg, wu, h, M, N, K, ldx, ldwg, ldwu, ldh, std::is_same_v<T, bf16_t>, s);
    if (vec && M >= G2M && N >= 256 && K % G2K == 0 && (int64_t)cdiv(M, G2M) * cdiv(N, 128) >= 96) {
        // prefill sizes: the phased 256 x 128 tile (staggered schedule, grouped rasterization)
        const int tm = cdiv(M, G2M), tn = cdiv(N, 128);
        const int64_t nb = (int64_t)tm * tn;
        PLI_REQUIRE(nb < (1ll << 31), "pli_gemm_swiglu: grid too large");
        hipLaunchKernelGGL((gemm_256p<T, true, false, 7, true>), dim3((unsigned)nb), dim3(512), 0, s,
                           X, G, Hh, nullptr, M, N, K, ldx, ldwg, ldh, tn, (int)nb, 4, U, ldwu);
        return launch_status("gemm_256p<swiglu>");
    }
    if (vec) {
        const int tm = cdiv(M, BM), tn = cdiv(N, BN / 2);
        const int64_t nb = (int64_t)tm * tn;
        PLI_REQUIRE(nb < (1ll << 31), "pli_gemm_swiglu: grid too large");
        hipLaunchKernelGGL((gemm_mfma<T, true, false, true>), dim3((unsigned)nb), dim3(256), 0, s,
                           X, G, Hh, nullptr, M, N, K, ldx, ldwg, ldh, tn, (int)nb, U, ldwu);
        return launch_status("gemm_mfma<swiglu>");
    }
    }  // 16-bit paths
    const dim3 grid(cdiv(N, GT / 2), cdiv(M, GT)), block(256);
    hipLaunchKernelGGL((gemm_generic<T, true, true>), grid, block, 0, s, (const T*)x, (const T*)wg,
                       (T*)h, nullptr, M, N, K, ldx, ldwg, ldh, (const T*)wu, ldwu);
    return launch_status("gemm_generic<swiglu>");
}

}  // namespace
}  // namespace pli

static int swiglu_dispatch(const void* x, const void* wg, const void* wu, void* h, int m, int n,
                           int k, int64_t ldx, int64_t ldwg, int64_t ldwu, int64_t ldh, int dtype,
                           void* stream, void* ws, size_t ws_bytes, int variant = 0);

// split-K slices of the SwiGLU decode-batch route (0: not taken); force:
// ignore the short-K rule (A/B)
static int swiglu_slices(int m, int n, int k, bool force = false) {
    if (m <= 16 || m > 256) return 0;
    if (force) return pli::splitk_slices(m, n, k, 512);
    // short K splits too here (unlike the plain GEMM): gate + up are twice
    // the weights per output (32 / 64 / 128 x 5632 x 2048: 18.1 / 21.1 / 32.5
    // vs 20.9 / 27.9 / 45.7 us unsplit, tools/tune.py swr)
    // the phased 256 x 128 SwiGLU tile has enough tiles here (M 256 x 14336:
    // 104.5 vs 126 us split)
    if (m >= 256 && (int64_t)pli::cdiv(m, 256) * pli::cdiv(n, 128) >= 96) return 0;
    return pli::splitk_slices(m, n, k, 512);
}

extern "C" size_t pli_gemm_swiglu_workspace_size(int m, int n, int k, int dtype) {
    if ((dtype != PLI_BF16 && dtype != PLI_F16) || m <= 0 || n <= 0 || k <= 0) return 0;
    const int ks = swiglu_slices(m, n, k, true);  // the most any route or variant uses
    return ks > 0 ? (size_t)2 * ks * m * n * sizeof(float) : 0;
}

extern "C" int pli_gemm_swiglu(const void* x, const void* wg, const void* wu, void* h, int m,
                               int n, int k, int64_t ldx, int64_t ldwg, int64_t ldwu, int64_t ldh,
                               int dtype, void* stream) {
    return swiglu_dispatch(x, wg, wu, h, m, n, k, ldx, ldwg, ldwu, ldh, dtype, stream, nullptr, 0);
}

extern "C" int pli_gemm_swiglu_ws(const void* x, const void* wg, const void* wu, void* h, int m,
                                  int n, int k, int64_t ldx, int64_t ldwg, int64_t ldwu,
                                  int64_t ldh, int dtype, void* workspace, size_t workspace_bytes,
                                  void* stream) {
    return swiglu_dispatch(x, wg, wu, h, m, n, k, ldx, ldwg, ldwu, ldh, dtype, stream, workspace,
                           workspace_bytes);
}

// variant 1 = split K wherever the split-K route applies, 2 = never split
// (A/B of the decode-batch routing), 3 = gemm_w5's SwiGLU tile, 4 = the
// phased 256 x 128 tile (3 and 4 never split)
extern "C" int pli_gemm_swiglu_ws_variant(const void* x, const void* wg, const void* wu, void* h,
                                          int m, int n, int k, int64_t ldx, int64_t ldwg,
                                          int64_t ldwu, int64_t ldh, int dtype, void* workspace,
                                          size_t workspace_bytes, void* stream, int variant) {
    return swiglu_dispatch(x, wg, wu, h, m, n, k, ldx, ldwg, ldwu, ldh, dtype, stream, workspace,
                           workspace_bytes, variant);
}

static int swiglu_dispatch(const void* x, const void* wg, const void* wu, void* h, int m, int n,
                           int k, int64_t ldx, int64_t ldwg, int64_t ldwu, int64_t ldh, int dtype,
                           void* stream, void* ws, size_t ws_bytes, int variant) {
    using namespace pli;
    clear_error();
    PLI_REQUIRE(m >= 0 && n >= 0 && k >= 0, "pli_gemm_swiglu: bad shape m=%d n=%d k=%d", m, n, k);
    PLI_REQUIRE(dtype == PLI_F32 || dtype == PLI_F16 || dtype == PLI_BF16,
                "pli_gemm_swiglu: bad dtype %d", dtype);
    if (m == 0 || n == 0) return PLI_OK;  // (empty operands may be NULL, pli.h)
    PLI_REQUIRE(h && (k == 0 || (x && wg && wu)), "pli_gemm_swiglu: null pointer");
    PLI_REQUIRE(ldx >= k && ldwg >= k && ldwu >= k && ldh >= n,
                "pli_gemm_swiglu: leading dimension too small (ldx=%lld ldwg=%lld ldwu=%lld ldh=%lld)",
                (long long)ldx, (long long)ldwg, (long long)ldwu, (long long)ldh);
    hipStream_t s = (hipStream_t)stream;
    const bool vec = (dtype == PLI_BF16 || dtype == PLI_F16) && k > 0 && k % 8 == 0 &&
                     n % 8 == 0 && ldx % 8 == 0 && ldwg % 8 == 0 && ldwu % 8 == 0 && ldh % 8 == 0 &&
                     al16(x) && al16(wg) && al16(wu) && al16(h);
    // decode batches (16 < m <= 256, K > 2048 or m > 128) with a workspace:
    // gate and up split-K planes in one LDS-staged launch, silu(g) * u in the
    // fixed-order reduce (profiles/r01/gemm/tune_swiglu_splitk.log)
    // (variants 2, 3 and 4 name a one-launch tile: never split)
    const int ks = vec && variant != 2 && variant != 3 && variant != 4 ? swiglu_slices(m, n, k, variant == 1) : 0;
    if (ks > 0 && ws != nullptr && ws_bytes >= (size_t)2 * ks * m * n * sizeof(float)) {
        PLI_REQUIRE(((uintptr_t)ws & 15) == 0, "pli_gemm_swiglu_ws: workspace must be 16-byte aligned");
        if (dtype == PLI_BF16)
            return launch_splitk_swiglu<bf16_t>(x, wg, wu, h, m, n, k, ldx, ldwg, ldwu, ldh, ks, (float*)ws, s);
        return launch_splitk_swiglu<f16_t>(x, wg, wu, h, m, n, k, ldx, ldwg, ldwu, ldh, ks, (float*)ws, s);
    }
    switch (dtype) {
        case PLI_BF16: return launch_swiglu<bf16_t>(x, wg, wu, h, m, n, k, ldx, ldwg, ldwu, ldh, vec, s, variant);
        case PLI_F16: return launch_swiglu<f16_t>(x, wg, wu, h, m, n, k, ldx, ldwg, ldwu, ldh, vec, s, variant);
        default: return launch_swiglu<float>(x, wg, wu, h, m, n, k, ldx, ldwg, ldwu, ldh, false, s);
    }
}

// variant: 0 = default routing (large shapes: phased 256x256 tile, staggered
// two-barrier schedule, grouped rasterization), 1 = force the 128x128 MFMA
// tile, 2 = force the one-phase 256x256 LDS-DMA tile, 3 = the phased tile
// with one barrier per phase, 4 = the one-phase tile with s_setprio(1) around
// its MFMA clusters, 5-8 = phased SCHED 1/3/5/7, 9-11 = one-phase with
// group_m 4/8/16, 12-15 = phased SCHED 7 with group_m 8/4/2/16 (where their
// shape conditions hold)
namespace pli {
namespace {
// split-K target workgroups by variant (0: default 256; 22: 512; 24: 128)
inline int splitk_target(int variant) {
    return (variant == 0 || variant == 22 || variant == 26 || variant == 28) ? 512
           : (variant == 24 || variant == 27 || variant == 29) ? 128
                                                          : 256;
}
inline bool splitk_variant(int v) { return v == 0 || v == 22 || v == 24 || (v >= 25 && v <= 29); }
}  // namespace
}  // namespace pli

extern "C" size_t pli_gemm_workspace_size(int m, int n, int k, int trans_b, int dtype) {
    using namespace pli;
    if (!trans_b || (dtype != PLI_BF16 && dtype != PLI_F16) || m <= 0 || n <= 0 || k <= 0) return 0;
    const int ks = splitk_slices(m, n, k, splitk_target(22), 2048);  // the largest any variant uses
    return ks > 1 ? (size_t)ks * m * n * sizeof(float) : 0;
}

static int gemm_dispatch(const void* a, const void* b, void* c, const void* bias, int m, int n,
                         int k, int64_t lda, int64_t ldb, int64_t ldc, int trans_b, int dtype,
                         void* stream, int variant, void* ws, size_t ws_bytes);

extern "C" int pli_gemm_variant(const void* a, const void* b, void* c, const void* bias, int m,
                                int n, int k, int64_t lda, int64_t ldb, int64_t ldc, int trans_b,
                                int dtype, void* stream, int variant) {
    return gemm_dispatch(a, b, c, bias, m, n, k, lda, ldb, ldc, trans_b, dtype, stream, variant,
                         nullptr, 0);
}

extern "C" int pli_gemm_ws(const void* a, const void* b, void* c, const void* bias, int m, int n,
                           int k, int64_t lda, int64_t ldb, int64_t ldc, int trans_b, int dtype,
                           void* workspace, size_t workspace_bytes, void* stream) {
    return gemm_dispatch(a, b, c, bias, m, n, k, lda, ldb, ldc, trans_b, dtype, stream, 0,
                         workspace, workspace_bytes);
}

extern "C" int pli_gemm_ws_variant(const void* a, const void* b, void* c, const void* bias, int m,
                                   int n, int k, int64_t lda, int64_t ldb, int64_t ldc, int trans_b,
                                   int dtype, void* workspace, size_t workspace_bytes, void* stream,
                                   int variant) {
    return gemm_dispatch(a, b, c, bias, m, n, k, lda, ldb, ldc, trans_b, dtype, stream, variant,
                         workspace, workspace_bytes);
}

static int gemm_dispatch(const void* a, const void* b, void* c, const void* bias, int m, int n,
                         int k, int64_t lda, int64_t ldb, int64_t ldc, int trans_b, int dtype,
                         void* stream, int variant, void* ws, size_t ws_bytes) {
    using namespace pli;
    clear_error();
    PLI_REQUIRE(m >= 0 && n >= 0 && k >= 0, "pli_gemm: bad shape m=%d n=%d k=%d", m, n, k);
    // empty operands may be NULL (pli.h): no output -> nothing to do; K == 0
    // -> C = bias (or 0), A and B not read
    if (m == 0 || n == 0) return PLI_OK;
    PLI_REQUIRE(c && (k == 0 || (a && b)), "pli_gemm: null pointer");
    PLI_REQUIRE(lda >= k && ldc >= n && ldb >= (trans_b ? k : n),
                "pli_gemm: leading dimension too small (lda=%lld ldb=%lld ldc=%lld)",
                (long long)lda, (long long)ldb, (long long)ldc);
    hipStream_t s = (hipStream_t)stream;
    if (k == 0) {  // C = bias (or 0): the generic kernel handles K == 0
        switch (dtype) {
            case PLI_F32: return launch_generic<float>(a, b, c, bias, m, n, k, lda, ldb, ldc, trans_b, s);
            case PLI_F16: return launch_generic<f16_t>(a, b, c, bias, m, n, k, lda, ldb, ldc, trans_b, s);
            case PLI_BF16: return launch_generic<bf16_t>(a, b, c, bias, m, n, k, lda, ldb, ldc, trans_b, s);
            default: set_error("pli_gemm: bad dtype %d", dtype); return PLI_EINVAL;
        }
    }
    const bool vec = (dtype == PLI_BF16 || dtype == PLI_F16) && k % 8 == 0 && n % 8 == 0 &&
                     lda % 8 == 0 && ldb % 8 == 0 && ldc % 8 == 0 && al16(a) && al16(b) &&
                     al16(c) && (bias == nullptr || ((uintptr_t)bias & 7) == 0);
    // decode batches: W streamed once.  M == 1: GEMV-style VALU kernel;
    // M <= 128 (K a multiple of 128, N of 16): small-M MFMA kernel.
    if (vec && trans_b && m == 1) {
        // no bias: y = W x is pli_gemv (same per-row chunk and FMA order as the
        // skinny kernel, so bitwise the same; 8192^2 5.85 vs 5.18 TB/s, 4096^2
        // 4.48 vs 3.98, tools/gemv_vs_skinny.py, profiles/r01/gemm/)
        if (bias == nullptr) return pli_gemv(b, a, c, n, k, ldb, dtype, stream);
        if (dtype == PLI_BF16)
            return launch_skinny<bf16_t>(a, b, c, bias, m, n, k, lda, ldb, ldc, s);
        return launch_skinny<f16_t>(a, b, c, bias, m, n, k, lda, ldb, ldc, s);
    }
    // Decode-batch / TP-shard NT shapes, 16 < M <= 256 (tools/tune.py midm,
    // profiles/r01/gemm/tune_midm.log).  With a workspace: the LDS-staged
    // split-K kernel (~ hipBLASLt at M 17-256 for K >= 4096: M 128 x 8192^2
    // 38.6 us vs 146 on the small-M kernel); short K (<= 2048) at M <= 128 is
    // better served without splitting: the mid-M kernel for M > 32 (also the
    // no-workspace route), the small-M kernel below that.
    // A/B: 22/24 direct-load split-K (512/128 target workgroups), 25/26/27
    // LDS split-K (256/512/128), 20 mid-M, 21 small-M.
    // Few-tile NT shapes above that (256 < M <= 2048, fewer than 128 tiles of
    // 256^2) take the same split-K kernel with 128-row slabs: 512 x 4096 x
    // 4096 220 -> 476 TF, 1024 x 4096^2 417 -> 645, 2048^3 400 -> 469
    // (hipBLASLt 571 / 897 / 716).
    // short K keeps the unsplit kernels only where they win: a wide N (the TP-8
    // row shard 8192 x 1024: mid-M 14.1 vs split 16.5-19 us at M 128) below
    // 16384 columns (an lm_head 32 x 32000 x 2048: split 26 vs 56 us), or
    // M <= 32 with few columns (32 x 2048 x 2048: small-M 8.3 vs 11.3 us);
    // M 33-128 with few columns splits (64 x 2048 x 2048: 11.8 vs 16.7 us)
    const bool short_k = k <= 2048 && m <= 128 && n < 16384 && (m <= 32 || n / 128 >= 64);
    const bool few_tiles = m > 256 && m <= 2048 && (int64_t)cdiv(m, G2M) * cdiv(n, G2N) < 128;
    if (vec && trans_b && splitk_variant(variant) && ws != nullptr && !(variant == 0 && short_k) &&
        (variant != 0 || m <= 256 || few_tiles)) {
        const int target = (variant == 0 && m > 256 && k < 4096) ? 128 : splitk_target(variant);
        const int ks = splitk_slices(m, n, k, target, (variant == 0 || variant >= 25) ? 2048 : 256);
        if (ks >= 1 && (ks == 1 || ws_bytes >= (size_t)ks * m * n * sizeof(float))) {
            PLI_REQUIRE(((uintptr_t)ws & 15) == 0, "pli_gemm_ws: workspace must be 16-byte aligned");
            const bool lds = variant == 0 || variant >= 25;
            const bool nb3 = variant == 28 || variant == 29;
            if (dtype == PLI_BF16)
                return launch_splitk<bf16_t>(a, b, c, bias, m, n, k, lda, ldb, ldc, ks, (float*)ws, s, lds, nb3);
            return launch_splitk<f16_t>(a, b, c, bias, m, n, k, lda, ldb, ldc, ks, (float*)ws, s, lds, nb3);
        }
    }
    if (vec && trans_b && k % 256 == 0 &&
        ((variant == 20 && m <= 256) || (variant == 0 && m > 32 && m <= 128))) {
        if (dtype == PLI_BF16)
            return launch_midm<bf16_t>(a, b, c, bias, m, n, k, lda, ldb, ldc, s);
        return launch_midm<f16_t>(a, b, c, bias, m, n, k, lda, ldb, ldc, s);
    }
    if (vec && trans_b && m <= 128 && k % 128 == 0 && n % 16 == 0) {
        if (dtype == PLI_BF16)
            return launch_smallm<bf16_t>(a, b, c, bias, m, n, k, lda, ldb, ldc, s);
        return launch_smallm<f16_t>(a, b, c, bias, m, n, k, lda, ldb, ldc, s);
    }
    if (vec && trans_b && m <= 16) {
        if (dtype == PLI_BF16)
            return launch_skinny<bf16_t>(a, b, c, bias, m, n, k, lda, ldb, ldc, s);
        return launch_skinny<f16_t>(a, b, c, bias, m, n, k, lda, ldb, ldc, s);
    }
    // large problems: 256x256 LDS-DMA tile (K a multiple of 64; at least a 2x2
    // grid of tiles so the block count is not tiny)
    // (fewer than 128 tiles of 256^2 leave CUs idle: the 128^2 tile's 4x grid
    // wins there, +20-60 % at 16-64 tiles, profiles/r01/gemm/tune_few_tiles.log)
    // variant 40: gemm_w4v (gemm_w4v.hip), one wave per SIMD, 128x128 per wave
    if (variant == 40 && vec && gemm_w4v_ok(m, n, k, lda, ldb, ldc, trans_b))
        return launch_gemm_w4v(a, b, c, bias, m, n, k, lda, ldb, ldc, trans_b, dtype == PLI_BF16, s, 4);
    // variant 41: gemm_w5 (gemm_w5.hip), the same tile with K staged 64 deep
    if (variant == 41 && vec && gemm_w5_ok(m, n, k, lda, ldb, ldc, trans_b))
        return launch_gemm_w5(a, b, c, bias, m, n, k, lda, ldb, ldc, trans_b, dtype == PLI_BF16, s, 4);
    // variant 43: gemm_w5 persistent (M, N multiples of 256)
    if (variant == 43 && vec && m % 256 == 0 && n % 256 == 0 && gemm_w5_ok(m, n, k, lda, ldb, ldc, trans_b))
        return launch_gemm_w5(a, b, c, bias, m, n, k, lda, ldb, ldc, trans_b, dtype == PLI_BF16, s, 4, true);
    const bool big = vec && k % G2K == 0 && m >= 2 * G2M && n >= 2 * G2N && variant != 1 &&
                     (variant != 0 || (int64_t)cdiv(m, G2M) * cdiv(n, G2N) >= 128);
    // default for the large shapes since round 3: gemm_w5 (one wave per SIMD,
    // K staged 64 deep), +10-25 % over the round-2 phased 8-wave tile (variant
    // 13) and at or past hipBLASLt on most shapes (same process, NT / NN TF/s:
    // 4096^3 1422 / 1378 vs 1206 / 1175, torch 1400 / 1281; 8192^3 1536 / 1488
    // vs 1344 / 1305, torch 1560 / 1391; profiles/r03/gemm/ab_w5.log).
    // gemm_w4v (variant 40, K 32 deep) sits between them.
    // Its persistent walk (variant 43, K stream continued across tiles) where
    // M, N are multiples of 256 and K >= 128: the per-tile prologue is a
    // larger share at short K (8192^2 x 1024 NT / NN 1260 / 1188 vs 1180 /
    // 1114, 16384 x 8192 x 1024 1320 / 1245 vs 1187 / 1163, hipBLASLt 1237 /
    // 1083 and 1284 / 1109; profiles/r03/gemm/ab_w5_persistent.log); with the
    // split DMA schedule it is also level or ahead at K = 8192 / 16384 (NN
    // 8192^3 1508 vs 1491, 8192^2 x 16384 NT / NN 1520 / 1505 vs 1508 / 1490;
    // profiles/r04/gemm/ab_w5_persistent_deepK.log)
    if (variant == 0 && big && gemm_w5_ok(m, n, k, lda, ldb, ldc, trans_b)) {
        const bool persist = m % 256 == 0 && n % 256 == 0 && k >= 128;
        return launch_gemm_w5(a, b, c, bias, m, n, k, lda, ldb, ldc, trans_b, dtype == PLI_BF16, s, 4, persist);
    }
    if (big || (vec && variant >= 2 && k % G2K == 0 && n >= 8)) {
        // variant 3: phased (SCHED 0); 5-8: phased with SCHED 1, 3, 5, 7;
        // 9-11: one-phase tile with grouped rasterization (group_m 4, 8, 16);
        // 12-15: phased SCHED 7 with group_m 8, 4, 2, 16
        // default (0): phased SCHED 7 with group_m 4 (= variant 13; NT 8192^3
        // 1371-1414 vs 1145-1185 TF for the ungrouped one-phase tile, NN 4096^3
        // 1104 vs 935), except NT with K <= 4096 (below)
        int phased = variant == 3 ? 0 : (variant >= 5 && variant <= 8) ? 2 * (variant - 5) + 1 : -1;
        int group_m = 0;
        if (variant == 0) {
            // NT with K <= 4096: the one-phase tile, grouped (= variant 9;
            // sustained, interleaved: 8192^2 x 1024 947 -> 1016 TF, x 2048
            // 1109 -> 1166, 4096^3 1213 -> 1274, 4096 x 14336 x 4096 1109 ->
            // 1179, profiles/r01/gemm/sustained.log); NN and deep K keep the
            // phased schedule (NN 8192^3 1258 vs 1070)
            phased = trans_b && k <= 4096 ? -1 : 7;
            group_m = 4;
        }
        if (variant >= 9 && variant <= 11) group_m = 4 << (variant - 9);
        if (variant == 12 || variant == 13) {
            phased = 7;
            group_m = variant == 12 ? 8 : 4;
        }
        if (variant == 14 || variant == 15) {  // phased SCHED 7 with group_m 2, 16
            phased = 7;
            group_m = variant == 14 ? 2 : 16;
        }
        const bool prio = variant == 4;
        if (dtype == PLI_BF16)
            return launch_256<bf16_t>(a, b, c, bias, m, n, k, lda, ldb, ldc, trans_b, s, phased, prio, group_m);
        return launch_256<f16_t>(a, b, c, bias, m, n, k, lda, ldb, ldc, trans_b, s, phased, prio, group_m);
    }
    if (vec) {
        if (dtype == PLI_BF16)
            return launch_mfma<bf16_t>(a, b, c, bias, m, n, k, lda, ldb, ldc, trans_b, s);
        return launch_mfma<f16_t>(a, b, c, bias, m, n, k, lda, ldb, ldc, trans_b, s);
    }
    // fp32 (the ch01 MHA / ch05 demo dtype): v_mfma_f32_32x32x2_f32 tiles
    // (gemm_f32.hip); the VALU kernel below keeps unaligned / K % 4 != 0 shapes
    if (dtype == PLI_F32 && gemm_f32_mfma_ok(a, b, c, k, n, lda, ldb, trans_b))
        return launch_gemm_f32_mfma(a, b, c, bias, m, n, k, lda, ldb, ldc, trans_b, s);
    switch (dtype) {
        case PLI_F32: return launch_generic<float>(a, b, c, bias, m, n, k, lda, ldb, ldc, trans_b, s);
        case PLI_F16: return launch_generic<f16_t>(a, b, c, bias, m, n, k, lda, ldb, ldc, trans_b, s);
        case PLI_BF16: return launch_generic<bf16_t>(a, b, c, bias, m, n, k, lda, ldb, ldc, trans_b, s);
        default: set_error("pli_gemm: bad dtype %d", dtype); return PLI_EINVAL;
    }
}

extern "C" int pli_gemm(const void* a, const void* b, void* c, const void* bias, int m, int n,
                        int k, int64_t lda, int64_t ldb, int64_t ldc, int trans_b, int dtype,
                        void* stream) {
    return pli_gemm_variant(a, b, c, bias, m, n, k, lda, ldb, ldc, trans_b, dtype, stream, 0);
}

namespace pli {
namespace {
// fp32-output fallback for shapes the LDS kernel does not take: one thread
// per output, fp32 accumulation in k order
template <typename T>
__global__ __launch_bounds__(256) void gemm_f32out_generic(const T* __restrict__ A, const T* __restrict__ Bm,
                                                           float* __restrict__ C, int M, int N, int K,
                                                           int64_t lda, int64_t ldb) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)M * N) return;
    const int m = (int)(i / N), n = (int)(i % N);
    const T* a = A + (int64_t)m * lda;
    const T* b = Bm + (int64_t)n * ldb;
    float acc = 0.f;
    for (int k = 0; k < K; ++k) acc = fmaf(elem<T>::to_f32(a[k]), elem<T>::to_f32(b[k]), acc);
    C[i] = acc;
}
}  // namespace
}  // namespace pli

// C[m][n] = sum_k A[m][k] B[n][k] (NT, the F.linear layout) with bf16 / fp16
// inputs and an fp32 output, contiguous [m, n]: the row-parallel partial of
// ch09/tensor_parallel.py:66-68 kept in fp32 for the all-reduce.  The LDS
// split-K kernel of pli_gemm_ws with one slice writes its fp32 tile straight
// to C; other shapes take a one-thread-per-output kernel.
extern "C" int pli_gemm_f32out(const void* a, const void* b, float* c, int m, int n, int k, int64_t lda,
                               int64_t ldb, int dtype, void* stream) {
    using namespace pli;
    clear_error();
    PLI_REQUIRE(m >= 0 && n >= 0 && k >= 0 && lda >= k && ldb >= k,
                "pli_gemm_f32out: bad shape m=%d n=%d k=%d lda=%lld ldb=%lld", m, n, k, (long long)lda,
                (long long)ldb);
    PLI_REQUIRE(dtype == PLI_BF16 || dtype == PLI_F16, "pli_gemm_f32out: bf16 / fp16 inputs only (%d)", dtype);
    if (m == 0 || n == 0) return PLI_OK;  // (empty operands may be NULL, pli.h)
    PLI_REQUIRE(c && (k == 0 || (a && b)), "pli_gemm_f32out: null pointer");
    hipStream_t s = (hipStream_t)stream;
    const bool lds = k % 64 == 0 && k > 0 && n % 32 == 0 && lda % 8 == 0 && ldb % 8 == 0 && al16(a) &&
                     al16(b) && al16(c);
    // large shapes (128+ tiles of 256^2): gemm_w5 with its fp32 epilogue
    // (persistent where M, N are multiples of 256 and K >= 128); the
    // TP-8 shard at M 8192 ran 214 us on the split-K kernel below
    if (lds && m >= 512 && n >= 512 && (int64_t)cdiv(m, 256) * cdiv(n, 256) >= 128 &&
        gemm_w5_ok(m, n, k, lda, ldb, n, 1)) {
        const bool persist = m % 256 == 0 && n % 256 == 0 && k >= 128;
        return launch_gemm_w5(a, b, c, nullptr, m, n, k, lda, ldb, n, 1, dtype == PLI_BF16, s, 4, persist, true);
    }
    if (lds) {
        if (dtype == PLI_BF16)
            return launch_splitk<bf16_t>(a, b, nullptr, nullptr, m, n, k, lda, ldb, n, 1, c, s, true, false,
                                         true);
        return launch_splitk<f16_t>(a, b, nullptr, nullptr, m, n, k, lda, ldb, n, 1, c, s, true, false, true);
    }
    const int64_t total = (int64_t)m * n;
    PLI_REQUIRE(total / 256 < (1ll << 31), "pli_gemm_f32out: grid too large");
    const dim3 grid((unsigned)((total + 255) / 256));
    if (dtype == PLI_BF16)
        hipLaunchKernelGGL(gemm_f32out_generic<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)a, (const bf16_t*)b,
                           c, m, n, k, lda, ldb);
    else
        hipLaunchKernelGGL(gemm_f32out_generic<f16_t>, grid, dim3(256), 0, s, (const f16_t*)a, (const f16_t*)b,
                           c, m, n, k, lda, ldb);
    return launch_status("gemm_f32out_generic");
}

// Grouped NT GEMM over experts (see gemm_grouped_nt): C[r] = X[gather[r]] W_e^T
// (or silu(. W1_e^T) * (. W3_e^T) when wu_ptrs != NULL) for r in expert e's
// row range [offsets[e], offsets[e+1]).  rows_bound (host) bounds every
// expert's row count and sizes the per-workgroup batch groups.
static int grouped_dispatch(const void* x, const int32_t* gather, const void* const* w_ptrs,
                            const void* const* wu_ptrs, void* c, const int32_t* offsets,
                            int experts, int rows_bound, int n, int k, int64_t ldx, int64_t ldw,
                            int64_t ldc, int dtype, void* stream, int variant);

extern "C" int pli_gemm_grouped(const void* x, const int32_t* gather, const void* const* w_ptrs,
                                const void* const* wu_ptrs, void* c, const int32_t* offsets,
                                int experts, int rows_bound, int n, int k, int64_t ldx,
                                int64_t ldw, int64_t ldc, int dtype, void* stream) {
    return grouped_dispatch(x, gather, w_ptrs, wu_ptrs, c, offsets, experts, rows_bound, n, k, ldx,
                            ldw, ldc, dtype, stream, 0);
}

// Not in pli.h: variant 1 = the weight-streaming / 256-row-tile routes only,
// 2 = the LDS-staged grouped kernel wherever it applies.
extern "C" int pli_gemm_grouped_variant(const void* x, const int32_t* gather,
                                        const void* const* w_ptrs, const void* const* wu_ptrs,
                                        void* c, const int32_t* offsets, int experts,
                                        int rows_bound, int n, int k, int64_t ldx, int64_t ldw,
                                        int64_t ldc, int dtype, void* stream, int variant) {
    return grouped_dispatch(x, gather, w_ptrs, wu_ptrs, c, offsets, experts, rows_bound, n, k, ldx,
                            ldw, ldc, dtype, stream, variant);
}

static int grouped_dispatch(const void* x, const int32_t* gather, const void* const* w_ptrs,
                            const void* const* wu_ptrs, void* c, const int32_t* offsets,
                            int experts, int rows_bound, int n, int k, int64_t ldx, int64_t ldw,
                            int64_t ldc, int dtype, void* stream, int variant) {
    using namespace pli;
    clear_error();
    PLI_REQUIRE(experts > 0 && rows_bound >= 0 && n > 0 && k > 0,
                "pli_gemm_grouped: bad shape E=%d rows=%d n=%d k=%d", experts, rows_bound, n, k);
    if (rows_bound == 0) return PLI_OK;  // (empty operands may be NULL, pli.h)
    PLI_REQUIRE(x && w_ptrs && c && offsets, "pli_gemm_grouped: null pointer");
    PLI_REQUIRE(dtype == PLI_BF16 || dtype == PLI_F16, "pli_gemm_grouped: bf16/fp16 only");
    PLI_REQUIRE(k % 128 == 0 && n % 16 == 0 && ldx % 8 == 0 && ldw % 8 == 0 && ldc % 8 == 0 &&
                    al16(x) && al16(c),
                "pli_gemm_grouped: needs k %% 128 == 0, n %% 16 == 0, 16-byte aligned rows");
    PLI_REQUIRE(ldx >= k && ldw >= k && ldc >= n, "pli_gemm_grouped: leading dimension too small");
    if (rows_bound == 0) return PLI_OK;
    hipStream_t st = (hipStream_t)stream;
    // decode-sized routing, 16 < rows <= 1024: the LDS-staged grouped kernel
    // (n % 64 for the SwiGLU form, n % 128 plain; k % 128 holds).  MoEConfig
    // defaults, both grouped GEMMs (profiles/r01/gemm/tune_moe_grouped.log):
    // 32 tokens 717 -> 599 us (4.7 TB/s of expert weights), 128 tokens 734 ->
    // 682, 256 tokens 791 -> 701; 1-8 tokens keep the weight-streaming kernel
    // (1 token: 140 vs 312 us).
    const bool sw = wu_ptrs != nullptr;
    const bool lds_ok = rows_bound <= 1024 && n % (sw ? 64 : 128) == 0;
    if (lds_ok && variant != 1 && (variant == 2 || rows_bound > 16)) {
        const int mc = cdiv(min(rows_bound, 128), 32);
        const dim3 grid((unsigned)(n / (sw ? 64 : 128)), (unsigned)cdiv(rows_bound, 128), (unsigned)experts);
        const auto* Xg = (const uint16_t*)x;
        const auto* const* Wg = (const uint16_t* const*)w_ptrs;
        const auto* const* Wug = (const uint16_t* const*)wu_ptrs;
#define PLI_GLDS(TT, MCC, SWW)                                                                   \
    hipLaunchKernelGGL((gemm_grouped_lds_nt<TT, MCC, SWW>), grid, dim3(256), 0, st, Xg, ldx, gather, \
                       Wg, Wug, ldw, (uint16_t*)c, ldc, offsets, n, k)
#define PLI_GLDS_MC(TT, SWW)                  \
    do {                                      \
        if (mc == 1) PLI_GLDS(TT, 1, SWW);    \
        else if (mc == 2) PLI_GLDS(TT, 2, SWW); \
        else if (mc == 3) PLI_GLDS(TT, 3, SWW); \
        else PLI_GLDS(TT, 4, SWW);            \
    } while (0)
        if (dtype == PLI_BF16) {
            if (sw) PLI_GLDS_MC(bf16_t, true); else PLI_GLDS_MC(bf16_t, false);
        } else {
            if (sw) PLI_GLDS_MC(f16_t, true); else PLI_GLDS_MC(f16_t, false);
        }
#undef PLI_GLDS_MC
#undef PLI_GLDS
        return launch_status("gemm_grouped_lds_nt");
    }
    if (variant != 2 && rows_bound >= 16 * experts) {
        // prefill-sized routing (>= 16 rows per expert on average): the phased
        // 256-row tile per (expert, slot); decode sizes stay on the
        // weight-streaming kernel below
        const bool sw = wu_ptrs != nullptr;
        const int slots = cdiv(rows_bound, G2M) + experts;
        const int tn = cdiv(n, sw ? 128 : G2N);
        const int64_t nb = (int64_t)slots * tn;
        PLI_REQUIRE(nb < (1ll << 31), "pli_gemm_grouped: grid too large");
        const auto* Xg = (const uint16_t*)x;
        const auto* const* Wg = (const uint16_t* const*)w_ptrs;
        const auto* const* Wug = (const uint16_t* const*)wu_ptrs;
#define PLI_G256G(TT, SW)                                                                          \
    hipLaunchKernelGGL((gemm_256g<TT, SW>), dim3((unsigned)nb), dim3(512), 0, st, Xg, ldx, gather, \
                       Wg, Wug, ldw, (uint16_t*)c, ldc, offsets, experts, n, k, slots, tn, (int)nb)
        if (dtype == PLI_BF16) {
            if (sw) PLI_G256G(bf16_t, true); else PLI_G256G(bf16_t, false);
        } else {
            if (sw) PLI_G256G(f16_t, true); else PLI_G256G(f16_t, false);
        }
#undef PLI_G256G
        return launch_status("gemm_256g");
    }
    const int nblk = n / 16;
    PLI_REQUIRE((int64_t)experts * nblk < (1ll << 31), "pli_gemm_grouped: grid too large");
    const dim3 grid((unsigned)(experts * nblk)), block(256);
    hipStream_t s = (hipStream_t)stream;
    const auto* X = (const uint16_t*)x;
    const auto* const* W = (const uint16_t* const*)w_ptrs;
    const auto* const* Wu = (const uint16_t* const*)wu_ptrs;
    auto* Cc = (uint16_t*)c;
#define PLI_GRP(TT, NBG, SW)                                                                      \
    hipLaunchKernelGGL((gemm_grouped_nt<TT, NBG, SW>), grid, block, 0, s, X, gather, W, Wu, Cc, \
                       offsets, n, k, ldx, ldw, ldc, nblk)
#define PLI_GRP_NBG(TT, SW)                                                                       \
    do {                                                                                          \
        if (rows_bound <= 16) PLI_GRP(TT, 1, SW);                                                 \
        else if (rows_bound <= 32) PLI_GRP(TT, 2, SW);                                            \
        else if (rows_bound <= 64) PLI_GRP(TT, 4, SW);                                            \
        else PLI_GRP(TT, 8, SW);                                                                  \
    } while (0)
    if (dtype == PLI_BF16) {
        if (wu_ptrs) PLI_GRP_NBG(bf16_t, true); else PLI_GRP_NBG(bf16_t, false);
    } else {
        if (wu_ptrs) PLI_GRP_NBG(f16_t, true); else PLI_GRP_NBG(f16_t, false);
    }
#undef PLI_GRP_NBG
#undef PLI_GRP
    return launch_status("pli_gemm_grouped");
}

// Multi-output decode projection (see gemm_skinny_multi): up to 3 groups
// sharing X [m, k] (m <= 16 rows = batch x tokens_per_batch); each group g
// writes c_g[b * stride_batch + (s + *row_offset) * stride_token + n] for
// row r = b * tokens_per_batch + s (row_offset may be NULL = 0; rows at or
// past `capacity` are dropped).
extern "C" int pli_gemm_multi_nt(const void* x, int64_t ldx, int m, int k, int tokens_per_batch,
                                 const void* const* w, void* const* c, const int* n,
                                 const int64_t* ldw, const int64_t* stride_batch,
                                 const int64_t* stride_token, const int32_t* const* row_offset,
                                 const int* capacity, int ngroups, int dtype, void* stream) {
    using namespace pli;
    clear_error();
    PLI_REQUIRE(x && w && c && n && ldw && stride_batch && stride_token && row_offset && capacity,
                "pli_gemm_multi_nt: null pointer");
    PLI_REQUIRE(ngroups >= 1 && ngroups <= 3, "pli_gemm_multi_nt: 1..3 groups, got %d", ngroups);
    PLI_REQUIRE(m >= 1 && m <= 128 && k > 0 && k % 8 == 0 && ldx >= k && ldx % 8 == 0 &&
                    tokens_per_batch >= 1 && m % tokens_per_batch == 0 && al16(x),
                "pli_gemm_multi_nt: needs 1 <= m <= 128 rows (whole batches), k %% 8 == 0, aligned x");
    PLI_REQUIRE(m <= 16 || k % 128 == 0, "pli_gemm_multi_nt: m > 16 needs k %% 128 == 0");
    PLI_REQUIRE(dtype == PLI_BF16 || dtype == PLI_F16, "pli_gemm_multi_nt: bf16/fp16 only");
    MultiArgs args{};
    int ntot = 0;
    for (int g = 0; g < ngroups; ++g) {
        PLI_REQUIRE(w[g] && c[g] && n[g] > 0 && ldw[g] >= k && ldw[g] % 8 == 0 && al16(w[g]),
                    "pli_gemm_multi_nt: bad group %d", g);
        PLI_REQUIRE(m <= 16 || (n[g] % 16 == 0 && stride_batch[g] % 4 == 0 &&
                                stride_token[g] % 4 == 0 && ((uintptr_t)c[g] & 7) == 0),
                    "pli_gemm_multi_nt: m > 16 needs group widths %% 16 == 0 and 8-byte "
                    "aligned output rows (group %d)", g);
        args.g[g] = MultiGroup{(const uint16_t*)w[g], (uint16_t*)c[g], n[g], ldw[g],
                               stride_batch[g], stride_token[g], row_offset[g], capacity[g]};
        ntot += n[g];
    }
    args.ngroups = ngroups;
    if (m > 16) {
        // 16 < m <= 128: the small-M MFMA kernel with the per-group row
        // addressing in its epilogue (one launch for q/k/v + the cache append)
        hipStream_t st = (hipStream_t)stream;
        const dim3 grid(ntot / 16), block(256);
        const auto* X = (const uint16_t*)x;
#define PLI_MSM(TT, G)                                                                        \
    hipLaunchKernelGGL((gemm_smallm_nt<TT, G, false, false, true>), grid, block, 0, st, X,     \
                       nullptr, nullptr, nullptr, m, 0, k, ldx, 0, 0, nullptr, 0, args,         \
                       tokens_per_batch)
#define PLI_MSM_G(TT)                          \
    do {                                       \
        if (m <= 32) PLI_MSM(TT, 2);           \
        else if (m <= 64) PLI_MSM(TT, 4);      \
        else PLI_MSM(TT, 8);                   \
    } while (0)
        if (dtype == PLI_BF16) PLI_MSM_G(bf16_t); else PLI_MSM_G(f16_t);
#undef PLI_MSM_G
#undef PLI_MSM
        return launch_status("pli_gemm_multi_nt<smallm>");
    }
    const dim3 grid(cdiv(ntot, 2)), block(128);
    hipStream_t s = (hipStream_t)stream;
    const auto* X = (const uint16_t*)x;
    const int nch = k / 8;
#define PLI_MULTI(TT, NB)                                                                              \
    do {                                                                                               \
        if (nch <= 128) /* K <= 1024: 2 chunks per lane, same chunk order */                          \
            hipLaunchKernelGGL((gemm_skinny_multi<TT, NB, 2>), grid, block, 0, s, X, m, tokens_per_batch, nch, ldx, args); \
        else if (nch <= 256) /* K <= 2048: 4 chunks per lane */                                        \
            hipLaunchKernelGGL((gemm_skinny_multi<TT, NB, 4>), grid, block, 0, s, X, m, tokens_per_batch, nch, ldx, args); \
        else                                                                                           \
            hipLaunchKernelGGL((gemm_skinny_multi<TT, NB>), grid, block, 0, s, X, m, tokens_per_batch, nch, ldx, args); \
    } while (0)
#define PLI_MULTI_NB(TT)                  \
    do {                                  \
        if (m <= 1) PLI_MULTI(TT, 1);     \
        else if (m <= 2) PLI_MULTI(TT, 2);\
        else if (m <= 4) PLI_MULTI(TT, 4);\
        else if (m <= 8) PLI_MULTI(TT, 8);\
        else PLI_MULTI(TT, 16);           \
    } while (0)
    if (dtype == PLI_BF16) PLI_MULTI_NB(bf16_t); else PLI_MULTI_NB(f16_t);
#undef PLI_MULTI_NB
#undef PLI_MULTI
    return launch_status("pli_gemm_multi_nt");
}
