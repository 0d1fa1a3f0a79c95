// Split-K decode attention over a KV cache (flash-decoding) for gfx950.
//
// Replaces the decode branch of the reference's cached attention
// (ch02/kv_cache.py:74-101, ch02/cached_generation.py:58-98): there the
// cache [B, S, Hkv, D] is transposed, repeat_interleave'd to Hq heads
// (ch02/kv_cache.py:85-86 materialises G copies of the whole cache) and run
// through matmul -> softmax -> matmul.  Here every K/V byte is read from HBM
// once per kv head, whatever the group size.
//
// Work decomposition (HBM-bound: a decode step reads the whole cache and does
// ~2 FLOP per byte):
//   * one workgroup = (batch, kv head, chunk of keys); 4 waves, each wave runs
//     its own online softmax over 32-key steps of its quarter of the chunk;
//   * the M = n_q * G query rows of the kv head (G = Hq/Hkv, rows ordered
//     m = qi*G + gi) are the columns of one 16-wide MFMA tile, so M <= 16;
//   * S^T[32 keys][16 rows] = K . Q^T by v_mfma_f32_16x16x32: the A operand
//     (K rows) is loaded straight from HBM into registers in fragment order,
//     no LDS; Q^T is the register-resident B operand;
//   * P^T stays in the S registers (keys permuted: j<4 -> 4g+j, j>=4 ->
//     16+4g+j-4), V^T comes from a wave-private LDS tile through
//     ds_read_b64_tr_b16 (rows padded to 2D+32 B: conflict-free);
//   * next step's K/V loads are issued before this step's MFMAs, so each wave
//     keeps 16 KB (D=128) in flight;
//   * waves merge in LDS; with more than one chunk per head the partial
//     (m, l, O) go to a caller-provided fp32 workspace and a combine kernel
//     merges them (log-sum-exp weights) into the output.
// fp32 statistics; the row sum is taken over the rounded P that P.V uses.
#include <cmath>

#include "pli_common.h"

namespace pli {
namespace {

struct DecStrides {
    int64_t qb, qh, qn, kb, kh, kn, vb, vh, vn, ob, oh, on;
};

constexpr int DEC_WAVES = 4;
constexpr int DEC_STEP = 32;                        // keys per wave step
constexpr int DEC_QUANT = DEC_WAVES * DEC_STEP;     // chunk granularity
constexpr int DEC_MAXM = 16;                        // query rows per kv head

template <int D, bool KLDS> struct DecLayout {
    static constexpr int KS = 2 * D + 16;             // K row stride in LDS (bytes)
    static constexpr int VS = 2 * D + 32;             // V row stride in LDS (bytes)
    static constexpr int KBYTES = KLDS ? DEC_STEP * KS : 0;
    static constexpr int WAVE_BYTES = KBYTES + DEC_STEP * VS;  // per-wave K? + V tile
    static constexpr int MERGE_BYTES = DEC_WAVES * (DEC_MAXM * D + 2 * DEC_MAXM) * 4;
    static constexpr int LDS = WAVE_BYTES * DEC_WAVES > MERGE_BYTES ? WAVE_BYTES * DEC_WAVES
                                                                     : MERGE_BYTES;
};

// MODE 0: K/V of step t+1 loaded into a second register set during step t
//         (2 waves/SIMD);
// MODE 1: as 0 with non-temporal loads (the cache is streamed once);
// MODE 2: one register set; step t+1's loads are issued as soon as step t's
//         K has fed its MFMAs and its V is in LDS; <= 168 VGPRs, 3 waves/SIMD;
// MODE | 4: kv head innermost in the block order;
// MODE | 8: K and V loaded as whole rows (each load instruction covers
//           64/(D/8) complete rows, full 128-B lines) into wave-private LDS
//           tiles; K fragments are then read back with ds_read_b128.
template <typename T, int D, int MODE>
__global__ __launch_bounds__(256, (MODE & 2) ? 3 : 2) void attn_decode_chunk(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
    const uint16_t* __restrict__ v, uint16_t* __restrict__ o, float* __restrict__ part_o,
    float2* __restrict__ part_ml, int Hkv, int G, int Nq, int Nk, int M, DecStrides st, float c,
    int causal, int chunk, int splits, const int* __restrict__ nk_dev, int nk_add) {
    // graph-replayable form: the valid length lives in device memory (the
    // grid is planned for the capacity Nk; chunks past the length exit empty)
    if (nk_dev != nullptr) Nk = max(0, min(Nk, *nk_dev + nk_add));
    constexpr bool RM = (MODE & 8) != 0;
    using L = DecLayout<D, RM>;
    constexpr int KSTEPS = D / 32;  // 32-d k-steps of K.Q^T
    constexpr int DB = D / 16;      // 16-d blocks of O
    __shared__ __attribute__((aligned(16))) char smem[L::LDS];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int l16 = lane & 15, g = lane >> 4;
    // block order: (b, split, hk) with the kv head innermost, so co-resident
    // workgroups sweep the same keys of all heads (contiguous cache rows)
    int split, bh, b, hk;
    if constexpr ((MODE & 4) != 0) {
        hk = blockIdx.x % Hkv;
        split = (blockIdx.x / Hkv) % splits;
        b = blockIdx.x / (Hkv * splits);
        bh = b * Hkv + hk;
    } else {
        split = blockIdx.x % splits;
        bh = blockIdx.x / splits;
        b = bh / Hkv;
        hk = bh % Hkv;
    }

    // query row of this lane's MFMA column
    const int m_row = l16;
    const bool row_ok = m_row < M;
    const int qi = row_ok ? m_row / G : 0, gi = row_ok ? m_row % G : 0;
    const int hq = hk * G + gi;
    i32x4 qf[KSTEPS];
    {
        const uint16_t* src = q + b * st.qb + hq * st.qh + (int64_t)qi * st.qn + 8 * g;
#pragma unroll
        for (int ks = 0; ks < KSTEPS; ++ks) {
            const i32x4 x = *reinterpret_cast<const i32x4*>(src + 32 * ks);
            qf[ks] = row_ok ? x : i32x4{0, 0, 0, 0};
        }
    }
    // bottom-right causal: row qi sees keys <= Nk - Nq + qi
    const int lim = causal ? Nk - Nq + qi : Nk - 1;

    const int c0 = split * chunk;
    const int per_wave = chunk / DEC_WAVES;
    const int w0 = c0 + wave * per_wave;
    const int w1 = min(w0 + per_wave, Nk);
    const int nsteps = w1 > w0 ? cdiv(w1 - w0, DEC_STEP) : 0;

    // fragment-order loads: lane loads rows l16 and 16+l16 of a step,
    // d-chunks 32ks + 8g.  Row-major loads (RM): lane loads chunk rch of row
    // i*RPI + rrow for instruction i = kb*KSTEPS + ks.
    constexpr int CPR = D / 8, RPI = 64 / CPR;
    const int rrow = lane / CPR, rch = lane % CPR;
    const uint16_t* kp = k + b * st.kb + hk * st.kh + (RM ? 8 * rch : 8 * g);
    const uint16_t* vp = v + b * st.vb + hk * st.vh + (RM ? 8 * rch : 8 * g);
    i32x4 kc[2][KSTEPS], vc[2][KSTEPS];
    auto ld = [](const uint16_t* p) {
        if constexpr ((MODE & 1) != 0) return __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(p));
        else return *reinterpret_cast<const i32x4*>(p);
    };
    auto load_step = [&](int key0, i32x4 (&kr)[2][KSTEPS], i32x4 (&vr)[2][KSTEPS]) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
            for (int ks = 0; ks < KSTEPS; ++ks) {
                if constexpr (RM) {
                    const int64_t key = min(key0 + (kb * KSTEPS + ks) * RPI + rrow, Nk - 1);
                    kr[kb][ks] = ld(kp + key * st.kn);
                    vr[kb][ks] = ld(vp + key * st.vn);
                } else {
                    const int64_t key = min(key0 + 16 * kb + l16, Nk - 1);
                    kr[kb][ks] = ld(kp + key * st.kn + 32 * ks);
                    vr[kb][ks] = ld(vp + key * st.vn + 32 * ks);
                }
            }
        }
    };

    char* kt = smem + wave * L::WAVE_BYTES;
    char* vt = kt + L::KBYTES;
    const int vw = RM ? rrow * L::VS + rch * 16 : l16 * L::VS + g * 16;
    const int kw = rrow * L::KS + rch * 16;                     // RM: K row-major write
    const int kr_off = l16 * L::KS + g * 16;                    // RM: K fragment read
    const int qq = l16 >> 2, pp = lane & 3;
    const int vr_off = (4 * g + qq) * L::VS + 8 * pp;           // tr read: key 4g+qq, col 4pp

    f32x4 oacc[DB];
#pragma unroll
    for (int d = 0; d < DB; ++d) oacc[d] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m_run = -1e30f, l_run = 0.f;

    if (nsteps > 0) load_step(w0, kc, vc);
    for (int it = 0; it < nsteps; ++it) {
        const int key0 = w0 + it * DEC_STEP;
        i32x4 kn[2][KSTEPS], vn[2][KSTEPS];
        if constexpr ((MODE & 2) == 0) {
            if (it + 1 < nsteps) load_step(key0 + DEC_STEP, kn, vn);
        }

        // V step -> LDS (row-major, padded) for the transposed reads
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int ks = 0; ks < KSTEPS; ++ks) {
                if constexpr (RM) {
                    const int row0 = (kb * KSTEPS + ks) * RPI;
                    lds_write_b128(vt, vw + row0 * L::VS, vc[kb][ks]);
                    lds_write_b128(kt, kw + row0 * L::KS, kc[kb][ks]);
                } else {
                    lds_write_b128(vt, vw + 16 * kb * L::VS + 64 * ks, vc[kb][ks]);
                }
            }
        // the tile is wave-private and a wave's LDS operations execute in
        // order; the fence only stops the compiler moving the transposed reads
        // (a different pointer type) above these writes
        asm volatile("" ::: "memory");

        f32x4 s[2];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            s[kb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < KSTEPS; ++ks) {
                if constexpr (RM) {
                    const i32x4 kf = lds_read_b128(kt, kr_off + 16 * kb * L::KS + 64 * ks);
                    s[kb] = mfma16x16x32<T>(kf, qf[ks], s[kb]);
                } else {
                    s[kb] = mfma16x16x32<T>(kc[kb][ks], qf[ks], s[kb]);
                }
            }
        }
        if constexpr ((MODE & 2) != 0) {
            if (it + 1 < nsteps) load_step(key0 + DEC_STEP, kc, vc);
        }
        // mask: keys past this wave's range / the cache / the causal limit
        const int hi = min(w1 - 1, lim);
        if (key0 + DEC_STEP - 1 > hi) {
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (key0 + 16 * kb + 4 * g + r > hi) s[kb][r] = -INFINITY;
        }
        float mx = max3(s[0][0], s[0][1], s[0][2]);
        mx = max3(mx, s[0][3], s[1][0]);
        mx = max3(mx, s[1][1], s[1][2]);
        mx = fmaxf(mx, s[1][3]);
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float m_new = fmaxf(m_run, mx * c);
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        m_run = m_new;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int r = 0; r < 4; ++r) s[kb][r] = __builtin_amdgcn_exp2f(fmaf(s[kb][r], c, -m_new));
        const uint32_t p0 = pack2<T>(s[0][0], s[0][1]), p1 = pack2<T>(s[0][2], s[0][3]);
        const uint32_t p2 = pack2<T>(s[1][0], s[1][1]), p3 = pack2<T>(s[1][2], s[1][3]);
        const i32x4 pb = {(int)p0, (int)p1, (int)p2, (int)p3};
        l_run = fmaf(l_run, alpha, add_pair<T>(p0, add_pair<T>(p1, add_pair<T>(p2, add_pair<T>(p3, 0.f)))));

#pragma unroll
        for (int d = 0; d < DB; ++d) {
            const i32x2 lo = lds_read_tr16(vt, vr_off + 32 * d);
            const i32x2 hi2 = lds_read_tr16(vt, vr_off + 32 * d + 16 * L::VS);
            oacc[d] = mfma16x16x32<T>(i32x4{lo.x, lo.y, hi2.x, hi2.y}, pb, oacc[d] * alpha);
        }
        asm volatile("" ::: "memory");  // next step's writes stay below these reads
        if ((MODE & 2) == 0 && it + 1 < nsteps) {
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int ks = 0; ks < KSTEPS; ++ks) {
                    kc[kb][ks] = kn[kb][ks];
                    vc[kb][ks] = vn[kb][ks];
                }
        }
    }
    // row sum over the 4 lane groups holding the row
    l_run += __shfl_xor(l_run, 16, 64);
    l_run += __shfl_xor(l_run, 32, 64);

    // ---- merge the 4 waves in LDS: [wave][row][D] O, then [wave][row] (m, l)
    __syncthreads();  // every wave is done with its V tile
    float* mo = reinterpret_cast<float*>(smem);
    float* mml = mo + DEC_WAVES * DEC_MAXM * D;
#pragma unroll
    for (int d = 0; d < DB; ++d)
        *reinterpret_cast<f32x4*>(mo + (wave * DEC_MAXM + l16) * D + 16 * d + 4 * g) = oacc[d];
    if (g == 0) {
        mml[(wave * DEC_MAXM + l16) * 2] = m_run;
        mml[(wave * DEC_MAXM + l16) * 2 + 1] = l_run;
    }
    __syncthreads();
    constexpr int CH = D / 4;  // float4 chunks per row
    for (int item = tid; item < M * CH; item += 256) {
        const int row = item / CH, cc = item % CH;
        float mw[DEC_WAVES], mt = -1e30f;
#pragma unroll
        for (int w = 0; w < DEC_WAVES; ++w) {
            mw[w] = mml[(w * DEC_MAXM + row) * 2];
            mt = fmaxf(mt, mw[w]);
        }
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        float lt = 0.f;
#pragma unroll
        for (int w = 0; w < DEC_WAVES; ++w) {
            const float wgt = __builtin_amdgcn_exp2f(mw[w] - mt);
            lt = fmaf(mml[(w * DEC_MAXM + row) * 2 + 1], wgt, lt);
            acc += *reinterpret_cast<const f32x4*>(mo + (w * DEC_MAXM + row) * D + 4 * cc) * wgt;
        }
        if (splits == 1) {
            const float inv = lt > 0.f ? 1.f / lt : 0.f;
            const int rqi = row / G, rgi = row % G;
            uint16_t* op = o + b * st.ob + (hk * G + rgi) * st.oh + (int64_t)rqi * st.on + 4 * cc;
            *reinterpret_cast<i32x2*>(op) =
                i32x2{(int)pack2<T>(acc[0] * inv, acc[1] * inv), (int)pack2<T>(acc[2] * inv, acc[3] * inv)};
        } else {
            const int64_t prow = ((int64_t)bh * splits + split) * M + row;
            *reinterpret_cast<f32x4*>(part_o + prow * D + 4 * cc) = acc;
            if (cc == 0) part_ml[prow] = float2{mt, lt};
        }
    }
}

// Merge `splits` partial (m, l, O) rows per (batch, kv head, row) into the
// output.  One workgroup per (bh, row); thread = (16-byte chunk of the row,
// split lane): each thread folds every LANES-th split into a running
// (m, l, O) in one pass (loads independent, unrolled), then the split lanes
// are merged in LDS.  (A first pass over all splits for the global max would
// be a serial chain of `splits` dependent loads.)
template <typename T, int D>
__global__ __launch_bounds__(256) void attn_decode_combine(
    const float* __restrict__ part_o, const float2* __restrict__ part_ml, uint16_t* __restrict__ o,
    int Hkv, int G, int M, DecStrides st, int splits) {
    constexpr int CH = D / 4, LANES = 256 / CH;
    __shared__ f32x4 red_o[LANES][CH];
    __shared__ float2 red_ml[LANES][CH];
    const int tid = threadIdx.x, cc = tid % CH, sl = tid / CH;
    const int row = blockIdx.x % M, bh = blockIdx.x / M;
    const int b = bh / Hkv, hk = bh % Hkv;
    const int64_t base = (int64_t)bh * splits * M + row;  // + s*M
    float mt = -1e30f, lt = 0.f;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int s = sl; s < splits; s += LANES) {
        const int64_t pr = base + (int64_t)s * M;
        const float2 ml = part_ml[pr];
        const f32x4 po = *reinterpret_cast<const f32x4*>(part_o + pr * D + 4 * cc);
        const float mn = fmaxf(mt, ml.x);
        const float wa = __builtin_amdgcn_exp2f(mt - mn), wb = __builtin_amdgcn_exp2f(ml.x - mn);
        acc = acc * wa + po * wb;
        lt = lt * wa + ml.y * wb;
        mt = mn;
    }
    red_o[sl][cc] = acc;
    red_ml[sl][cc] = float2{mt, lt};
    __syncthreads();
    if (sl == 0) {
        for (int j = 1; j < LANES; ++j) {
            const float2 ml = red_ml[j][cc];
            const float mn = fmaxf(mt, ml.x);
            const float wa = __builtin_amdgcn_exp2f(mt - mn), wb = __builtin_amdgcn_exp2f(ml.x - mn);
            acc = acc * wa + red_o[j][cc] * wb;
            lt = lt * wa + ml.y * wb;
            mt = mn;
        }
        const float inv = lt > 0.f ? 1.f / lt : 0.f;
        const int rqi = row / G, rgi = row % G;
        uint16_t* op = o + b * st.ob + (hk * G + rgi) * st.oh + (int64_t)rqi * st.on + 4 * cc;
        *reinterpret_cast<i32x2*>(op) =
            i32x2{(int)pack2<T>(acc[0] * inv, acc[1] * inv), (int)pack2<T>(acc[2] * inv, acc[3] * inv)};
    }
}

// Chunking: enough workgroups to keep every CU's loads in flight (~4 per CU),
// at least one 32-key step per wave; chunk is a multiple of 4 waves x 32 keys.
struct DecPlan {
    int chunk, splits;
};
constexpr int64_t kDefaultTargetWgs = 1024;
// Short caches (<= kNoSplitKeys keys) with >= kNoSplitWgs (batch, kv head)
// pairs take one chunk per pair: the combine launch (~4.7 us) costs more than
// the serial key loop it saves (graph decode step, batch 32, 560-key cache:
// 1.279 -> 1.246 ms/token); with few pairs the split stays (batch 1: 8
// one-chunk workgroups ran 0.715 vs 0.681 ms/token).
constexpr int kNoSplitKeys = 1024, kNoSplitWgs = 128;
DecPlan plan_decode(int64_t bh, int n_kv, int64_t kTargetWgs = kDefaultTargetWgs) {
    const int64_t max_splits = cdiv(n_kv, DEC_QUANT);
    int64_t splits = bh >= kTargetWgs || (n_kv <= kNoSplitKeys && bh >= kNoSplitWgs)
                         ? 1
                         : cdiv(kTargetWgs, bh);
    splits = splits < 1 ? 1 : (splits > max_splits ? max_splits : splits);
    const int chunk = (int)(cdiv(cdiv(n_kv, splits), DEC_QUANT) * DEC_QUANT);
    return {chunk, (int)cdiv(n_kv, chunk)};
}

bool decode_fast_path(int heads, int kv_heads, int n_q, int n_kv, int head_dim, int dtype,
                      const int64_t* strides) {
    if (!(dtype == PLI_BF16 || dtype == PLI_F16)) return false;
    if (!(head_dim == 64 || head_dim == 128) || n_kv <= 0) return false;
    if ((int64_t)n_q * (heads / kv_heads) > DEC_MAXM) return false;
    for (int i = 0; i < 12; ++i)
        if (strides[i] % 8 != 0) return false;
    return true;
}

// default: whole-row non-temporal loads, K/V via LDS, kv head innermost in the grid
// (4.3-6.1 TB/s over 128 MiB-1 GiB caches vs 2.4-5.1 for fragment-order loads)
constexpr int kDefaultDecodeMode = 13;

template <typename T, int D>
int launch_decode(const void* q, const void* k, const void* v, void* o, int B, int Hkv, int G,
                  int Nq, int Nk, const DecStrides& st, float scale, int causal, float* ws,
                  hipStream_t stream, int mode, int target, const int* nk_dev = nullptr,
                  int nk_add = 0) {
    const int64_t bh = (int64_t)B * Hkv;
    const DecPlan p = plan_decode(bh, Nk, target > 0 ? target : kDefaultTargetWgs);
    if (nk_dev == nullptr && Nk == 0) return PLI_OK;
    const int M = Nq * G;
    PLI_REQUIRE(bh * p.splits < (1ll << 31), "pli_attn_decode: grid too large");
    const float c = scale * 1.4426950408889634f;
    float* part_o = ws;
    float2* part_ml = reinterpret_cast<float2*>(ws + bh * p.splits * M * D);
#define PLI_DEC_LAUNCH(MODE)                                                                     \
    hipLaunchKernelGGL((attn_decode_chunk<T, D, MODE>), dim3((unsigned)(bh * p.splits)), dim3(256), \
                       0, stream, (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v,     \
                       (uint16_t*)o, part_o, part_ml, Hkv, G, Nq, Nk, M, st, c, causal, p.chunk, \
                       p.splits, nk_dev, nk_add)
    switch (mode < 0 ? kDefaultDecodeMode : mode) {
        case 1: PLI_DEC_LAUNCH(1); break;
        case 2: PLI_DEC_LAUNCH(2); break;
        case 4: PLI_DEC_LAUNCH(4); break;
        case 5: PLI_DEC_LAUNCH(5); break;
        case 6: PLI_DEC_LAUNCH(6); break;
        case 8: PLI_DEC_LAUNCH(8); break;
        case 9: PLI_DEC_LAUNCH(9); break;
        case 10: PLI_DEC_LAUNCH(10); break;
        case 11: PLI_DEC_LAUNCH(11); break;
        case 13: PLI_DEC_LAUNCH(13); break;
        default: PLI_DEC_LAUNCH(0); break;
    }
#undef PLI_DEC_LAUNCH
    if (p.splits > 1)
        hipLaunchKernelGGL((attn_decode_combine<T, D>), dim3((unsigned)(bh * M)), dim3(256), 0,
                           stream, part_o, part_ml, (uint16_t*)o, Hkv, G, M, st, p.splits);
    return launch_status(p.splits > 1 ? "attn_decode_chunk+attn_decode_combine" : "attn_decode_chunk");
}

// Append n_new tokens of K and V to the caches at the device-resident
// position *pos (+ i); rows past the capacity are dropped.  One thread per
// 16-byte chunk.
__global__ __launch_bounds__(256) void kv_append_kernel(
    const uint16_t* __restrict__ kn, const uint16_t* __restrict__ vn, uint16_t* __restrict__ kc,
    uint16_t* __restrict__ vc, int B, int T, int Hkv, int D, int cap, DecStrides st,
    const int* __restrict__ pos) {
    const int cpr = D / 8;
    const int64_t total = (int64_t)B * T * Hkv * cpr;
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= total) return;
    const int ch = idx % cpr;
    const int h = (idx / cpr) % Hkv;
    const int t = (idx / ((int64_t)cpr * Hkv)) % T;
    const int b = idx / ((int64_t)cpr * Hkv * T);
    const int row = *pos + t;
    if (row < 0 || row >= cap) return;
    // strides: q.. slots carry the new tensors, k/v slots the caches
    const uint16_t* ks = kn + b * st.qb + h * st.qh + (int64_t)t * st.qn + 8 * ch;
    const uint16_t* vs = vn + b * st.ob + h * st.oh + (int64_t)t * st.on + 8 * ch;
    uint16_t* kd = kc + b * st.kb + h * st.kh + (int64_t)row * st.kn + 8 * ch;
    uint16_t* vd = vc + b * st.vb + h * st.vh + (int64_t)row * st.vn + 8 * ch;
    *reinterpret_cast<i32x4*>(kd) = *reinterpret_cast<const i32x4*>(ks);
    *reinterpret_cast<i32x4*>(vd) = *reinterpret_cast<const i32x4*>(vs);
}

}  // namespace
}  // namespace pli

extern "C" int pli_kv_append(const void* k_new, const void* v_new, void* k_cache, void* v_cache,
                             int batch, int n_new, int kv_heads, int head_dim, int capacity,
                             const int64_t* strides, const int32_t* pos_dev, int dtype,
                             void* stream) {
    using namespace pli;
    clear_error();
    PLI_REQUIRE(batch >= 0 && n_new >= 0 && kv_heads > 0 && head_dim > 0 && capacity >= 0,
                "pli_kv_append: bad shape B=%d T=%d Hkv=%d D=%d cap=%d", batch, n_new, kv_heads,
                head_dim, capacity);
    // nothing to append: the (possibly NULL, pli.h) operands are not read
    if (batch == 0 || n_new == 0) return PLI_OK;
    PLI_REQUIRE(k_new && v_new && k_cache && v_cache && strides && pos_dev,
                "pli_kv_append: null pointer");
    PLI_REQUIRE(dtype == PLI_F16 || dtype == PLI_BF16, "pli_kv_append: dtype %d (16-bit caches only)",
                dtype);
    PLI_REQUIRE(head_dim % 8 == 0 && aligned16(k_new) && aligned16(v_new) && aligned16(k_cache) &&
                    aligned16(v_cache),
                "pli_kv_append: head_dim %% 8 and 16-byte aligned operands required");
    for (int i = 0; i < 12; ++i)
        PLI_REQUIRE(strides[i] % 8 == 0, "pli_kv_append: stride %d not a multiple of 8", i);
    const int64_t total = (int64_t)batch * n_new * kv_heads * (head_dim / 8);
    if (total == 0) return PLI_OK;
    // strides[12] = {kn_b, kn_h, kn_n, kc_b, kc_h, kc_n, vc_b, vc_h, vc_n, vn_b, vn_h, vn_n}
    const DecStrides st{strides[0], strides[1], strides[2], strides[3], strides[4], strides[5],
                        strides[6], strides[7], strides[8], strides[9], strides[10], strides[11]};
    hipLaunchKernelGGL(kv_append_kernel, dim3((unsigned)cdiv(total, (int64_t)256)), dim3(256), 0,
                       (hipStream_t)stream, (const uint16_t*)k_new, (const uint16_t*)v_new,
                       (uint16_t*)k_cache, (uint16_t*)v_cache, batch, n_new, kv_heads, head_dim,
                       capacity, st, pos_dev);
    return launch_status("pli_kv_append");
}

extern "C" size_t pli_attn_decode_workspace_size(int batch, int heads, int kv_heads, int n_q,
                                                 int n_kv, int head_dim) {
    using namespace pli;
    if (batch <= 0 || heads <= 0 || kv_heads <= 0 || heads % kv_heads || n_q <= 0 || n_kv <= 0 ||
        head_dim <= 0)
        return 0;
    const int64_t M = (int64_t)n_q * (heads / kv_heads);
    if (M > DEC_MAXM || !(head_dim == 64 || head_dim == 128)) return 0;
    const int64_t bh = (int64_t)batch * kv_heads;
    const DecPlan p = plan_decode(bh, n_kv);
    if (p.splits == 1) return 0;
    return (size_t)(bh * p.splits * M * ((int64_t)head_dim + 2) * sizeof(float));
}

extern "C" int pli_flash_attn_fwd(const void* q, const void* k, const void* v, void* o, int batch,
                                  int heads, int kv_heads, int n_q, int n_kv, int head_dim,
                                  const int64_t* strides, float scale, int causal, int dtype,
                                  void* stream);

// tuning entry (not in include/pli.h): explicit kernel mode, -1 = default
extern "C" int pli_attn_decode_variant(const void* q, const void* k, const void* v, void* o,
                                       int batch, int heads, int kv_heads, int n_q, int n_kv,
                                       int head_dim, const int64_t* strides, float scale,
                                       int causal, void* workspace, size_t workspace_bytes,
                                       int dtype, void* stream, int mode, int target_wgs) {
    using namespace pli;
    clear_error();
    PLI_REQUIRE(batch >= 0 && heads > 0 && kv_heads > 0 && n_q >= 0 && n_kv >= 0 && head_dim > 0,
                "pli_attn_decode: bad shape B=%d H=%d Hkv=%d Nq=%d Nk=%d D=%d", batch, heads,
                kv_heads, n_q, n_kv, head_dim);
    PLI_REQUIRE(heads % kv_heads == 0, "pli_attn_decode: heads %d not a multiple of kv_heads %d",
                heads, kv_heads);
    PLI_REQUIRE(dtype == PLI_F32 || dtype == PLI_F16 || dtype == PLI_BF16,
                "pli_attn_decode: bad dtype %d", dtype);
    PLI_REQUIRE(std::isfinite(scale), "pli_attn_decode: non-finite scale");
    PLI_REQUIRE(!causal || n_q <= n_kv || n_kv == 0,
                "pli_attn_decode: causal needs n_q (%d) <= n_kv (%d)", n_q, n_kv);
    // empty operands may be NULL (pli.h); an empty cache gives O = 0, written
    // by the prefill path's generic kernel (it reads no K / V)
    if (batch == 0 || n_q == 0) return PLI_OK;
    PLI_REQUIRE(q && o && strides && (n_kv == 0 || (k && v)), "pli_attn_decode: null pointer");
    if (n_kv == 0)
        return pli_flash_attn_fwd(q, k, v, o, batch, heads, kv_heads, n_q, n_kv, head_dim, strides,
                                  scale, causal, dtype, stream);
    const bool fast = decode_fast_path(heads, kv_heads, n_q, n_kv, head_dim, dtype, strides) &&
                      aligned16(q) && aligned16(k) && aligned16(v) && aligned16(o);
    // many query rows per kv head (or shapes the decode tile does not take):
    // the prefill kernel handles GQA and bottom-right causal masking itself
    if (!fast)
        return pli_flash_attn_fwd(q, k, v, o, batch, heads, kv_heads, n_q, n_kv, head_dim, strides,
                                  scale, causal, dtype, stream);
    size_t need = 0;
    {
        const int64_t bh = (int64_t)batch * kv_heads;
        const DecPlan p = plan_decode(bh, n_kv, target_wgs > 0 ? target_wgs : kDefaultTargetWgs);
        if (p.splits > 1)
            need = (size_t)(bh * p.splits * n_q * (heads / kv_heads) * ((int64_t)head_dim + 2) *
                            sizeof(float));
    }
    PLI_REQUIRE(workspace_bytes >= need && (need == 0 || workspace != nullptr),
                "pli_attn_decode: workspace of %zu bytes needed, %zu given", need,
                workspace_bytes);
    PLI_REQUIRE(need == 0 || (reinterpret_cast<uintptr_t>(workspace) & 15) == 0,
                "pli_attn_decode: workspace must be 16-byte aligned");
    const DecStrides st{strides[0], strides[1], strides[2], strides[3], strides[4], strides[5],
                        strides[6], strides[7], strides[8], strides[9], strides[10], strides[11]};
    const int G = heads / kv_heads;
    hipStream_t s = (hipStream_t)stream;
    float* ws = (float*)workspace;
    if (dtype == PLI_BF16)
        return head_dim == 128
                   ? launch_decode<bf16_t, 128>(q, k, v, o, batch, kv_heads, G, n_q, n_kv, st, scale, causal, ws, s, mode, target_wgs)
                   : launch_decode<bf16_t, 64>(q, k, v, o, batch, kv_heads, G, n_q, n_kv, st, scale, causal, ws, s, mode, target_wgs);
    return head_dim == 128
               ? launch_decode<f16_t, 128>(q, k, v, o, batch, kv_heads, G, n_q, n_kv, st, scale, causal, ws, s, mode, target_wgs)
               : launch_decode<f16_t, 64>(q, k, v, o, batch, kv_heads, G, n_q, n_kv, st, scale, causal, ws, s, mode, target_wgs);
}

extern "C" int pli_attn_decode_dev(const void* q, const void* k, const void* v, void* o,
                                   int batch, int heads, int kv_heads, int n_q, int n_kv_max,
                                   int head_dim, const int64_t* strides, float scale, int causal,
                                   const int32_t* n_kv_dev, int n_kv_add, void* workspace,
                                   size_t workspace_bytes, int dtype, void* stream) {
    using namespace pli;
    clear_error();
    PLI_REQUIRE(batch >= 0 && heads > 0 && kv_heads > 0 && n_q >= 0 && n_kv_max >= 0 &&
                    head_dim > 0 && heads % kv_heads == 0,
                "pli_attn_decode_dev: bad shape B=%d H=%d Hkv=%d Nq=%d Nmax=%d D=%d", batch, heads,
                kv_heads, n_q, n_kv_max, head_dim);
    PLI_REQUIRE(std::isfinite(scale), "pli_attn_decode_dev: non-finite scale");
    if (batch == 0 || n_q == 0) return PLI_OK;
    PLI_REQUIRE(q && k && v && o && strides && n_kv_dev, "pli_attn_decode_dev: null pointer");
    if (!(decode_fast_path(heads, kv_heads, n_q, n_kv_max, head_dim, dtype, strides) &&
          aligned16(q) && aligned16(k) && aligned16(v) && aligned16(o))) {
        set_error("pli_attn_decode_dev: needs bf16/fp16, head_dim 64/128, <= 16 rows per kv "
                  "head, 16-byte aligned operands");
        return PLI_EUNSUPPORTED;
    }
    const size_t need =
        pli_attn_decode_workspace_size(batch, heads, kv_heads, n_q, n_kv_max, head_dim);
    PLI_REQUIRE(workspace_bytes >= need && (need == 0 || workspace != nullptr),
                "pli_attn_decode_dev: workspace of %zu bytes needed, %zu given", need,
                workspace_bytes);
    const DecStrides st{strides[0], strides[1], strides[2], strides[3], strides[4], strides[5],
                        strides[6], strides[7], strides[8], strides[9], strides[10], strides[11]};
    const int G = heads / kv_heads;
    hipStream_t s = (hipStream_t)stream;
    float* ws = (float*)workspace;
    if (dtype == PLI_BF16)
        return head_dim == 128
                   ? launch_decode<bf16_t, 128>(q, k, v, o, batch, kv_heads, G, n_q, n_kv_max, st, scale, causal, ws, s, -1, 0, n_kv_dev, n_kv_add)
                   : launch_decode<bf16_t, 64>(q, k, v, o, batch, kv_heads, G, n_q, n_kv_max, st, scale, causal, ws, s, -1, 0, n_kv_dev, n_kv_add);
    return head_dim == 128
               ? launch_decode<f16_t, 128>(q, k, v, o, batch, kv_heads, G, n_q, n_kv_max, st, scale, causal, ws, s, -1, 0, n_kv_dev, n_kv_add)
               : launch_decode<f16_t, 64>(q, k, v, o, batch, kv_heads, G, n_q, n_kv_max, st, scale, causal, ws, s, -1, 0, n_kv_dev, n_kv_add);
}

extern "C" int pli_attn_decode(const void* q, const void* k, const void* v, void* o, int batch,
                               int heads, int kv_heads, int n_q, int n_kv, int head_dim,
                               const int64_t* strides, float scale, int causal, void* workspace,
                               size_t workspace_bytes, int dtype, void* stream) {
    return pli_attn_decode_variant(q, k, v, o, batch, heads, kv_heads, n_q, n_kv, head_dim, strides,
                                   scale, causal, workspace, workspace_bytes, dtype, stream, -1, 0);
}
