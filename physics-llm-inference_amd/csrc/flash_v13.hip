// attn_fwd_v13: flash-attention forward on v_mfma_f32_16x16x32_bf16
// (reference ch06/flash_attention.py:14-74; gfx950, bf16 / fp16, D = 128 /
// 64, Nk a multiple of 64 and >= 128 or -- attn_fwd_v13r -- any Nk > 64;
// causal -- bottom-right, any Nq <= Nk -- as attn_fwd_v13c / v13rc; other
// cases take v12 / v10).
//
// One wave per SIMD, 64 query rows per wave (4 q-blocks of 16), persistent
// workgroups of 4 waves walking 256-row blocks.  The body is ONE generated
// instruction stream (flash_v13_asm.h from tools/gen_flash_v13.py; the
// layout, schedule and the reasons for them are in tools/v13/kernel.py): the
// 16x16x32 MFMA shape holds a higher clock under load than 32x32x16 (DESIGN
// 3.1), but its 16-cycle gaps leave 8 issue cycles each, so the softmax
// stream, the fragment reads and the LDS-DMA are placed gap by gap, with the
// hazard padding and wait counts computed by the generator (hipcc pads
// nothing inside an asm statement).  tests/test_v13_emu.py runs the same
// program in a CPU emulator; tests/test_gpu_flash_v13.py on the device.
//
// Differences from v12 a caller can see: none in the contract; numerically
// P = bf16(exp2(s c - mu)) with mu = (row max) c + muoff (62 from the
// launcher: P <= 2^-62 when the max is taken, checked < 2 per tile, so a row
// max may grow by 63 log2 units before the rescale path -- v12's THR 64
// rule), l from the same rounded P on the matrix core, 1/l by v_rcp.
#include <cstring>

#include "flash_v7.h"
#ifdef PLI_V13_AB_HEADER  // timing-only A/B builds (tools/build_v13_ab.sh)
#include PLI_V13_AB_HEADER
#else
#include "flash_v13_asm.h"
#endif
#include "pli_common.h"
#include "flash_v13.h"

namespace pli {
namespace {

// (A_SHIFTS packs the three magic-division shifts and the head count:
// shq | shh << 5 | shg << 10 | H << 16 -- the block-parameter dwords 0..36
// then fit s56..s92 and the program keeps off s32 / s100 / s101)
enum : int {
    A_Q = 0, A_K = 2, A_V = 4, A_O = 6, A_QB = 8, A_QH = 10, A_KB = 12, A_KH = 14, A_VB = 16, A_VH = 18,
    A_OB = 20, A_OH = 22, A_QN = 24, A_ON, A_NQ, A_NT, A_QBLOCKS, A_NBLOCKS, A_MAGQ, A_MAGH, A_MAGG, A_SHIFTS,
    A_CW, A_HX, A_G, A_KN, A_VN, A_C, A_MUOFF, A_TBK, A_TBV, A_STAMP, A_STAMP_HI, A_OFFT
};
static_assert(A_G == 36 && A_OFFT == 45, "argument layout (tools/v13/kernel.py ARG_LAYOUT)");

__global__ __launch_bounds__(256, 1) void attn_fwd_v13(V13Args args) {
    __shared__ __attribute__((aligned(1024))) char smem[163840];
    (void)args;
    const void* kp = (const void*)__builtin_amdgcn_kernarg_segment_ptr();
    const unsigned wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const unsigned wg = blockIdx.x;
    asm volatile(PLI_V13_BODY::"s"(kp), "s"(wg), "s"(wave), "s"((unsigned)(uintptr_t)smem) : PLI_V13_CLOBBERS);
}

// causal (bottom-right mask): the same program with the masked step bodies
// and the causal walks (tools/v13/kernel.py Gen(causal=True))
__global__ __launch_bounds__(256, 1) void attn_fwd_v13c(V13Args args) {
    __shared__ __attribute__((aligned(1024))) char smem[163840];
    (void)args;
    const void* kp = (const void*)__builtin_amdgcn_kernarg_segment_ptr();
    const unsigned wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const unsigned wg = blockIdx.x;
    asm volatile(PLI_V13C_BODY::"s"(kp), "s"(wg), "s"(wave), "s"((unsigned)(uintptr_t)smem) : PLI_V13_CLOBBERS);
}

// fp16 Q / K / V / O: the same programs on v_mfma_f32_16x16x32_f16, P packed
// to fp16 (RNE) and checked with the bit-14 test (tools/v13/kernel.py
// Gen(dtype="f16"); the launcher passes mu offset PLI_V13_MUOFF_F16)
__global__ __launch_bounds__(256, 1) void attn_fwd_v13h(V13Args args) {
    __shared__ __attribute__((aligned(1024))) char smem[163840];
    (void)args;
    const void* kp = (const void*)__builtin_amdgcn_kernarg_segment_ptr();
    const unsigned wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const unsigned wg = blockIdx.x;
    asm volatile(PLI_V13H_BODY::"s"(kp), "s"(wg), "s"(wave), "s"((unsigned)(uintptr_t)smem) : PLI_V13_CLOBBERS);
}

__global__ __launch_bounds__(256, 1) void attn_fwd_v13hc(V13Args args) {
    __shared__ __attribute__((aligned(1024))) char smem[163840];
    (void)args;
    const void* kp = (const void*)__builtin_amdgcn_kernarg_segment_ptr();
    const unsigned wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const unsigned wg = blockIdx.x;
    asm volatile(PLI_V13HC_BODY::"s"(kp), "s"(wg), "s"(wave), "s"((unsigned)(uintptr_t)smem) : PLI_V13_CLOBBERS);
}

// Nk % 64 != 0 (non-causal): the last key tile is streamed from key Nk - 64,
// inside the head, and the keys it shares with the tile before get P = 0
// (tools/v13/kernel.py RAGGED; P0 = 64 - Nk % 64 in the cw argument)
__global__ __launch_bounds__(256, 1) void attn_fwd_v13r(V13Args args) {
    __shared__ __attribute__((aligned(1024))) char smem[163840];
    (void)args;
    const void* kp = (const void*)__builtin_amdgcn_kernarg_segment_ptr();
    const unsigned wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const unsigned wg = blockIdx.x;
    asm volatile(PLI_V13R_BODY::"s"(kp), "s"(wg), "s"(wave), "s"((unsigned)(uintptr_t)smem) : PLI_V13_CLOBBERS);
}

__global__ __launch_bounds__(256, 1) void attn_fwd_v13hr(V13Args args) {
    __shared__ __attribute__((aligned(1024))) char smem[163840];
    (void)args;
    const void* kp = (const void*)__builtin_amdgcn_kernarg_segment_ptr();
    const unsigned wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const unsigned wg = blockIdx.x;
    asm volatile(PLI_V13HR_BODY::"s"(kp), "s"(wg), "s"(wave), "s"((unsigned)(uintptr_t)smem) : PLI_V13_CLOBBERS);
}

// causal with Nk % 64 != 0: the shifted last key tile, masked by VALU on its
// shifted keys (tools/v13/kernel.py rag step; P0 in the top byte of hx)
__global__ __launch_bounds__(256, 1) void attn_fwd_v13rc(V13Args args) {
    __shared__ __attribute__((aligned(1024))) char smem[163840];
    (void)args;
    const void* kp = (const void*)__builtin_amdgcn_kernarg_segment_ptr();
    const unsigned wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const unsigned wg = blockIdx.x;
    asm volatile(PLI_V13RC_BODY::"s"(kp), "s"(wg), "s"(wave), "s"((unsigned)(uintptr_t)smem) : PLI_V13_CLOBBERS);
}

__global__ __launch_bounds__(256, 1) void attn_fwd_v13hrc(V13Args args) {
    __shared__ __attribute__((aligned(1024))) char smem[163840];
    (void)args;
    const void* kp = (const void*)__builtin_amdgcn_kernarg_segment_ptr();
    const unsigned wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const unsigned wg = blockIdx.x;
    asm volatile(PLI_V13HRC_BODY::"s"(kp), "s"(wg), "s"(wave), "s"((unsigned)(uintptr_t)smem) : PLI_V13_CLOBBERS);
}

// floor(x / d) == ((x * m) >> 31) >> l for 0 <= x < 2^31 (Granlund-Montgomery,
// N = 31: m = ceil(2^(31+l) / d) < 2^32 with l = ceil(log2 d))
void magic31(uint32_t d, uint32_t& m, uint32_t& l) {
    l = 0;
    while ((1ull << l) < d) ++l;
    const unsigned __int128 num = (unsigned __int128)1 << (31 + l);
    m = (uint32_t)((num + d - 1) / d);
}

void put64(V13Args& a, int at, uint64_t v) {
    a.w[at] = (uint32_t)v;
    a.w[at + 1] = (uint32_t)(v >> 32);
}

#ifdef PLI_FLASH_STAMPS
// diagnostic build only (tools/build_diag.sh): the same program with
// s_memtime / s_memrealtime at each wave's entry and exit (8 dwords per wave
// at args.stamp + 128 * (workgroup * 4 + wave); lanes 15-21: the seam sums of
// tools/v13/kernel.py Gen.seam_stamp)
#include "flash_v13_stamp_asm.h"
int g_diag_grid = 0;  // pli_diag_v13_set_grid: persistent grid override (0: the CU count)
__global__ __launch_bounds__(256, 1) void attn_fwd_v13_stamp(V13Args args) {
    __shared__ __attribute__((aligned(1024))) char smem[163840];
    (void)args;
    const void* kp = (const void*)__builtin_amdgcn_kernarg_segment_ptr();
    const unsigned wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const unsigned wg = blockIdx.x;
    asm volatile(PLI_V13_STAMP_BODY::"s"(kp), "s"(wg), "s"(wave), "s"((unsigned)(uintptr_t)smem) : PLI_V13_CLOBBERS);
}
#endif

}  // namespace

bool attn_v13_ok(int D, int is_bf16, int causal, int Nq, int Nk, const V7Strides& st) {
    (void)is_bf16;  // bf16 and fp16 programs
    // head dim 128, or 64 (the D = 64 bodies in flash_v13_d64.hip); Nk a
    // multiple of 64 from 128, or (non-causal) any Nk > 64: the ragged bodies
    if ((D != 128 && D != 64) || Nq < 1) return false;
    if (Nk % 64 == 0 ? Nk < 128 : Nk <= 64) return false;
    // causal: Nq <= Nk, any diagonal offset -- rows are processed as Nq + s
    // virtual rows, s = (Nk - Nq) & 63, which puts the bottom-right diagonal
    // on 64-key tile boundaries (tools/v13/kernel.py qshift; rows below s are
    // neither loaded nor stored); Nk % 64 != 0 on the ragged causal bodies
    if (causal && Nq > Nk) return false;
    // causal: the stream's tile count and index carry the block's order in
    // bit 16 (tools/v13/kernel.py block_params), so counts stay below 2^16
    if (causal && cdiv(Nk, 64) > 0xFFFF) return false;
    // 32-bit per-lane offsets: a Q / O head's rows, a K / V tile
    const int64_t q_ext = ((int64_t)Nq - 1) * st.qn * 2 + 2 * D, o_ext = ((int64_t)Nq - 1) * st.on * 2 + 2 * D;
    const int64_t kv_tile = 64 * std::max(st.kn, st.vn) * 2;
    if (q_ext >= (1ll << 32) || o_ext >= (1ll << 32) || kv_tile >= (1ll << 31)) return false;
    for (int64_t s : {st.qb, st.qh, st.kb, st.kh, st.vb, st.vh, st.ob, st.oh, st.qn, st.kn, st.vn, st.on})
        if (s < 0) return false;
    return true;
}

bool attn_pp64_ok(int D, bool fp16, bool causal, int Nq, int Nk) {
    (void)fp16;  // bf16 and fp16 bodies
    if (D != 64 || Nk % 64 != 0) return false;
    return !causal || (Nq % 64 == 0 && Nk >= Nq && (Nk - Nq) % 64 == 0);
}

int launch_attn_v13(const void* q, const void* k, const void* v, void* o, int B, int H, int group, int Nq,
                    int Nk, const V7Strides& st, float scale, hipStream_t stream, bool persistent, float muoff,
                    uint32_t* stamps, bool causal, bool fp16, int D, bool pp64) {
    PLI_REQUIRE(attn_v13_ok(D, fp16 ? 0 : 1, causal, Nq, Nk, st), "attn_fwd_v13: shape not supported");
    PLI_REQUIRE(H > 0 && H < (1 << 16), "attn_fwd_v13: H = %d past the packed 16-bit head count", H);
    PLI_REQUIRE(!((fp16 || D != 128 || Nk % 64 != 0 || causal) && stamps),
                "attn_fwd_v13: the stamp build is bf16, D = 128, non-causal, Nk % 64 == 0");
    const int nqv = causal ? Nq + ((Nk - Nq) & 63) : Nq;  // causal: virtual rows, (Nk - nqv) % 64 == 0
    // attn_fwd_pp64: 512-row blocks (8 waves of 64 rows), one per workgroup
    const bool pp = pp64 && !stamps && attn_pp64_ok(D, fp16, causal, Nq, Nk);
    const int qblocks = cdiv(nqv, pp ? 512 : 256);
    const int64_t nb = (int64_t)B * H * qblocks;
    PLI_REQUIRE(nb < (1ll << 31) && nb > 0, "attn_fwd_v13: grid too large");
    int grid = (int)nb;
    // (pp64's persistent walk streams the next block's first four key tiles
    // during the current block: it needs Nk >= 256)
    if (persistent && (!pp || (Nk / 64 >= 4 && !causal))) {
        const int g = cu_count(stream) / 8 * 8;
        if (g >= 8 && nb > g) grid = g;
    }
    // causal walk: the pair walk where it tiles the grid exactly (query
    // heights QB-1-a then a of one head per workgroup step, the QB/2
    // workgroups of a head in step on one XCD; G/8 and QB/2 powers of two),
    // else one block per workgroup, heaviest first
    uint32_t cw = 0, hx = 0;
    if (causal && pp) {
        cw = 2u;  // pp64c: block_params' remap walk, heaviest block first, one per workgroup
    } else if (causal) {
        const int64_t bh = nb / qblocks, w = grid / 8, hq = qblocks / 2;
        auto pw2 = [](int64_t x) { return x > 0 && (x & (x - 1)) == 0; };
        const bool pair = grid < nb && qblocks % 2 == 0 && hq > 0 && w % hq == 0 && bh % 8 == 0 &&
                          (bh / 8) % (w / hq) == 0 && nb % grid == 0 && (nb / grid) % 2 == 0 && pw2(w) && pw2(hq);
        if (pair) {
            uint32_t lg8 = 0, lghq = 0;
            while ((1ll << lg8) < w) ++lg8;
            while ((1ll << lghq) < hq) ++lghq;
            cw = 1u | (lg8 << 8) | (lghq << 16) | ((uint32_t)(w / hq) << 24);
            hx = (uint32_t)(bh / 8);
        } else {
            cw = 2u;
            grid = (int)nb;
        }
    }
    V13Args a;
    std::memset(&a, 0, sizeof(a));
    put64(a, A_Q, (uint64_t)(uintptr_t)q);
    put64(a, A_K, (uint64_t)(uintptr_t)k);
    put64(a, A_V, (uint64_t)(uintptr_t)v);
    put64(a, A_O, (uint64_t)(uintptr_t)o);
    put64(a, A_QB, (uint64_t)st.qb * 2);
    put64(a, A_QH, (uint64_t)st.qh * 2);
    put64(a, A_KB, (uint64_t)st.kb * 2);
    put64(a, A_KH, (uint64_t)st.kh * 2);
    put64(a, A_VB, (uint64_t)st.vb * 2);
    put64(a, A_VH, (uint64_t)st.vh * 2);
    put64(a, A_OB, (uint64_t)st.ob * 2);
    put64(a, A_OH, (uint64_t)st.oh * 2);
    a.w[A_QN] = (uint32_t)(st.qn * 2);
    a.w[A_KN] = (uint32_t)(st.kn * 2);
    a.w[A_VN] = (uint32_t)(st.vn * 2);
    a.w[A_ON] = (uint32_t)(st.on * 2);
    a.w[A_NQ] = (uint32_t)Nq;
    a.w[A_NT] = (uint32_t)cdiv(Nk, 64);
    a.w[A_QBLOCKS] = (uint32_t)qblocks;
    a.w[A_NBLOCKS] = (uint32_t)nb;
    uint32_t shq, shh, shg;
    magic31((uint32_t)qblocks, a.w[A_MAGQ], shq);
    magic31((uint32_t)H, a.w[A_MAGH], shh);
    magic31((uint32_t)group, a.w[A_MAGG], shg);
    a.w[A_SHIFTS] = shq | (shh << 5) | (shg << 10) | ((uint32_t)H << 16);
    // ragged Nk: P0 = 64 - Nk % 64 in cw (non-causal: the walk word is free)
    // or in the top byte of hx (causal: the pair walk uses cw, hx < 2^24)
    const bool ragged = Nk % 64 != 0;
    const uint32_t p0 = ragged ? (uint32_t)(64 - Nk % 64) : 0u;
    PLI_REQUIRE(hx < (1u << 24), "attn_fwd_v13: %u heads per XCD past the 24-bit walk field", hx);
    a.w[A_CW] = ragged && !causal ? p0 : cw;
    a.w[A_HX] = causal ? hx | (p0 << 24) : hx;
    a.w[A_OFFT] = causal ? (uint32_t)((Nk - nqv) / 64) : 0u;
    const float c = scale * 1.4426950408889634f;
    std::memcpy(&a.w[A_C], &c, 4);
    std::memcpy(&a.w[A_MUOFF], &muoff, 4);
    a.w[A_G] = (uint32_t)grid;
    a.w[A_TBK] = (uint32_t)(64 * st.kn * 2);
    a.w[A_TBV] = (uint32_t)(64 * st.vn * 2);
#ifdef PLI_FLASH_STAMPS
    if (stamps) {
        // diagnostic: a smaller persistent grid (a multiple of 8) when asked
        if (g_diag_grid >= 8 && g_diag_grid % 8 == 0 && g_diag_grid < grid) {
            grid = g_diag_grid;
            a.w[A_G] = (uint32_t)grid;
        }
        put64(a, A_STAMP, (uint64_t)(uintptr_t)stamps);
        hipLaunchKernelGGL(attn_fwd_v13_stamp, dim3((unsigned)grid), dim3(256), 0, stream, a);
        return launch_status("attn_fwd_v13_stamp");
    }
#else
    (void)stamps;
#endif
    if (pp) return launch_pp64(fp16, causal, (unsigned)grid, a, stream);
    if (D == 64) return launch_v13_d64(fp16, causal, ragged, (unsigned)grid, a, stream);
    if (ragged && causal) {
        if (fp16) {
            hipLaunchKernelGGL(attn_fwd_v13hrc, dim3((unsigned)grid), dim3(256), 0, stream, a);
            return launch_status("attn_fwd_v13hrc");
        }
        hipLaunchKernelGGL(attn_fwd_v13rc, dim3((unsigned)grid), dim3(256), 0, stream, a);
        return launch_status("attn_fwd_v13rc");
    }
    if (ragged) {
        if (fp16) {
            hipLaunchKernelGGL(attn_fwd_v13hr, dim3((unsigned)grid), dim3(256), 0, stream, a);
            return launch_status("attn_fwd_v13hr");
        }
        hipLaunchKernelGGL(attn_fwd_v13r, dim3((unsigned)grid), dim3(256), 0, stream, a);
        return launch_status("attn_fwd_v13r");
    }
    if (fp16) {
        if (causal) {
            hipLaunchKernelGGL(attn_fwd_v13hc, dim3((unsigned)grid), dim3(256), 0, stream, a);
            return launch_status("attn_fwd_v13hc");
        }
        hipLaunchKernelGGL(attn_fwd_v13h, dim3((unsigned)grid), dim3(256), 0, stream, a);
        return launch_status("attn_fwd_v13h");
    }
    if (causal) {
        hipLaunchKernelGGL(attn_fwd_v13c, dim3((unsigned)grid), dim3(256), 0, stream, a);
        return launch_status("attn_fwd_v13c");
    }
    hipLaunchKernelGGL(attn_fwd_v13, dim3((unsigned)grid), dim3(256), 0, stream, a);
    return launch_status("attn_fwd_v13");
}

}  // namespace pli

#ifdef PLI_FLASH_STAMPS
// Diagnostic entry (tools/libpli_diag.so only): one clock-stamped launch of
// attn_fwd_v13 (persistent) on contiguous [B,H,N,128] bf16; stamps: 8 dwords
// per wave (entry s_memtime lo/hi, s_memrealtime lo/hi, then the exit ones)
extern "C" int pli_diag_v13_clock(const void* q, const void* k, const void* v, void* o, int B, int H, int N,
                                  uint32_t* stamps) {
    using namespace pli;
    const int64_t sn = 128, sh = (int64_t)N * 128, sb = (int64_t)H * N * 128;
    const V7Strides st{sb, sh, sn, sb, sh, sn, sb, sh, sn, sb, sh, sn};
    const int rc = launch_attn_v13(q, k, v, o, B, H, 1, N, N, st, 1.f / sqrtf(128.f), 0, true, 62.f, stamps, false,
                                   false, 128);
    if (rc != 0 || hipDeviceSynchronize() != hipSuccess) return -1;
    return 0;
}
// the stamped launches' persistent grid (a multiple of 8 below the CU count;
// 0 = the product's): the seam's cost against how many CUs seam together
extern "C" void pli_diag_v13_set_grid(int grid) { pli::g_diag_grid = grid; }
#endif
