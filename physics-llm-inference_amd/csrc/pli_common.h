// Shared helpers for the gfx950 kernels of libpli_hip.so.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <cstring>

#include "pli.h"

namespace pli {

// ---------------------------------------------------------------- errors --
void set_error(const char* fmt, ...);
void clear_error();

#define PLI_REQUIRE(cond, ...)                  \
    do {                                        \
        if (!(cond)) {                          \
            ::pli::set_error(__VA_ARGS__);      \
            return PLI_EINVAL;                  \
        }                                       \
    } while (0)

// Check the launch that was just enqueued.
int launch_status(const char* what);
// Compute units of the device `stream` runs on (cached per device id).
int cu_count(hipStream_t stream);

// ------------------------------------------------------------ vector types --
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(8))) short i16x8;
typedef __attribute__((ext_vector_type(4))) short i16x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) int i32x4;
typedef __attribute__((ext_vector_type(2))) int i32x2;

// Storage tags: kernels move raw 16-bit words and convert at the edges.
struct bf16_t { uint16_t bits; };
struct f16_t { uint16_t bits; };

template <typename T> struct elem;
template <> struct elem<float> {
    static constexpr int bytes = 4;
    __device__ __forceinline__ static float to_f32(float x) { return x; }
    __device__ __forceinline__ static float from_f32(float x) { return x; }
};
template <> struct elem<bf16_t> {
    static constexpr int bytes = 2;
    __device__ __forceinline__ static float to_f32(bf16_t x) {
        return __uint_as_float(uint32_t(x.bits) << 16);
    }
    __device__ __forceinline__ static bf16_t from_f32(float x) {
        __bf16 b = (__bf16)x;  // v_cvt_pk_bf16_f32: RNE, NaN-preserving
        return bf16_t{__builtin_bit_cast(uint16_t, b)};
    }
};
template <> struct elem<f16_t> {
    static constexpr int bytes = 2;
    __device__ __forceinline__ static float to_f32(f16_t x) {
        return (float)__builtin_bit_cast(_Float16, x.bits);
    }
    __device__ __forceinline__ static f16_t from_f32(float x) {
        return f16_t{__builtin_bit_cast(uint16_t, (_Float16)x)};
    }
};

// Pack two fp32 into one dword of two 16-bit values of T (lo in bits 0..15).
template <typename T> __device__ __forceinline__ uint32_t pack2(float lo, float hi);
template <> __device__ __forceinline__ uint32_t pack2<bf16_t>(float lo, float hi) {
    typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
    bf16x2 v = {(__bf16)lo, (__bf16)hi};
    return __builtin_bit_cast(uint32_t, v);
}
template <> __device__ __forceinline__ uint32_t pack2<f16_t>(float lo, float hi) {
    typedef __attribute__((ext_vector_type(2))) _Float16 f16x2;
    f16x2 v = {(_Float16)lo, (_Float16)hi};
    return __builtin_bit_cast(uint32_t, v);
}

// acc + lo + hi of a packed pair of T (v_dot2c against {1,1}): sums the
// values exactly as rounded into the pair.
template <typename T> __device__ __forceinline__ float add_pair(uint32_t p, float acc);
template <> __device__ __forceinline__ float add_pair<bf16_t>(uint32_t p, float acc) {
    typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
    const bf16x2 one = {(__bf16)1.0f, (__bf16)1.0f};
    return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, p), one, acc, false);
}
template <> __device__ __forceinline__ float add_pair<f16_t>(uint32_t p, float acc) {
    typedef __attribute__((ext_vector_type(2))) _Float16 f16x2;
    const f16x2 one = {(_Float16)1.0f, (_Float16)1.0f};
    return __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2, p), one, acc, false);
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// ------------------------------------------------------------- MFMA glue --
// D(32x32,f32) += A(32x16) * B(16x32) for 16-bit inputs held as raw words.
template <typename T>
__device__ __forceinline__ f32x16 mfma32x32x16(i32x4 a, i32x4 b, f32x16 c);
template <>
__device__ __forceinline__ f32x16 mfma32x32x16<bf16_t>(i32x4 a, i32x4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
template <>
__device__ __forceinline__ f32x16 mfma32x32x16<f16_t>(i32x4 a, i32x4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

// D(16x16,f32) += A(16x32) * B(32x16): lane l holds A[l&15][8(l>>4)+j],
// B[8(l>>4)+j][l&15]; D col = l&15, row = 4(l>>4) + reg.
template <typename T>
__device__ __forceinline__ f32x4 mfma16x16x32(i32x4 a, i32x4 b, f32x4 c);
template <>
__device__ __forceinline__ f32x4 mfma16x16x32<bf16_t>(i32x4 a, i32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
template <>
__device__ __forceinline__ f32x4 mfma16x16x32<f16_t>(i32x4 a, i32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

// ------------------------------------------------------------ LDS access --
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ i32x4 lds_read_b128(const char* base, int byte_off) {
    return *reinterpret_cast<const i32x4*>(base + byte_off);
}
__device__ __forceinline__ void lds_write_b128(char* base, int byte_off, i32x4 v) {
    *reinterpret_cast<i32x4*>(base + byte_off) = v;
}
// gfx950 ds_read_b64_tr_b16: per 16-lane group, lane 4q+p addresses row q,
// columns 4p..4p+3 of a 4x16 block of 16-bit values; lane i receives column i.
__device__ __forceinline__ i32x2 lds_read_tr16(const char* base, int byte_off) {
    typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
    i16x4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_i16x4*)(base + byte_off));
    return __builtin_bit_cast(i32x2, r);
}

// max3 without the IEEE-mode canonicalising v_max_f32 that hipcc puts in
// front of fmaxf on MFMA results (values here are finite or -inf, never NaN).
__device__ __forceinline__ float max3(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// ------------------------------------------------------- wave reductions --
__device__ __forceinline__ float wave_max(float x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = fmaxf(x, __shfl_xor(x, o, 64));
    return x;
}
__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

__host__ __device__ constexpr int cdiv(int a, int b) { return (a + b - 1) / b; }

// XCD-aware remap (bijective for any grid): blocks b and b+8 share an XCD
// under the observed round-robin dispatch, so give each XCD a contiguous
// range of logical tiles.  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
    constexpr int NX = 8;
    if (nblocks < NX) return bid;
    const int q = nblocks / NX, r = nblocks % NX;
    const int x = bid % NX, i = bid / NX;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

}  // namespace pli
