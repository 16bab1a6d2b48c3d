// common.h -- shared device helpers for libpgmi (gfx950 / CDNA4 only).
//
// bf16 is carried as raw uint16 bit patterns; all arithmetic is fp32 with an
// explicit round-to-nearest-even back to bf16 exactly where the reference's bf16
// PyTorch modules round ("rounding points").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pgmi {

typedef uint16_t bf16_t;
typedef short short8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

struct alignas(16) u16x8 { uint16_t v[8]; };

__device__ __forceinline__ float bf2f(uint16_t b) {
    return __uint_as_float(((uint32_t)b) << 16);
}

// round-to-nearest-even f32 -> bf16: one v_cvt_pk_bf16_f32 on gfx950 (the integer form
// u + 0x7FFF + ((u >> 16) & 1) took four VALU ops per element; same result for finite inputs, and a
// NaN stays a NaN -- MI355X_MICROARCH.md, correctness boundaries)
__device__ __forceinline__ uint16_t f2bf(float f) {
    return __builtin_bit_cast(uint16_t, (__bf16)f);
}

__device__ __forceinline__ float rbf(float f) { return bf2f(f2bf(f)); }

// gelu(approximate="tanh") in fp32 (torch: 0.5*x*(1+tanh(sqrt(2/pi)*(x+0.044715*x^3)))), as the
// identity 0.5*(1+tanh(u)) = 1/(1+exp(-2u)): one v_exp_f32 and one v_rcp_f32 (a few fp32 ulp, far
// below the bf16 rounding that follows every use) instead of the library tanhf, whose branches and
// division made the GELU epilogues of the fc1 / gate|up GEMMs cost up to a third of the kernel.
// exp(-2u) overflowing to +inf gives x * 0 = -0 (gelu of a large negative x).
__device__ __forceinline__ float gelu_tanh(float x) {
    const float k = 0.7978845608028654f;
    const float u = k * (x + 0.044715f * x * x * x);
    const float e = __builtin_amdgcn_exp2f(u * -2.8853900817779268f);  // exp(-2u) = 2^(-2u log2 e)
    return x * __builtin_amdgcn_rcpf(1.0f + e);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// 8 bf16 (16 B) dot 8 bf16 with fp32 accumulation via v_dot2_f32_bf16
__device__ __forceinline__ float dot8(const uint4 a, const uint4 b, float acc) {
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, a.x), __builtin_bit_cast(bf16x2, b.x), acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, a.y), __builtin_bit_cast(bf16x2, b.y), acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, a.z), __builtin_bit_cast(bf16x2, b.z), acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, a.w), __builtin_bit_cast(bf16x2, b.w), acc, false);
    return acc;
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 ldg_nt(const void* p) {
    u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ uint4 ldg16(const void* p) {
    return *reinterpret_cast<const uint4*>(p);
}

// 16-B load whose lane may be out of range: the load is ALWAYS issued (from `safe` when !ok) and
// the value zeroed afterwards -- a conditional load (ok ? load : 0) makes hipcc branch around the
// load and wait vmcnt(0) for it, one dependent round trip per element (cdna_hip_programming.md
// sec.5 "Projection GEMM at M = 256", trap (c))
__device__ __forceinline__ uint4 ldg16_sel(const void* p, bool ok, const void* safe) {
    const uint4 v = *reinterpret_cast<const uint4*>(ok ? p : safe);
    return ok ? v : make_uint4(0, 0, 0, 0);
}

__device__ __forceinline__ f32x4 mfma16(const short8 a, const short8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

}  // namespace pgmi
