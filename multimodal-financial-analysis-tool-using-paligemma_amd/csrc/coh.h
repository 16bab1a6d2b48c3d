// coh.h -- coherent (write-through / L2-bypassing) loads and stores for cross-workgroup hand-offs
// inside one launch (gfx950, 8 XCDs with private L2s): relaxed agent-scope atomic stores and loads,
// no fences (cdna_hip_programming.md sec.6 Guideline 16, form R1).  Used by the lm_head's folded
// argmax: each workgroup publishes its partial write-through, counts its arrival, and the last
// one to arrive reads every partial coherently (no workgroup ever waits on another).
#pragma once
#include "common.h"

namespace pgmi {

__device__ __forceinline__ uint4 ld16_coh(const void* p) {
    const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
    const unsigned long long a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return make_uint4((unsigned)a, (unsigned)(a >> 32), (unsigned)b, (unsigned)(b >> 32));
}
__device__ __forceinline__ float ldf_coh(const float* p) {
    return __uint_as_float(__hip_atomic_load(reinterpret_cast<const unsigned*>(p), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ int ldi_coh(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint16_t ldh_coh(const uint16_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void sth_coh(uint16_t* p, uint16_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void stf_coh(float* p, float v) {
    __hip_atomic_store(reinterpret_cast<unsigned*>(p), __float_as_uint(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void sti_coh(int* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st16_coh(void* p, uint4 v) {
    unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
    __hip_atomic_store(q, (unsigned long long)v.x | ((unsigned long long)v.y << 32), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(q + 1, (unsigned long long)v.z | ((unsigned long long)v.w << 32), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// plain or coherent, chosen at compile time
template <bool C>
__device__ __forceinline__ uint4 ldx16(const uint16_t* p) {
    if constexpr (C) return ld16_coh(p);
    else return ldg16(p);
}
template <bool C>
__device__ __forceinline__ float ldxf(const float* p) {
    if constexpr (C) return ldf_coh(p);
    else return *p;
}
template <bool C>
__device__ __forceinline__ f32x4 ldxf4(const float* p) {
    if constexpr (C) return __builtin_bit_cast(f32x4, ld16_coh(p));
    else return *reinterpret_cast<const f32x4*>(p);
}
template <bool C>
__device__ __forceinline__ uint16_t ldxh(const uint16_t* p) {
    if constexpr (C) return ldh_coh(p);
    else return *p;
}
template <bool C>
__device__ __forceinline__ void stxh(uint16_t* p, uint16_t v) {
    if constexpr (C) sth_coh(p, v);
    else *p = v;
}
template <bool C>
__device__ __forceinline__ void stxf(float* p, float v) {
    if constexpr (C) stf_coh(p, v);
    else *p = v;
}
template <bool C>
__device__ __forceinline__ void stxi(int* p, int v) {
    if constexpr (C) sti_coh(p, v);
    else *p = v;
}

}  // namespace pgmi
