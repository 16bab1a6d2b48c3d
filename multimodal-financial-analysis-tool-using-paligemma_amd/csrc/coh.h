// coh.h -- in-launch hand-off primitives for the fused decode step (gfx950, 8 XCDs with private L2s).
//
// Protocol (cdna_hip_programming.md sec.6 Guideline 16, form R1):
//   * every handed-off byte is STORED write-through (sc1: relaxed agent-scope atomic stores) and
//     LOADED with sc1 loads (relaxed agent-scope atomic loads), so no acquire/release fences;
//   * a producer workgroup drains its stores (s_waitcnt vmcnt(0) in EVERY wave), meets at a
//     barrier, then one lane adds 1 to the phase counter (relaxed, agent scope);
//   * a consumer workgroup has one lane poll the counter (relaxed, with s_sleep) until it reaches
//     the producer count, then a barrier releases the other waves.
// Deadlock freedom: a workgroup only ever waits on counters fed by workgroups with LOWER ids,
// which the in-order dispatcher has already placed; the lowest unfinished workgroup therefore
// always has its inputs.  Every spin is bounded: on timeout the error word is set and the
// workgroup proceeds (wrong result, never a hang).
#pragma once
#include "common.h"

namespace pgmi {

struct Dep {
    const unsigned* wait = nullptr;  // counter to wait on (nullptr: none)
    unsigned target = 0;             // ... until it reaches this value
    unsigned* arrive = nullptr;      // counter to add 1 to when the workgroup's outputs are out
    // two-level arrival (many producers): add to arrive_shard; the workgroup completing its
    // shard (shard_n arrivals) adds 1 to `arrive` -- one word sees few atomics
    unsigned* arrive_shard = nullptr;
    unsigned shard_n = 0;
    unsigned* err = nullptr;         // sticky error word (spin timeout)
    long long* trace = nullptr;      // optional [4] timestamps of this workgroup: entry, ready, done
};

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

constexpr unsigned kSpinLimit = 1u << 16;  // polls (each >= ~0.1 us): a stuck phase gives up in ~10-60 ms
constexpr unsigned kErrSpin = 1u;

// Whole workgroup: returns when *d.wait >= d.target (or on timeout, flagging d.err).
__device__ __forceinline__ void dep_wait(const Dep& d) {
    if (d.wait) {
        if (threadIdx.x == 0) {
            unsigned spins = 0;
            while (__hip_atomic_load(d.wait, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < d.target) {
                __builtin_amdgcn_s_sleep(4);
                // give up on timeout, or at once when another workgroup already timed out
                if (++spins > kSpinLimit ||
                    (d.err && (spins & 63) == 0 &&
                     __hip_atomic_load(d.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)) {
                    if (d.err) __hip_atomic_fetch_or(d.err, kErrSpin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
            }
        }
        if (d.trace && threadIdx.x == 0) d.trace[1] = __builtin_amdgcn_s_memrealtime();
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler barrier: no load hoisting
    }
}

// Whole workgroup, after its last hand-off store: drain, meet, count.
__device__ __forceinline__ void dep_arrive(const Dep& d) {
    if (d.arrive) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            if (!d.arrive_shard ||
                __hip_atomic_fetch_add(d.arrive_shard, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1 == d.shard_n)
                __hip_atomic_fetch_add(d.arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (d.trace) d.trace[2] = __builtin_amdgcn_s_memrealtime();
        }
    }
}

}  // namespace pgmi
