// kernels_fused.hip -- decode attention with its flash-decoding combine in the same launch (B >= 3).
//
// (Round 4 also built and measured the B <= 2 attention + o_proj as one launch -- chunk workgroups
// publishing write-through and counting, o_proj workgroups of the same grid waiting on the count: B = 1
// step 1.059 -> 1.121 ms, slower than the two launches, and removed)
#include <cstdlib>

#include "attn_decode_body.h"
#include "gemv_body.h"

namespace pgmi {

// ---------------------------------------------------------------- B >= 3: attention + its combine
// Flash-decoding chunks as k_attn_decode, each publishing its record write-through and counting on its
// row's counter; the chunk that arrives last for row b combines the row's records (coherent loads, the
// fixed chunk order of k_attn_combine) and writes o[b] -- the k_attn_combine launch disappears, no
// workgroup waits.  The last arriver re-arms the counter for the next step.
__device__ __forceinline__ void attn_combine_row(const float* __restrict__ part, int max_chunks, int nch, int b,
                                                 int K, uint16_t* __restrict__ o) {
    for (int e8 = threadIdx.x; e8 < K / 8; e8 += blockDim.x) {
        const int e = e8 * 8, h = e >> 8;
        const float* pb = part + (long)b * max_chunks * kAttnPartStride + h * 256 + (e & 255);
        const float* sp = part + (long)b * max_chunks * kAttnPartStride + 16 * 256 + h;
        float M = -INFINITY, S = 0.f, acc[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = 0.f;
        for (int c = 0; c < nch; ++c) M = fmaxf(M, ldf_coh(sp + (long)c * kAttnPartStride));
        for (int c = 0; c < nch; ++c) {
            const float w = expf(ldf_coh(sp + (long)c * kAttnPartStride) - M);
            S += w * ldf_coh(sp + (long)c * kAttnPartStride + 16);
            const f32x4 x0 = __builtin_bit_cast(f32x4, ld16_coh(pb + (long)c * kAttnPartStride));
            const f32x4 x1 = __builtin_bit_cast(f32x4, ld16_coh(pb + (long)c * kAttnPartStride + 4));
#pragma unroll
            for (int j = 0; j < 4; ++j) { acc[j] += w * x0[j]; acc[4 + j] += w * x1[j]; }
        }
        u16x8 ob;
#pragma unroll
        for (int j = 0; j < 8; ++j) ob.v[j] = f2bf(acc[j] / S);
        *reinterpret_cast<u16x8*>(o + (long)b * K + e) = ob;
    }
}

__global__ void __launch_bounds__(256) k_attn_decode_comb(AttnArgs a, const StepState* st, float* __restrict__ part,
                                                          int max_chunks, unsigned* __restrict__ cnt) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[kAttnDecodeLds];
    __shared__ int last;
    const int b = blockIdx.z;
    const int nch = (st->kv_len + 1 + kAttnChunk - 1) / kAttnChunk;
    if ((int)blockIdx.x >= nch) return;  // (attn_decode_block returns there too, before counting)
    unsigned* c = cnt + (long)b * 32;
    attn_decode_block<true>(a, st, part, max_chunks, blockIdx.x, blockIdx.y, b, lds);
    if (threadIdx.x == 0)
        last = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1 == (unsigned)nch;
    __syncthreads();
    if (!last) return;
    attn_combine_row(part, max_chunks, nch, b, a.G * 256, a.o);  // o row b at a.o + b * K (o_b_stride == K)
    if (threadIdx.x == 0) __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// measured slower than its own combine launch (B = 8 step 1.5585 / 1.5572 -> 1.5832 / 1.5803 ms, same
// box): off unless PGMI_FUSED_COMB=1 (kept for A/Bs; tests/test_gpu_full_batch.py runs it)
bool attn_comb_fused(int B) {
    static const bool on = [] { const char* e = getenv("PGMI_FUSED_COMB"); return e && atoi(e) != 0; }();
    return on && B >= 3;
}

void attention_decode_comb(hipStream_t s, const AttnArgs& a, const StepState* st, int launch_keys, float* part,
                           int max_chunks, unsigned* cnt) {
    int nch = (launch_keys + kAttnChunk - 1) / kAttnChunk;
    if (nch > max_chunks) nch = max_chunks;
    hipLaunchKernelGGL(k_attn_decode_comb, dim3(nch, a.n_kv, a.B), dim3(256), 0, s, a, st, part, max_chunks, cnt);
}

}  // namespace pgmi
