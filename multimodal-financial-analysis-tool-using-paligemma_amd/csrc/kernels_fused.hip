// kernels_fused.hip -- the decode step's attention and o_proj as ONE launch (B <= 2, the v_dot2 path).
//
// Separately, GemmaAttention's flash-decoding chunks (k_attn_decode, 5-9 workgroups) and the o_proj
// GEMV with the chunk combine in its prologue (gemv_body.h GV_ORES, 256 workgroups) are two
// latency-bound launches (≈5.9 + 5.3 µs, 8 MB of weights between them).  Here the chunk workgroups
// come first in the grid and the o_proj workgroups after them:
//   - a chunk workgroup runs attn_decode_block, publishes its partial record write-through and counts
//     its arrival on the layer's counter once its stores have drained (coh.h protocol);
//   - an o_proj workgroup issues its weight stream first, then waits (one lane, s_sleep, bounded) for
//     nch x B arrivals, reads the records coherently, combines and multiplies.
// The chunk workgroups never wait and have the lowest workgroup ids, so they are dispatched before
// any o_proj workgroup on every XCD: no residency assumption, no deadlock.  The counter is zeroed by
// the layer's q|k|v launch (stream-ordered before this one).  The arithmetic is the two-launch form's.
#include <cstdlib>

#include "attn_decode_body.h"
#include "gemv_body.h"

namespace pgmi {

template <int B>
__global__ void __launch_bounds__(256) k_attn_ores(AttnArgs a, GemvArgs g, float* __restrict__ part, int max_chunks,
                                                   int nchg) {
    extern __shared__ __attribute__((aligned(16))) uint16_t xs[];  // o_proj: the combined rows [B][K]
    __shared__ __attribute__((aligned(16))) unsigned char lds[kAttnDecodeLds];
    const int n_attn = nchg * B;
    const int bx = blockIdx.x;
    if (bx < n_attn) {
        attn_decode_block<true>(a, g.st, part, max_chunks, bx % nchg, 0, bx / nchg, lds, g.arrive);
        return;
    }
    gemv_block<B, 4, 2, GV_ORES, 1, false, 1, false, true>(g, bx - n_attn, (int)gridDim.x - n_attn, xs);
}

bool attn_ores_fused(int B) {
    static const bool off = [] { const char* e = getenv("PGMI_FUSED_ATTN"); return e && atoi(e) == 0; }();
    return !off && B <= 2;
}

void attn_ores(hipStream_t s, int B, const AttnArgs& a, const StepState* st, int launch_keys, float* part,
               int max_chunks, const uint16_t* Wo, int N, uint16_t* h_inout, unsigned* arrive) {
    int nch = (launch_keys + kAttnChunk - 1) / kAttnChunk;
    if (nch > max_chunks) nch = max_chunks;
    GemvArgs g{};
    g.x = nullptr; g.norm_w = nullptr; g.W = Wo; g.n_units = N; g.K = a.G * 256; g.nb = B; g.out = h_inout;
    g.part = part; g.max_chunks = max_chunks; g.G = a.G; g.st = st; g.o_out = nullptr; g.arrive = arrive;
    constexpr int per_block = 4 * 2;  // 4 unit groups x 2 rows (the two-launch form's o_proj grid)
    const int oblocks = (N + per_block - 1) / per_block;
    const size_t lds = (size_t)B * g.K * sizeof(uint16_t);
    if (B <= 1)
        hipLaunchKernelGGL(k_attn_ores<1>, dim3(nch * 1 + oblocks), dim3(256), lds, s, a, g, part, max_chunks, nch);
    else
        hipLaunchKernelGGL(k_attn_ores<2>, dim3(nch * 2 + oblocks), dim3(256), lds, s, a, g, part, max_chunks, nch);
}

}  // namespace pgmi
