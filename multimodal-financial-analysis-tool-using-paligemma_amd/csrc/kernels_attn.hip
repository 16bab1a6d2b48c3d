// kernels_attn.hip -- non-causal attention for SigLIP (MHA, d=72) and Gemma (MQA, d=256).
//
// Reference semantics (rounding points kept):
//   SiglipAttention   modeling_siglip.py:116-131:  s = bf16(bf16(q.k) * d^-1/2); p = bf16(softmax_f32(s));
//                                                  o = bf16(p.v)
//   GemmaAttention    modeling_gemma.py:262-277:   s = bf16(bf16(q.k) / 16) (+ zero mask, :269);
//                                                  repeat_kv is never materialised: the G query heads of
//                                                  a KV head are rows of one MFMA tile sharing its K/V.
// The softmax is the exact two-pass one (global max and sum before any p is rounded), so p
// rounds to bf16 exactly where the reference rounds it.
//
// Prefill (k_attn_full): one workgroup = 16 query rows x all keys; QK^T on MFMA straight from
// global (both operands K-contiguous), scores in LDS (fp32), P in LDS (bf16), V staged
// transposed in LDS 32 keys at a time for the PV MFMA.
// Decode (Lq = 1): keys split over 64-key chunks across workgroups (flash-decoding), in three
// short kernels: scores -> (global max/sum, P, partial P.V) -> fixed-order combine.
#include "common.h"
#include "launch.h"

namespace pgmi {

constexpr int VTS = 40;  // transposed-V LDS row stride (elements)

template <int HD>
struct HDInfo {
    static constexpr int KS = (HD + 31) / 32;   // 32-deep k-steps for QK^T
    static constexpr int CT = (HD + 15) / 16;   // 16-wide output column tiles for PV
    static constexpr int CH = (HD + 7) / 8;     // 16-B chunks per head row
};

// load the 16-row A (or B) fragment: lane -> row (lane&15), k = 32*kk + 8*(lane>>4)
template <int HD>
__device__ __forceinline__ short8 load_frag(const uint16_t* rowp, bool valid, int kk, int lane) {
    const int k = 32 * kk + 8 * (lane >> 4);
    if (!valid || k >= HD) return short8{0, 0, 0, 0, 0, 0, 0, 0};
    return __builtin_bit_cast(short8, ldg16(rowp + k));
}

template <int HD>
__global__ void __launch_bounds__(256) k_attn_full(AttnArgs a) {
    using I = HDInfo<HD>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int LkP = (a.Lk + 31) & ~31;
    float* S = reinterpret_cast<float*>(smem_raw);                       // [16][LkP]
    uint16_t* P = reinterpret_cast<uint16_t*>(S + 16 * LkP);             // [16][LkP]
    uint16_t* VT = P + 16 * LkP;                                         // [CT*16][VTS]

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b = blockIdx.z, kvh = blockIdx.y;
    const int row0 = blockIdx.x * 16;
    const int nrows = a.Lq * a.G;

    // ---- phase 1: S = bf16(bf16(Q K^T) * scale)
    const int qi = row0 + (lane & 15);
    const bool qvalid = qi < nrows;
    const int qpos = qvalid ? qi / a.G : 0, qhead = kvh * a.G + (qvalid ? qi % a.G : 0);
    const uint16_t* qrow = a.q + b * a.q_b_stride + (long)qpos * a.q_row_stride + qhead * a.q_head_stride;
    short8 qf[I::KS];
#pragma unroll
    for (int kk = 0; kk < I::KS; ++kk) qf[kk] = load_frag<HD>(qrow, qvalid, kk, lane);

    const uint16_t* kbase = a.k + b * a.k_b_stride + kvh * a.k_head_stride;
    const int ntile = LkP / 16;
    for (int t = wave; t < ntile; t += 4) {
        const int key = t * 16 + (lane & 15);
        const bool kvalid = key < a.Lk;
        const uint16_t* krow = kbase + (long)key * a.k_row_stride;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < I::KS; ++kk) acc = mfma16(qf[kk], load_frag<HD>(krow, kvalid, kk, lane), acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = (lane >> 4) * 4 + r;
            S[row * LkP + key] = kvalid ? rbf(rbf(acc[r]) * a.scale) : -INFINITY;
        }
    }
    __syncthreads();

    // ---- phase 2: exact softmax per row (fp32), P = bf16(p)
    for (int row = wave; row < 16; row += 4) {
        float m = -INFINITY;
        for (int t = lane; t < a.Lk; t += 64) m = fmaxf(m, S[row * LkP + t]);
        m = wave_max(m);
        float sum = 0.f;
        for (int t = lane; t < a.Lk; t += 64) {
            const float e = expf(S[row * LkP + t] - m);
            S[row * LkP + t] = e;
            sum += e;
        }
        sum = wave_sum(sum);
        for (int t = lane; t < LkP; t += 64) P[row * LkP + t] = t < a.Lk ? f2bf(S[row * LkP + t] / sum) : 0;
    }
    __syncthreads();

    // ---- phase 3: O = bf16(P V), V staged transposed 32 keys at a time
    const uint16_t* vbase = a.v + b * a.v_b_stride + kvh * a.v_head_stride;
    f32x4 oacc[(I::CT + 3) / 4];
#pragma unroll
    for (int c = 0; c < (I::CT + 3) / 4; ++c) oacc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int t0 = 0; t0 < LkP; t0 += 32) {
        for (int e = tid; e < 32 * I::CH; e += 256) {
            const int tt = e / I::CH, ch = e % I::CH;
            const int key = t0 + tt;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (key < a.Lk) v = ldg16(vbase + (long)key * a.v_row_stride + ch * 8);
            const uint16_t* ve = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
            for (int j = 0; j < 8; ++j) VT[(ch * 8 + j) * VTS + tt] = ve[j];
        }
        if constexpr ((HD % 16) != 0) {  // zero the pad columns of the last tile
            for (int e = tid; e < (I::CT * 16 - I::CH * 8) * 32; e += 256) {
                VT[(I::CH * 8 + e / 32) * VTS + (e % 32)] = 0;
            }
        }
        __syncthreads();
        const short8 pa = *reinterpret_cast<const short8*>(P + (lane & 15) * LkP + t0 + 8 * (lane >> 4));
#pragma unroll
        for (int c = 0; c < (I::CT + 3) / 4; ++c) {
            const int ct = wave + 4 * c;
            if (ct < I::CT) {
                const short8 vb = *reinterpret_cast<const short8*>(VT + (ct * 16 + (lane & 15)) * VTS + 8 * (lane >> 4));
                oacc[c] = mfma16(pa, vb, oacc[c]);
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int c = 0; c < (I::CT + 3) / 4; ++c) {
        const int ct = wave + 4 * c;
        if (ct >= I::CT) continue;
        const int d = ct * 16 + (lane & 15);
        if (d >= HD) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = row0 + (lane >> 4) * 4 + r;
            if (i >= nrows) continue;
            const int pos = i / a.G, head = kvh * a.G + i % a.G;
            a.o[b * a.o_b_stride + (long)pos * a.o_row_stride + head * a.o_head_stride + d] = f2bf(oacc[c][r]);
        }
    }
}

static size_t attn_full_lds(int head_dim, int Lk) {
    const int LkP = (Lk + 31) & ~31;
    const int ct = (head_dim + 15) / 16;
    return (size_t)16 * LkP * 4 + (size_t)16 * LkP * 2 + (size_t)ct * 16 * VTS * 2;
}

void attention_prefill(hipStream_t s, int head_dim, const AttnArgs& a) {
    const size_t lds = attn_full_lds(head_dim, a.Lk);
    dim3 grid((a.Lq * a.G + 15) / 16, a.n_kv, a.B);
    if (head_dim == 256) {
        static bool attr = false;
        if (!attr) {
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_attn_full<256>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            attr = true;
        }
        hipLaunchKernelGGL(k_attn_full<256>, grid, dim3(256), lds, s, a);
    } else {
        static bool attr = false;
        if (!attr) {
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_attn_full<72>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            attr = true;
        }
        hipLaunchKernelGGL(k_attn_full<72>, grid, dim3(256), lds, s, a);
    }
}

int attention_prefill_max_keys(int head_dim) {
    const int ct = (head_dim + 15) / 16;
    return (int)((160 * 1024 - (size_t)ct * 16 * VTS * 2) / (16 * 6)) & ~31;
}

// ================================================================ decode (Lq = 1)
constexpr int DCH = 64;  // keys per chunk

// scores[b][kvh][row][t] for t in this chunk; rows = the G heads (<= 16)
__global__ void __launch_bounds__(256) k_attn_dec_scores(AttnArgs a, const StepState* st, int max_keys,
                                                          float* __restrict__ scores) {
    using I = HDInfo<256>;
    const int Lk = st->kv_len + 1;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int b = blockIdx.z, kvh = blockIdx.y;
    const int t0 = blockIdx.x * DCH + wave * 16;
    if (blockIdx.x * DCH >= Lk) return;
    const int qi = lane & 15;
    const bool qvalid = qi < a.G;
    const uint16_t* qrow = a.q + b * a.q_b_stride + (kvh * a.G + (qvalid ? qi : 0)) * a.q_head_stride;
    const int key = t0 + (lane & 15);
    const bool kvalid = key < Lk;
    const uint16_t* krow = a.k + b * a.k_b_stride + kvh * a.k_head_stride + (long)key * a.k_row_stride;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < I::KS; ++kk)
        acc = mfma16(load_frag<256>(qrow, qvalid, kk, lane), load_frag<256>(krow, kvalid, kk, lane), acc);
    float* srow = scores + ((long)(b * a.n_kv + kvh) * 16) * max_keys;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int row = (lane >> 4) * 4 + r;
        if (kvalid && row < a.G) srow[(long)row * max_keys + key] = rbf(rbf(acc[r]) * a.scale);
    }
}

// per chunk: global softmax stats from all scores, P for the chunk, partial O = P.V (fp32)
__global__ void __launch_bounds__(256) k_attn_dec_pv(AttnArgs a, const StepState* st, int max_keys,
                                                      const float* __restrict__ scores, float* __restrict__ opart,
                                                      int max_chunks) {
    const int Lk = st->kv_len + 1;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b = blockIdx.z, kvh = blockIdx.y, chunk = blockIdx.x;
    const int t0 = chunk * DCH;
    if (t0 >= Lk) return;
    __shared__ __attribute__((aligned(16))) uint16_t P[16 * DCH];
    __shared__ __attribute__((aligned(16))) uint16_t VT[256 * (DCH + 8)];
    const float* sbase = scores + ((long)(b * a.n_kv + kvh) * 16) * max_keys;
    for (int row = wave; row < 16; row += 4) {
        if (row < a.G) {
            const float* srow = sbase + (long)row * max_keys;
            float m = -INFINITY;
            for (int t = lane; t < Lk; t += 64) m = fmaxf(m, srow[t]);
            m = wave_max(m);
            float sum = 0.f;
            for (int t = lane; t < Lk; t += 64) sum += expf(srow[t] - m);
            sum = wave_sum(sum);
            const int t = t0 + lane;
            P[row * DCH + lane] = t < Lk ? f2bf(expf(srow[t] - m) / sum) : 0;
        } else {
            P[row * DCH + lane] = 0;
        }
    }
    // V chunk [64 keys][256] -> VT[d][key]
    const uint16_t* vbase = a.v + b * a.v_b_stride + kvh * a.v_head_stride;
    for (int e = tid; e < DCH * 32; e += 256) {
        const int tt = e >> 5, ch = e & 31;
        const int key = t0 + tt;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (key < Lk) v = ldg16(vbase + (long)key * a.v_row_stride + ch * 8);
        const uint16_t* ve = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
        for (int j = 0; j < 8; ++j) VT[(ch * 8 + j) * (DCH + 8) + tt] = ve[j];
    }
    __syncthreads();
    float* ob = opart + (((long)(b * a.n_kv + kvh) * max_chunks + chunk) * 16) * 256;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int ct = wave + 4 * c;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < DCH / 32; ++ks) {
            const short8 pa = *reinterpret_cast<const short8*>(P + (lane & 15) * DCH + ks * 32 + 8 * (lane >> 4));
            const short8 vb =
                *reinterpret_cast<const short8*>(VT + (ct * 16 + (lane & 15)) * (DCH + 8) + ks * 32 + 8 * (lane >> 4));
            acc = mfma16(pa, vb, acc);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) ob[((lane >> 4) * 4 + r) * 256 + ct * 16 + (lane & 15)] = acc[r];
    }
}

// O[b][head][d] = bf16(sum over chunks, fixed order)
__global__ void k_attn_dec_combine(AttnArgs a, const StepState* st, const float* __restrict__ opart,
                                   int max_chunks) {
    const int Lk = st->kv_len + 1;
    const int nch = (Lk + DCH - 1) / DCH;
    const int b = blockIdx.y, kvh = blockIdx.x;
    const float* pb = opart + ((long)(b * a.n_kv + kvh) * max_chunks) * 16 * 256;
    for (int e = threadIdx.x; e < a.G * 256; e += blockDim.x) {
        float s = 0.f;
        for (int c = 0; c < nch; ++c) s += pb[(long)c * 16 * 256 + e];
        const int row = e >> 8, d = e & 255;
        a.o[b * a.o_b_stride + (kvh * a.G + row) * a.o_head_stride + d] = f2bf(s);
    }
}

void attention_decode(hipStream_t s, const AttnArgs& a, const StepState* st, int max_keys, int launch_keys,
                      float* scores, float* opart, int max_chunks) {
    const int nch = (launch_keys + DCH - 1) / DCH;
    dim3 grid(nch, a.n_kv, a.B);
    hipLaunchKernelGGL(k_attn_dec_scores, grid, dim3(256), 0, s, a, st, max_keys, scores);
    hipLaunchKernelGGL(k_attn_dec_pv, grid, dim3(256), 0, s, a, st, max_keys, scores, opart, max_chunks);
    hipLaunchKernelGGL(k_attn_dec_combine, dim3(a.n_kv, a.B), dim3(256), 0, s, a, st, opart, max_chunks);
}

}  // namespace pgmi
