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
// Flash-decoding: workgroup c owns keys [64c, 64c+64) of one (b, kv head) for all G query
// heads.  Scores are rounded exactly as the reference (bf16(bf16(q.k) * scale)); each chunk
// writes (m_c, l_c = sum e^(s - m_c), O_c = sum e^(s - m_c) v) in fp32.  The combine
// o = bf16(sum_c e^(m_c - M) O_c / sum_c e^(m_c - M) l_c), in a fixed chunk order, is the
// prologue of the o_proj GEMV that consumes o (kernels_gemv.hip, GV_ORES): no inter-workgroup
// hand-off inside this kernel, the kernel boundary orders it.
// Deviation from the reference (documented in DESIGN.md): the reference rounds the normalised
// probabilities to bf16 before P.V (modeling_gemma.py:273,277); here P.V is accumulated from
// the fp32 probabilities (closer to the fp32 result; rel. difference ~2^-9 per term).
constexpr int DCH = 64;  // keys per chunk

constexpr int PSTRIDE = 16 * 256 + 32;  // per-chunk partial record: O_c[16][256], m_c[16], l_c[16]

__global__ void __launch_bounds__(256) k_attn_decode(AttnArgs a, const StepState* st, float* __restrict__ part,
                                                      int max_chunks) {
    const int Lk = st->kv_len + 1;
    const int nch = (Lk + DCH - 1) / DCH;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b = blockIdx.z, kvh = blockIdx.y, chunk = blockIdx.x;
    if (chunk >= nch) return;
    const int t0 = chunk * DCH;
    __shared__ __attribute__((aligned(16))) float S[16][DCH + 4];   // scores, then e = exp(s - m_c)
    __shared__ __attribute__((aligned(16))) float ET[DCH][16];      // e transposed: [key][head]
    __shared__ __attribute__((aligned(16))) float R[128][17];       // key-half reduction
    __shared__ float stat[2][16];

    // V rows of this chunk first (their latency overlaps the scores): thread = (d pair, key half),
    // all 32 row loads in flight; rows past the cache length are clamped (their e is 0)
    const int dp = tid & 127, kh = tid >> 7;
    const int nk = (Lk - t0) < DCH ? (Lk - t0) : DCH;
    uint32_t vv[DCH / 2];
    {
        const uint16_t* vb = a.v + b * a.v_b_stride + kvh * a.v_head_stride + 2 * dp;
#pragma unroll
        for (int tt = 0; tt < DCH / 2; ++tt) {
            int t = kh * (DCH / 2) + tt;
            t = t < nk ? t : nk - 1;
            vv[tt] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(vb + (long)(t0 + t) * a.v_row_stride));
        }
    }
    float acc0[8], acc1[8];
#pragma unroll
    for (int h = 0; h < 8; ++h) { acc0[h] = 0.f; acc1[h] = 0.f; }

    // ---- scores (MFMA): wave w -> keys t0 + 16w + (lane & 15)
    {
        const int qi = lane & 15;
        const bool qvalid = qi < a.G;
        const uint16_t* qrow = a.q + b * a.q_b_stride + (kvh * a.G + (qvalid ? qi : 0)) * a.q_head_stride;
        const int key = t0 + wave * 16 + (lane & 15);
        const bool kvalid = key < Lk;
        const uint16_t* krow = a.k + b * a.k_b_stride + kvh * a.k_head_stride + (long)key * a.k_row_stride;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 8; ++kk)
            acc = mfma16(load_frag<256>(qrow, qvalid, kk, lane), load_frag<256>(krow, kvalid, kk, lane), acc);
#pragma unroll
        for (int r = 0; r < 4; ++r)
            S[(lane >> 4) * 4 + r][wave * 16 + (lane & 15)] = kvalid ? rbf(rbf(acc[r]) * a.scale) : -INFINITY;
    }
    __syncthreads();
    // ---- chunk-local max / exp / sum: wave w handles rows 4w..4w+3, lane = key
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
        const int h = wave * 4 + rr;
        const float sv = S[h][lane];
        const float m = wave_max(sv);
        const float e = (t0 + lane < Lk && h < a.G) ? expf(sv - m) : 0.f;
        ET[lane][h] = e;
        const float l = wave_sum(e);
        if (lane == 0) { stat[0][h] = m; stat[1][h] = l; }
    }
    __syncthreads();
    // ---- O_c[h][d] = sum_t e[t][h] * v[t][d]: thread = (d pair, key half); V rows were loaded
    // at kernel entry
#pragma unroll
    for (int tt = 0; tt < DCH / 2; ++tt) {
        const int t = kh * (DCH / 2) + tt;
        const float v0 = __uint_as_float(vv[tt] << 16), v1 = __uint_as_float(vv[tt] & 0xFFFF0000u);
        const f32x4 e0 = *reinterpret_cast<const f32x4*>(&ET[t][0]);
        const f32x4 e1 = *reinterpret_cast<const f32x4*>(&ET[t][4]);
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            acc0[h] += e0[h] * v0; acc1[h] += e0[h] * v1;
            acc0[h + 4] += e1[h] * v0; acc1[h + 4] += e1[h] * v1;
        }
    }
    if (kh == 1) {
#pragma unroll
        for (int h = 0; h < 8; ++h) { R[dp][h] = acc0[h]; R[dp][8 + h] = acc1[h]; }
    }
    __syncthreads();
    float* pb = part + ((long)(b * a.n_kv + kvh) * max_chunks + chunk) * PSTRIDE;
    if (kh == 0) {
#pragma unroll
        for (int h = 0; h < 8; ++h) {
            if (h < a.G) {
                const float2 o = make_float2(acc0[h] + R[dp][h], acc1[h] + R[dp][8 + h]);
                *reinterpret_cast<float2*>(pb + h * 256 + 2 * dp) = o;
            }
        }
    }
    if (tid < 32) pb[16 * 256 + tid] = stat[tid >> 4][tid & 15];

}

size_t attention_decode_part_floats(int B, int n_kv, int max_chunks) {
    return (size_t)B * n_kv * max_chunks * PSTRIDE;
}

void attention_decode(hipStream_t s, const AttnArgs& a, const StepState* st, int launch_keys, float* part,
                      int max_chunks) {
    const int nch = (launch_keys + DCH - 1) / DCH;
    dim3 grid(nch < max_chunks ? nch : max_chunks, a.n_kv, a.B);
    hipLaunchKernelGGL(k_attn_decode, grid, dim3(256), 0, s, a, st, part, max_chunks);
}

}  // namespace pgmi
