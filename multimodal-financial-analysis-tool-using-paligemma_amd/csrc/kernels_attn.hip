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
#include "attn_decode_body.h"
#include "common.h"
#include "launch.h"

namespace pgmi {


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

typedef s4v_t s4v;

template <int HD>
__global__ void __launch_bounds__(256) k_attn_full(AttnArgs a) {
    using I = HDInfo<HD>;
    constexpr int HDP = I::CT * 16;      // head dim padded to whole 16-column tiles
    constexpr int VS = HDP + 16;         // V row stride in LDS (elements)
    constexpr int CHK = 32;              // keys per P.V chunk
    constexpr int VPT = (CHK * I::CH + 255) / 256;  // 16-B V chunks per thread per key chunk
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int LkP = (a.Lk + 31) & ~31;
    float* S = reinterpret_cast<float*>(smem_raw);                       // [16][LkP]
    uint16_t* P = reinterpret_cast<uint16_t*>(S + 16 * LkP);             // [16][LkP]
    uint16_t* Vl = P + 16 * LkP;                                         // [2][CHK][VS]

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b = blockIdx.z, kvh = blockIdx.y;
    const int row0 = blockIdx.x * 16;
    const int nrows = a.Lq * a.G;

    // ---- phase 1: S = bf16(bf16(Q K^T) * scale); K fragments of the next tile in flight
    const int qi = row0 + (lane & 15);
    const bool qvalid = qi < nrows;
    const int qpos = qvalid ? qi / a.G : 0, qhead = kvh * a.G + (qvalid ? qi % a.G : 0);
    const uint16_t* qrow = a.q + b * a.q_b_stride + (long)qpos * a.q_row_stride + qhead * a.q_head_stride;
    short8 qf[I::KS];
#pragma unroll
    for (int kk = 0; kk < I::KS; ++kk) qf[kk] = load_frag<HD>(qrow, qvalid, kk, lane);

    const uint16_t* kbase = a.k + b * a.k_b_stride + kvh * a.k_head_stride;
    const int ntile = LkP / 16;
    auto kload = [&](int t, short8 (&kf)[I::KS]) {
        const int key = t * 16 + (lane & 15);
        const uint16_t* krow = kbase + (long)(key < a.Lk ? key : 0) * a.k_row_stride;
#pragma unroll
        for (int kk = 0; kk < I::KS; ++kk) kf[kk] = load_frag<HD>(krow, key < a.Lk, kk, lane);
    };
    auto kcompute = [&](int t, const short8 (&kf)[I::KS]) {
        const int key = t * 16 + (lane & 15);
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < I::KS; ++kk) acc = mfma16(qf[kk], kf[kk], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = (lane >> 4) * 4 + r;
            S[row * LkP + key] = key < a.Lk ? rbf(rbf(acc[r]) * a.scale) : -INFINITY;
        }
    };
    {
        short8 kA[I::KS], kB[I::KS];
        int t = wave;
        if (t < ntile) kload(t, kA);
        for (; t < ntile; t += 8) {
            if (t + 4 < ntile) kload(t + 4, kB);
            kcompute(t, kA);
            if (t + 4 >= ntile) break;
            if (t + 8 < ntile) kload(t + 8, kA);
            kcompute(t + 4, kB);
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

    // ---- phase 3: O = bf16(P V); V chunks row-major in LDS (16-B stores), B fragments by
    // ds_read_b64_tr_b16 (transposed read); the next chunk's rows are in flight meanwhile
    const uint16_t* vbase = a.v + b * a.v_b_stride + kvh * a.v_head_stride;
    uint4 vr[VPT];
    auto vload = [&](int t0) {
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
            const int e = tid + 256 * i;
            const int tt = e / I::CH, ch = e % I::CH;
            const int key = t0 + tt;
            vr[i] = (e < CHK * I::CH && key < a.Lk) ? ldg16(vbase + (long)key * a.v_row_stride + ch * 8)
                                                    : make_uint4(0, 0, 0, 0);
        }
    };
    auto vstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
            const int e = tid + 256 * i;
            if (e < CHK * I::CH) {
                const int tt = e / I::CH, ch = e % I::CH;
                *reinterpret_cast<uint4*>(Vl + (buf * CHK + tt) * VS + ch * 8) = vr[i];
            }
        }
        if constexpr (HDP != I::CH * 8) {  // zero the pad columns of the last tile
            for (int e = tid; e < CHK; e += 256)
                *reinterpret_cast<uint4*>(Vl + (buf * CHK + e) * VS + I::CH * 8) = make_uint4(0, 0, 0, 0);
        }
    };
    f32x4 oacc[(I::CT + 3) / 4];
#pragma unroll
    for (int c = 0; c < (I::CT + 3) / 4; ++c) oacc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nch = LkP / CHK;
    vload(0);
    const int g = lane >> 4, li = lane & 15;
    for (int c = 0; c < nch; ++c) {
        const int buf = c & 1;
        vstore(buf);
        if (c + 1 < nch) vload((c + 1) * CHK);
        __syncthreads();  // V chunk (and, at c == 0, all of P) visible
        const short8 pa = *reinterpret_cast<const short8*>(P + (lane & 15) * LkP + c * CHK + 8 * g);
#pragma unroll
        for (int cc = 0; cc < (I::CT + 3) / 4; ++cc) {
            const int ct = wave + 4 * cc;
            if (ct < I::CT) {
                const uint16_t* vp = Vl + (buf * CHK + 8 * g + (li >> 2)) * VS + ct * 16 + 4 * (li & 3);
                const s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (__attribute__((address_space(3))) s4v*)(vp));
                const s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (__attribute__((address_space(3))) s4v*)(vp + 4 * VS));
                const short8 vb = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                oacc[cc] = mfma16(pa, vb, oacc[cc]);
            }
        }
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
    const int hdp = (head_dim + 15) / 16 * 16;
    return (size_t)16 * LkP * 4 + (size_t)16 * LkP * 2 + (size_t)2 * 32 * (hdp + 16) * 2;
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
    const int hdp = (head_dim + 15) / 16 * 16;
    return (int)((160 * 1024 - (size_t)2 * 32 * (hdp + 16) * 2) / (16 * 6)) & ~31;
}

// ================================================================ decode (Lq = 1)
// flash-decoding body: attn_decode_body.h
__global__ void __launch_bounds__(256) k_attn_decode(AttnArgs a, const StepState* st, float* __restrict__ part,
                                                      int max_chunks) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[kAttnDecodeLds];
    attn_decode_block<false>(a, st, part, max_chunks, blockIdx.x, blockIdx.y, blockIdx.z, lds, Dep{});
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
