#pragma once
// attn_decode_body.h -- flash-decoding workgroup body (kernel k_attn_decode: kernels_attn.hip).
//
// Workgroup c owns keys [64c, 64c+64) of one (b, kv head) for all G query heads.  Scores are
// rounded exactly as the reference (bf16(bf16(q.k) * scale), modeling_gemma.py:262-266); each
// chunk writes (m_c, l_c = sum e^(s - m_c), O_c = sum e^(s - m_c) v) in fp32.  The combine
// o = bf16(sum_c e^(m_c - M) O_c / sum_c e^(m_c - M) l_c), in a fixed chunk order, is the
// prologue of the o_proj GEMV that consumes o (gemv_body.h, GV_ORES).
// P.V runs on MFMA from bf16 e = exp(s - m_c) (the reference rounds the normalised p to bf16,
// modeling_gemma.py:273,277; here the unnormalised chunk-local e is rounded, the fp32 sum l_c
// normalises at the combine: same rounding granularity, documented in DESIGN.md).
#include "common.h"
#include "launch.h"

namespace pgmi {

constexpr int DCH = 64;                 // keys per chunk
constexpr int PSTRIDE = 16 * 256 + 32;  // per-chunk partial record: O_c[16][256], m_c[16], l_c[16]
constexpr int DVS = 256 + 16;           // V row stride in LDS (elements): tr16 reads 2-way at most
constexpr int DPS = DCH + 8;            // P row stride in LDS (elements)
constexpr int DVH = DCH / 2;           // V rows staged in LDS at a time (two halves per chunk)
constexpr int kAttnDecodeLds = DVH * DVS * 2 + 16 * (DCH + 4) * 4 + 16 * DPS * 2 + 2 * 16 * 4;

typedef short s4v_t __attribute__((ext_vector_type(4)));

// fragment of a row that is always valid memory (callers clamp the row): an unconditional load,
// no select on the loaded value (hipcc turns such a select back into a branch around the load)
__device__ __forceinline__ short8 frag256(const uint16_t* rowp, int kk, int lane) {
    const int k = 32 * kk + 8 * (lane >> 4);
    return __builtin_bit_cast(short8, ldg16(rowp + k));
}

__device__ __forceinline__ void attn_decode_block(const AttnArgs& a, const StepState* st, float* __restrict__ part,
                                                  int max_chunks, int chunk, int kvh, int b, unsigned char* lds) {
    const int kv_len = st->kv_len;
    const int Lk = kv_len + 1;
    const int nch = (Lk + DCH - 1) / DCH;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (chunk >= nch) return;
    const int t0 = chunk * DCH;
    const int nk = (Lk - t0) < DCH ? (Lk - t0) : DCH;
    uint16_t* Vs = reinterpret_cast<uint16_t*>(lds);                          // [DVH][DVS]
    float (*S)[DCH + 4] = reinterpret_cast<float (*)[DCH + 4]>(lds + DVH * DVS * 2);
    uint16_t* Ps = reinterpret_cast<uint16_t*>(lds + DVH * DVS * 2 + 16 * (DCH + 4) * 4);
    float (*stat)[16] = reinterpret_cast<float (*)[16]>(lds + DVH * DVS * 2 + 16 * (DCH + 4) * 4 + 16 * DPS * 2);

    const uint16_t* vb = a.v + b * a.v_b_stride + kvh * a.v_head_stride;
    uint4 vr[DCH * 32 / 256];
#pragma unroll
    for (int i = 0; i < DCH * 32 / 256; ++i) {
        const int e = tid + 256 * i, r = e >> 5, c = e & 31;
        // rows past the cache read the last row instead: their e is 0 (finite data times 0)
        vr[i] = ldg16(vb + (long)(r < nk ? t0 + r : Lk - 1) * a.v_row_stride + 8 * c);
    }
    const int qi = lane & 15;
    const bool qvalid = qi < a.G;
    const uint16_t* qrow = a.q + b * a.q_b_stride + (kvh * a.G + (qvalid ? qi : 0)) * a.q_head_stride;
    const int key = t0 + wave * 16 + (lane & 15);
    // rows past the cache are never read: the row is clamped (its scores are masked below), and
    // query lanes past G read head 0 (their score rows are never used)
    const uint16_t* krow = a.k + b * a.k_b_stride + kvh * a.k_head_stride + (long)(key < Lk ? key : 0) * a.k_row_stride;
    short8 qf[8], kf[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) kf[kk] = frag256(krow, kk, lane);
    // the additive mask of this lane's key (a zero word when there is none): issued with the K rows
    const float mval = a.mask[(long)b * a.mask_b_stride + (long)(key < Lk ? key : 0) * a.mask_k_stride];

#pragma unroll
    for (int kk = 0; kk < 8; ++kk) qf[kk] = frag256(qrow, kk, lane);

    // ---- scores (MFMA): wave w -> keys t0 + 16w + (lane & 15)
    {
        const bool kvalid = key < Lk;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) acc = mfma16(qf[kk], kf[kk], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            // bf16(bf16(q.k) * scale), then + mask (:266,269): rounded for a bf16 mask (exact for a zero one)
            const float sv = rbf(rbf(acc[r]) * a.scale) + mval;
            S[(lane >> 4) * 4 + r][wave * 16 + (lane & 15)] = kvalid ? (a.mask_round ? rbf(sv) : sv) : -INFINITY;
        }
    }
    constexpr int VPH = DVH * 32 / 256;  // V chunks per thread per half
    auto stage_v = [&](int half) {      // rows [32 half, 32 half + 32) of the chunk -> Vs
#pragma unroll
        for (int i = 0; i < VPH; ++i) {
            const int e = tid + 256 * i, r = e >> 5, c = e & 31;
            *reinterpret_cast<uint4*>(Vs + r * DVS + 8 * c) = vr[half * VPH + i];
        }
    };
    stage_v(0);
    __syncthreads();
    // ---- chunk-local max / exp / sum: wave w handles head rows 4w..4w+3, lane = key.  The four
    // rows' butterfly reductions are interleaved (four independent cross-lane chains instead of
    // one chain four times as long)
    {
        float sv[4], m[4], e[4], l[4];
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            sv[rr] = S[wave * 4 + rr][lane];
            m[rr] = sv[rr];
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) m[rr] = fmaxf(m[rr], __shfl_xor(m[rr], o, 64));
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            const int h = wave * 4 + rr;
            // (a chunk whose keys are all masked to -inf has m = -inf: e = 0, not exp(NaN))
            e[rr] = (lane < nk && h < a.G && m[rr] != -INFINITY) ? expf(sv[rr] - m[rr]) : 0.f;
            Ps[h * DPS + lane] = f2bf(e[rr]);
            l[rr] = e[rr];
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) l[rr] += __shfl_xor(l[rr], o, 64);
        if (lane == 0) {
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                stat[0][wave * 4 + rr] = m[rr];
                stat[1][wave * 4 + rr] = l[rr];
            }
        }
    }
    __syncthreads();
    // ---- O_c[h][d] = sum_t e[h][t] v[t][d] (MFMA): wave w -> d tiles 4w..4w+3; B operand by
    // ds_read_b64_tr_b16 from the row-major V image
    float* pb = part + ((long)(b * a.n_kv + kvh) * max_chunks + chunk) * PSTRIDE;
    {
        const int g = lane >> 4, li = lane & 15;
        f32x4 acc[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {  // V half kk holds keys [32 kk, 32 kk + 32)
            if (kk == 1) {
                __syncthreads();  // every wave is done with half 0
                stage_v(1);
                __syncthreads();
            }
            const short8 pa = *reinterpret_cast<const short8*>(Ps + li * DPS + 32 * kk + 8 * g);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int ct = wave * 4 + j;
                const uint16_t* vp = Vs + (8 * g + (li >> 2)) * DVS + ct * 16 + 4 * (li & 3);
                const s4v_t lo =
                    __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v_t*)(vp));
                const s4v_t hi =
                    __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v_t*)(vp + 4 * DVS));
                const short8 vbf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                acc[j] = mfma16(pa, vbf, acc[j]);
            }
        }
        // C map: col d = ct*16 + (lane & 15), row h = (lane >> 4)*4 + r
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int ct = wave * 4 + j;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int h = (lane >> 4) * 4 + r;
                if (h < a.G) pb[h * 256 + ct * 16 + li] = acc[j][r];
            }
        }
    }
    if (tid < 32) pb[16 * 256 + tid] = stat[tid >> 4][tid & 15];
}

}  // namespace pgmi
