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

#include <cmath>
#include <cstdlib>

namespace pgmi {


template <int HD>
struct HDInfo {
    static constexpr int KS = (HD + 31) / 32;   // 32-deep k-steps for QK^T
    static constexpr int CT = (HD + 15) / 16;   // 16-wide output column tiles for PV
    static constexpr int CH = (HD + 7) / 8;     // 16-B chunks per head row
};

// load the 16-row A (or B) fragment: lane -> row (lane&15), k = 32*kk + 8*(lane>>4)
// The row must be valid memory: callers clamp rows past the end (their scores are masked or their
// outputs never stored), so the load is unconditional -- a select on a loaded value is turned back
// into a branch around the load by hipcc.  Only head dims that are not a multiple of 32 zero the
// k range past HD (HD 72: the last 32-deep step).
template <int HD>
__device__ __forceinline__ short8 load_frag(const uint16_t* rowp, bool /*row valid: clamped by the caller*/,
                                            int kk, int lane) {
    const int k = 32 * kk + 8 * (lane >> 4);
    if constexpr (HD % 32 == 0) return __builtin_bit_cast(short8, ldg16(rowp + k));
    else {
        // chunks past HD: an unconditional load of the row's first chunk (the address is selected,
        // not the loaded value), zeroed by a mask -- no branch around the load
        uint4 v = ldg16(rowp + (k < HD ? k : 0));
        const unsigned msk = k < HD ? ~0u : 0u;
        v.x &= msk; v.y &= msk; v.z &= msk; v.w &= msk;
        return __builtin_bit_cast(short8, v);
    }
}

typedef s4v_t s4v;

// output rows of the C map (16x16x32: lane holds rows 4g + r, r < 4, of its 16-row group): the
// four row pointers are resolved once (row -> (position, head) takes a division by G), so the
// per-element stores are a plain offset (nullptr: row past the end)
__device__ __forceinline__ void attn_out_rows(const AttnArgs& a, int b, int kvh, int i0, int nrows,
                                              uint16_t* (&orow)[4]) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = i0 + r;
        const int pos = i / a.G, head = kvh * a.G + i % a.G;
        orow[r] = i < nrows ? a.o + b * a.o_b_stride + (long)pos * a.o_row_stride + head * a.o_head_stride : nullptr;
    }
}

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
            vr[i] = (e < CHK * I::CH) ? ldg16(vbase + (long)(key < a.Lk ? key : a.Lk - 1) * a.v_row_stride + ch * 8)
                                      : make_uint4(0, 0, 0, 0);  // rows past the keys: p = 0
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
    uint16_t* orow[4];
    attn_out_rows(a, b, kvh, row0 + (lane >> 4) * 4, nrows, orow);
#pragma unroll
    for (int c = 0; c < (I::CT + 3) / 4; ++c) {
        const int ct = wave + 4 * c;
        if (ct >= I::CT) continue;
        const int d = ct * 16 + (lane & 15);
        if (d >= HD) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (orow[r]) orow[r][d] = f2bf(oacc[c][r]);
    }
}

// ---------------------------------------------------------------- prefill, 16 rows, loads up front
// k_attn_full for short key ranges (Gemma at 224 px: 288 keys x d 256, MQA): the same three phases,
// but every global load of the workgroup is issued before the first one is consumed -- each wave's
// K fragments for all its 16-key tiles, then the V rows of every 32-key chunk (VGPR-resident until
// their chunk is staged) -- so the kernel pays one L2 round trip instead of one per K tile and per
// V chunk.  Keys <= 16 * 4 * MAXT and <= 32 * MAXC.  Scores are kept in LDS as bf16 (they are
// bf16-rounded values, modeling_gemma.py:266) and P overwrites them row by row.
template <int HD, int MAXT, int MAXC>
__global__ void __launch_bounds__(256) k_attn_full_pre(AttnArgs a) {
    using I = HDInfo<HD>;
    constexpr int HDP = I::CT * 16;
    constexpr int VS = HDP + 16;
    constexpr int CHK = 32;
    constexpr int VPT = (CHK * I::CH + 255) / 256;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int LkP = (a.Lk + 31) & ~31;
    uint16_t* S = reinterpret_cast<uint16_t*>(smem_raw);  // [16][LkP] bf16 P
    uint16_t* Vl = S + 16 * LkP;                          // [2][CHK][VS], then [2][4][16] fp32 row stats

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b = blockIdx.z, kvh = blockIdx.y;
    const int row0 = blockIdx.x * 16;
    const int nrows = a.Lq * a.G;
    const int qi = row0 + (lane & 15);
    const bool qvalid = qi < nrows;
    const int qpos = qvalid ? qi / a.G : 0, qhead = kvh * a.G + (qvalid ? qi % a.G : 0);
    const uint16_t* qrow = a.q + b * a.q_b_stride + (long)qpos * a.q_row_stride + qhead * a.q_head_stride;
    const uint16_t* kbase = a.k + b * a.k_b_stride + kvh * a.k_head_stride;
    const uint16_t* vbase = a.v + b * a.v_b_stride + kvh * a.v_head_stride;
    const int ntile = LkP / 16, nch = LkP / CHK;

    short8 qf[I::KS];
#pragma unroll
    for (int kk = 0; kk < I::KS; ++kk) qf[kk] = load_frag<HD>(qrow, qvalid, kk, lane);
    // K fragments of this wave's tiles t = wave + 4j, then every V chunk: all in flight together
    short8 kf[MAXT][I::KS];
#pragma unroll
    for (int j = 0; j < MAXT; ++j) {
        const int key = (wave + 4 * j) * 16 + (lane & 15);
        const bool ok = key < a.Lk;
        const uint16_t* krow = kbase + (long)(ok ? key : 0) * a.k_row_stride;
#pragma unroll
        for (int kk = 0; kk < I::KS; ++kk) kf[j][kk] = load_frag<HD>(krow, ok, kk, lane);
    }
    uint4 vr[MAXC][VPT];
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
            int e = tid + 256 * i;
            if (CHK * I::CH % 256 != 0 && e >= CHK * I::CH) e = 0;  // tail lanes (HD 72): re-read piece 0, not stored
            const int key = c * CHK + e / I::CH, ch = e % I::CH;
            vr[c][i] = ldg16(vbase + (long)(key < a.Lk ? key : a.Lk - 1) * a.v_row_stride + ch * 8);  // p = 0 past Lk
        }

    // ---- phase 1: s = bf16(bf16(Q K^T) * scale), kept in registers: lane (g, li) holds rows 4g + r
    // of keys 16 t + li for this wave's tiles t = wave + 4 j
    const int g = lane >> 4, li = lane & 15;
    float sc[MAXT][4];
#pragma unroll
    for (int j = 0; j < MAXT; ++j) {
        const int t = wave + 4 * j;
        const int key = t * 16 + li;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < I::KS; ++kk) acc = mfma16(qf[kk], kf[j][kk], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) sc[j][r] = (t < ntile && key < a.Lk) ? rbf(rbf(acc[r]) * a.scale) : -INFINITY;
    }
    // ---- phase 2: exact softmax per row: max and sum of exp over the row's keys (lane, then the 16
    // lanes of a row group, then the 4 waves in a fixed order), p = bf16(exp(s - max) / sum) -> LDS
    float* red = reinterpret_cast<float*>(Vl + 2 * CHK * VS);  // [2][4 waves][16 rows]
    float mx[4], sm[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        mx[r] = sc[0][r];
#pragma unroll
        for (int j = 1; j < MAXT; ++j) mx[r] = fmaxf(mx[r], sc[j][r]);
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx[r] = fmaxf(mx[r], __shfl_xor(mx[r], o, 64));
    if (li == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) red[wave * 16 + 4 * g + r] = mx[r];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int row = 4 * g + r;
        mx[r] = fmaxf(fmaxf(red[row], red[16 + row]), fmaxf(red[32 + row], red[48 + row]));
        sm[r] = 0.f;
#pragma unroll
        for (int j = 0; j < MAXT; ++j) {
            sc[j][r] = sc[j][r] == -INFINITY ? 0.f : expf(sc[j][r] - mx[r]);
            sm[r] += sc[j][r];
        }
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1)
#pragma unroll
        for (int r = 0; r < 4; ++r) sm[r] += __shfl_xor(sm[r], o, 64);
    if (li == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) red[64 + wave * 16 + 4 * g + r] = sm[r];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int row = 4 * g + r;
        const float L = ((red[64 + row] + red[80 + row]) + red[96 + row]) + red[112 + row];
#pragma unroll
        for (int j = 0; j < MAXT; ++j) {
            const int key = (wave + 4 * j) * 16 + li;
            if (key < LkP) S[row * LkP + key] = key < a.Lk ? f2bf(sc[j][r] / L) : 0;
        }
    }
    // ---- phase 3: O = bf16(P V), V chunks staged from registers into two LDS buffers
    f32x4 oacc[(I::CT + 3) / 4];
#pragma unroll
    for (int c = 0; c < (I::CT + 3) / 4; ++c) oacc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        if (c < nch) {  // uniform: no early exit, so the register arrays stay statically indexed
        const int buf = c & 1;
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
            const int e = tid + 256 * i;
            if (e < CHK * I::CH)
                *reinterpret_cast<uint4*>(Vl + (buf * CHK + e / I::CH) * VS + (e % I::CH) * 8) = vr[c][i];
        }
        if constexpr (HDP != I::CH * 8) {
            for (int e = tid; e < CHK; e += 256)
                *reinterpret_cast<uint4*>(Vl + (buf * CHK + e) * VS + I::CH * 8) = make_uint4(0, 0, 0, 0);
        }
        __syncthreads();  // V chunk (and, at c == 0, all of P) visible; buffer buf^1 free
        const short8 pa = *reinterpret_cast<const short8*>(S + (lane & 15) * LkP + c * CHK + 8 * g);
#pragma unroll
        for (int cc = 0; cc < (I::CT + 3) / 4; ++cc) {
            const int ct = wave + 4 * cc;
            if (ct < I::CT) {
                const uint16_t* vp = Vl + (buf * CHK + 8 * g + (li >> 2)) * VS + ct * 16 + 4 * (li & 3);
                const s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v*)(vp));
                const s4v hi =
                    __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v*)(vp + 4 * VS));
                const short8 vb = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                oacc[cc] = mfma16(pa, vb, oacc[cc]);
            }
        }
        }
    }
    uint16_t* orow[4];
    attn_out_rows(a, b, kvh, row0 + (lane >> 4) * 4, nrows, orow);
#pragma unroll
    for (int c = 0; c < (I::CT + 3) / 4; ++c) {
        const int ct = wave + 4 * c;
        if (ct >= I::CT) continue;
        const int d = ct * 16 + (lane & 15);
        if (d >= HD) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (orow[r]) orow[r][d] = f2bf(oacc[c][r]);
    }
}

// ---------------------------------------------------------------- prefill, K/V-tiled (two pass)
// One workgroup = RG x 16 query rows (RG waves, one 16-row group each) x all keys, K/V streamed
// through LDS in 32-key tiles that every wave of the workgroup shares (the 16-row kernel above
// re-read the whole K and V from L2 for every 16 rows).  KSPL key-split groups of RG waves
// take alternate tiles and meet in LDS at the two combine points.  No score matrix is kept,
// so the key count is unbounded; the reference's rounding points stay exact:
//   pass 1: s = bf16(bf16(k.q) * scale) per tile, lane-local online (max, sum exp) -> per-row
//           M, L after a fixed-order combine (lanes, then split groups);
//   pass 2: s recomputed, p = bf16(exp(s - M) / L) (the reference's bf16(softmax_f32)),
//           O += p.V on MFMA, O summed over split groups in a fixed order, rounded once.
// Scores are computed transposed, S^T = K Q^T (A = K rows from LDS, B = Q fragments held in
// registers): lane (g = lane >> 4) then holds query (lane & 15) x keys {4g..4g+3, 16+4g..16+4g+3}
// of the tile, which is exactly an A fragment of P for the P.V MFMA under the k-slot order
// j<4 -> 4g+j, j>=4 -> 16+4g+j-4; the V operand is read in that key order by transposed LDS reads.
// K rows in LDS: 16-B chunk c of row r at chunk (c ^ (r & 15)) -- conflict-free ds_read_b128 of
// 16 rows x one 64-B k slice; rows padded with zero chunks to 16 (HD 72) / 32 (HD 256) chunks.
template <int HD>
struct FAInfo {
    static constexpr int KS = (HD + 31) / 32;                  // 32-deep k-steps of K.Q
    static constexpr int CT = (HD + 15) / 16;                  // 16-wide output tiles of P.V
    static constexpr int CH = (HD + 7) / 8;                    // 16-B chunks of a head row
    static constexpr int KRC = KS * 4 <= 16 ? 16 : KS * 4;     // K row chunks in LDS (>= 16 for the swizzle)
    static constexpr int KRS = KRC * 8;                        // K row stride (elements)
    static constexpr int VS = (CT * 16 + 127) / 128 * 128 + 16;  // V row stride: 8 mod 64 dwords
};

__device__ __forceinline__ float fa_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }

// combine two (max, sum-of-exp) pairs (exact when one side is empty)
__device__ __forceinline__ void fa_comb(float& m, float& l, float m2, float l2) {
    const float M = fmaxf(m, m2);
    if (M == -INFINITY) return;
    l = (m == -INFINITY ? 0.f : l * fa_exp(m - M)) + (m2 == -INFINITY ? 0.f : l2 * fa_exp(m2 - M));
    m = M;
}

// LDS hand-off between the tile loads and the MFMA reads: wait for this wave's own LDS stores,
// then a raw s_barrier -- __syncthreads()'s release fence would also wait vmcnt(0) and drain the
// register prefetch of the next PD tiles at every tile
#define PGMI_LDS_BARRIER() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")

template <int HD, int RG, int KSPL, int PD>
__global__ void __launch_bounds__(64 * RG * KSPL) k_attn_fa(AttnArgs a) {
    using I = FAInfo<HD>;
    constexpr int KS = I::KS, CT = I::CT, CH = I::CH, KRC = I::KRC, KRS = I::KRS, VS = I::VS;
    constexpr int TK = 32;                                 // keys per tile
    constexpr int NTH = 64 * RG;                           // threads of one split group
    constexpr int LCH = (TK * CH + NTH - 1) / NTH;         // 16-B chunks per thread per tile (K; V alike)
    constexpr int KBUF = TK * KRS, VBUF = TK * VS;         // elements per buffer
    constexpr int GRP = 2 * (KBUF + VBUF);                 // elements per split group (2 buffers each)
    extern __shared__ __attribute__((aligned(16))) uint16_t fsm[];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int rg = wave % RG, ks = wave / RG, th = tid % NTH;
    const int g = lane >> 4, li = lane & 15;
    uint16_t* Kl = fsm + ks * GRP;
    uint16_t* Vl = Kl + 2 * KBUF;
    float* stat = reinterpret_cast<float*>(fsm + KSPL * GRP);  // [KSPL][RG][16][2]

    const int b = blockIdx.z, kvh = blockIdx.y;
    const int nrows = a.Lq * a.G;
    const int qi = blockIdx.x * (16 * RG) + rg * 16 + li;
    const bool qvalid = qi < nrows;
    const int qpos = qvalid ? qi / a.G : 0, qhead = kvh * a.G + (qvalid ? qi % a.G : 0);
    const uint16_t* qrow = a.q + b * a.q_b_stride + (long)qpos * a.q_row_stride + qhead * a.q_head_stride;
    short8 qf[KS];
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) qf[kk] = load_frag<HD>(qrow, qvalid, kk, lane);

    // zero the K pad chunks once (never written by tile stores; k-steps past HD read them)
    if constexpr (KRC > CH) {
        for (int e = th; e < 2 * TK * (KRC - CH); e += NTH) {
            const int r = e / (KRC - CH), c = CH + e % (KRC - CH);  // r over both buffers' rows
            *reinterpret_cast<uint4*>(Kl + r * KRS + ((c ^ (r & 15)) << 3)) = make_uint4(0, 0, 0, 0);
        }
    }

    const uint16_t* kbase = a.k + b * a.k_b_stride + kvh * a.k_head_stride;
    const uint16_t* vbase = a.v + b * a.v_b_stride + kvh * a.v_head_stride;
    const int nt = (a.Lk + TK - 1) / TK;
    // tiles per split group, padded to whole PD-groups: a tile past the keys is all zeros and
    // masked (s = -inf, p = 0), so the padded iterations change nothing and the loop body has no
    // branch around its loads (a branch would make hipcc wait for the whole prefetch)
    const int nit = ((nt + KSPL - 1) / KSPL + PD - 1) / PD * PD;

    // register ring: tile it (it >= 1) of this split group lives in slot (it - 1) % PD from its
    // issue until it is stored to LDS at iteration it - 1; tile 0 goes straight to LDS buffer 0
    uint4 kr[PD][LCH], vr[PD][LCH];
    // every load is issued, unconditionally: rows past the keys (and tiles past the end) read the
    // last key's row instead -- its scores are masked to -inf and its p is 0, so the duplicate
    // contributes nothing (V rows are finite data) -- and lanes past the tile's chunks re-read
    // chunk 0 (not stored).  No select touches a loaded value, so nothing branches around a load.
    auto gload = [&](int sl, int t, bool withv) {
#pragma unroll
        for (int i = 0; i < LCH; ++i) {
            int e = th + NTH * i;
            if (TK * CH % NTH != 0 && e >= TK * CH) e = 0;
            int key = t * TK + e / CH;
            key = key < a.Lk ? key : a.Lk - 1;
            const int ch = e % CH;
            kr[sl][i] = ldg16(kbase + (long)key * a.k_row_stride + ch * 8);
            if (withv) vr[sl][i] = ldg16(vbase + (long)key * a.v_row_stride + ch * 8);
        }
    };
    auto lstore = [&](int sl, int buf, bool withv) {
#pragma unroll
        for (int i = 0; i < LCH; ++i) {
            const int e = th + NTH * i;
            if (e < TK * CH) {
                const int r = e / CH, ch = e % CH;
                *reinterpret_cast<uint4*>(Kl + buf * KBUF + r * KRS + ((ch ^ (r & 15)) << 3)) = kr[sl][i];
                if (withv) *reinterpret_cast<uint4*>(Vl + buf * VBUF + r * VS + ch * 8) = vr[sl][i];
            }
        }
    };
    // S^T for the 32 keys of the tile in buffer buf: s[kt][r] = key t*32 + 16kt + 4g + r, query li.
    // Even and odd k-steps accumulate in separate registers (two independent MFMA chains per key
    // half, four in all, instead of one KS-deep dependent chain each), summed once at the end.
    auto scores = [&](int buf, int t, float (&s)[2][4]) {
        f32x4 acc[2][2];
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) acc[kt][0] = acc[kt][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < KS; ++kk)
#pragma unroll
            for (int kt = 0; kt < 2; ++kt) {
                const int r = kt * 16 + li;
                const short8 kf =
                    *reinterpret_cast<const short8*>(Kl + buf * KBUF + r * KRS + (((kk * 4 + g) ^ (r & 15)) << 3));
                acc[kt][kk & 1] = mfma16(kf, qf[kk], acc[kt][kk & 1]);
            }
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int key = t * TK + kt * 16 + 4 * g + j;
                const float v = rbf(rbf(acc[kt][0][j] + acc[kt][1][j]) * a.scale);  // computed for every key
                s[kt][j] = key < a.Lk ? v : -INFINITY;                              // then masked
            }
    };
    // pass prologue: tile 0 -> LDS buffer 0, tiles 1..PD -> the register ring
    auto prologue = [&](bool withv) {
        gload(0, ks, withv);
        lstore(0, 0, withv);
#pragma unroll
        for (int q = 0; q < PD; ++q) gload(q, (1 + q) * KSPL + ks, withv);
        PGMI_LDS_BARRIER();
    };

    // ---- pass 1: per-row max and sum of exp
    float m = -INFINITY, l = 0.f;
    prologue(false);
    for (int it0 = 0; it0 < nit; it0 += PD) {
#pragma unroll
        for (int q = 0; q < PD; ++q) {
            const int it = it0 + q;
            const int t = it * KSPL + ks, buf = it & 1;
            float s[2][4];
            scores(buf, t, s);
            float tm = -INFINITY;
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int j = 0; j < 4; ++j) tm = fmaxf(tm, s[kt][j]);
            const float mn = fmaxf(m, tm);
            if (mn != -INFINITY) {
                float ts = 0.f;
#pragma unroll
                for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                    for (int j = 0; j < 4; ++j) ts += fa_exp(s[kt][j] - mn);
                l = (m == -INFINITY ? 0.f : l * fa_exp(m - mn)) + ts;
                m = mn;
            }
            lstore(q, buf ^ 1, false);                   // tile it + 1
            gload(q, (it + 1 + PD) * KSPL + ks, false);  // tile it + 1 + PD into the freed slot
            PGMI_LDS_BARRIER();
        }
    }
    // lanes g = 0..3 of a query, in a fixed order
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1) {
        const float m2 = __shfl_xor(m, o, 64), l2 = __shfl_xor(l, o, 64);
        if (lane & o) fa_comb(m, l, m2, l2);  // the higher lane group folds the lower one in ...
        else {
            float mm = m2, ll = l2;
            fa_comb(mm, ll, m, l);            // ... the same way, so both sides agree bitwise
            m = mm;
            l = ll;
        }
    }
    if constexpr (KSPL > 1) {
        if (g == 0) {
            stat[((ks * RG + rg) * 16 + li) * 2 + 0] = m;
            stat[((ks * RG + rg) * 16 + li) * 2 + 1] = l;
        }
        __syncthreads();
        m = stat[(rg * 16 + li) * 2 + 0];
        l = stat[(rg * 16 + li) * 2 + 1];
#pragma unroll
        for (int q = 1; q < KSPL; ++q)
            fa_comb(m, l, stat[((q * RG + rg) * 16 + li) * 2 + 0], stat[((q * RG + rg) * 16 + li) * 2 + 1]);
    }
    const float invl = 1.0f / l;

    // ---- pass 2: O = sum over tiles of bf16(p) . V
    f32x4 oacc[CT];
#pragma unroll
    for (int c = 0; c < CT; ++c) oacc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    prologue(true);
    for (int it0 = 0; it0 < nit; it0 += PD) {
#pragma unroll
        for (int q = 0; q < PD; ++q) {
            const int it = it0 + q;
            const int t = it * KSPL + ks, buf = it & 1;
            float s[2][4];
            scores(buf, t, s);
            short8 pa;
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int j = 0; j < 4; ++j) pa[kt * 4 + j] = (short)f2bf(fa_exp(s[kt][j] - m) * invl);
            const uint16_t* vb0 = Vl + buf * VBUF + (4 * g + (li >> 2)) * VS + 4 * (li & 3);
#pragma unroll
            for (int c = 0; c < CT; ++c) {
                const s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (__attribute__((address_space(3))) s4v*)(vb0 + c * 16));
                const s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (__attribute__((address_space(3))) s4v*)(vb0 + 16 * VS + c * 16));
                const short8 vb = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                oacc[c] = mfma16(pa, vb, oacc[c]);
            }
            lstore(q, buf ^ 1, true);
            gload(q, (it + 1 + PD) * KSPL + ks, true);
            PGMI_LDS_BARRIER();
        }
    }
    // split groups 1.. hand their partial O to group 0 through LDS (the tile buffers are free)
    if constexpr (KSPL > 1) {
        float* ob = reinterpret_cast<float*>(fsm);
        static_assert((size_t)(KSPL - 1) * RG * CT * 64 * 16 <= (size_t)KSPL * GRP * 2, "O exchange fits");
        if (ks > 0) {
#pragma unroll
            for (int c = 0; c < CT; ++c)
                *reinterpret_cast<f32x4*>(ob + ((((ks - 1) * RG + rg) * CT + c) * 64 + lane) * 4) = oacc[c];
        }
        __syncthreads();
        if (ks > 0) return;
#pragma unroll
        for (int q = 1; q < KSPL; ++q)
#pragma unroll
            for (int c = 0; c < CT; ++c)
                oacc[c] += *reinterpret_cast<const f32x4*>(ob + ((((q - 1) * RG + rg) * CT + c) * 64 + lane) * 4);
    }
    // C map: d = 16c + li, query row 4g + r of the wave's 16
    uint16_t* orow[4];
    attn_out_rows(a, b, kvh, blockIdx.x * (16 * RG) + rg * 16 + 4 * g, nrows, orow);
#pragma unroll
    for (int c = 0; c < CT; ++c) {
        const int d = c * 16 + li;
        if (d >= HD) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (orow[r]) orow[r][d] = f2bf(oacc[c][r]);
    }
}

// ---------------------------------------------------------------- prefill, short key range, one pass
// SigLIP at 224 px (256 keys, d 72): one 4-wave workgroup per 16 query rows of one head; wave w owns
// keys [64 w, 64 w + 64).  Every load of the workgroup is issued before the first is consumed: Q and
// the wave's K fragments straight into registers (MFMA layout, L2-served: each head's K/V is read by
// its 16 workgroups), V by LDS-DMA into a dense [key][80] image (160-B rows: the transposed P.V reads
// are bank-conflict free).  Scores stay in registers (no second pass over the keys); the exact
// softmax's row max and sum meet across the 4 waves in LDS in a fixed order; each wave multiplies its
// own keys' p = bf16(exp(s - M) / L) by V, and the 4 partial O tiles are summed in a fixed order and
// rounded once -- the rounding points of k_attn_fa (s = bf16(bf16(k.q) * scale), p rounded after
// normalisation, O rounded once), one global round trip instead of one per 32-key tile and pass.
template <int HD, int MAXT>
__global__ void __launch_bounds__(256) k_attn_short(AttnArgs a) {
    using I = FAInfo<HD>;
    constexpr int KS = I::KS, CT = I::CT, CH = I::CH;
    constexpr int W = 4, KPW = 16 * MAXT, NK = W * KPW;
    constexpr int VRS = CT * 16, VCH = VRS / 8;  // V image row: CT 16-column tiles, VCH 16-B chunks
    static_assert(MAXT % 2 == 0, "whole 32-key P.V chunks per wave");
    __shared__ __attribute__((aligned(16))) uint16_t Vl[NK * VRS];
    __shared__ float red[2][W][16];
    __shared__ __attribute__((aligned(16))) f32x4 ob[W - 1][CT][64];

    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, li = lane & 15;
    const int b = blockIdx.z, kvh = blockIdx.y;
    const int row0 = blockIdx.x * 16, nrows = a.Lq * a.G;
    const int qi = row0 + li;
    const bool qvalid = qi < nrows;
    const int qpos = qvalid ? qi / a.G : 0, qhead = kvh * a.G + (qvalid ? qi % a.G : 0);
    const uint16_t* qrow = a.q + b * a.q_b_stride + (long)qpos * a.q_row_stride + qhead * a.q_head_stride;
    const uint16_t* kbase = a.k + b * a.k_b_stride + kvh * a.k_head_stride;
    const uint16_t* vbase = a.v + b * a.v_b_stride + kvh * a.v_head_stride;
    const int key0 = wave * KPW;

    // ---- loads: Q and this wave's K fragments (registers), then the V image (LDS-DMA, all waves)
    short8 qf[KS], kf[MAXT][KS];
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) qf[kk] = load_frag<HD>(qrow, qvalid, kk, lane);
#pragma unroll
    for (int t = 0; t < MAXT; ++t) {
        int key = key0 + 16 * t + li;
        key = key < a.Lk ? key : a.Lk - 1;  // rows past the keys: a valid row, score masked below
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) kf[t][kk] = load_frag<HD>(kbase + (long)key * a.k_row_stride, true, kk, lane);
    }
    const int vrows = (a.Lk + 31) & ~31;                  // whole 32-key chunks; rows * VCH is a multiple of 64
    const int n_ins = vrows * VCH / 64;
    for (int i = wave; i < n_ins; i += W) {
        const int e = i * 64 + lane;
        int key = e / VCH, ch = e % VCH;
        key = key < a.Lk ? key : a.Lk - 1;               // p = 0 there
        ch = ch < CH ? ch : CH - 1;                        // pad columns (never stored): a copy of the last chunk
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(vbase + (long)key * a.v_row_stride + ch * 8),
                                         (__attribute__((address_space(3))) void*)(Vl + i * 64 * 8), 16, 0, 0);
    }

    // ---- S^T = K Q^T for the wave's keys: lane holds keys 16 t + 4 g + r of query li
    float sc[MAXT][4];
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < MAXT; ++t) {
        f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
            if (kk & 1) a1 = mfma16(kf[t][kk], qf[kk], a1);
            else a0 = mfma16(kf[t][kk], qf[kk], a0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int key = key0 + 16 * t + 4 * g + r;
            const float v = rbf(rbf(a0[r] + a1[r]) * a.scale);
            sc[t][r] = key < a.Lk ? v : -INFINITY;
            mx = fmaxf(mx, sc[t][r]);
        }
    }
    // ---- exact softmax statistics: lane groups g, then the 4 waves in a fixed order
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    if (g == 0) red[0][wave][li] = mx;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's V DMAs landed (visible after the barrier)
    __syncthreads();
    const float M = fmaxf(fmaxf(red[0][0][li], red[0][1][li]), fmaxf(red[0][2][li], red[0][3][li]));
    float sm = 0.f;
#pragma unroll
    for (int t = 0; t < MAXT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            sc[t][r] = sc[t][r] == -INFINITY ? 0.f : fa_exp(sc[t][r] - M);
            sm += sc[t][r];
        }
    sm += __shfl_xor(sm, 16, 64);
    sm += __shfl_xor(sm, 32, 64);
    if (g == 0) red[1][wave][li] = sm;
    __syncthreads();
    const float invl = 1.0f / (((red[1][0][li] + red[1][1][li]) + red[1][2][li]) + red[1][3][li]);

    // ---- O = sum over this wave's 32-key chunks of bf16(p) . V (k_attn_fa's key order in the fragment)
    f32x4 oacc[CT];
#pragma unroll
    for (int c = 0; c < CT; ++c) oacc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ch = 0; ch < MAXT / 2; ++ch) {
        // chunks past the staged rows (keys >= Lk rounded up to 32) hold no V: p is 0 there, but
        // the unwritten LDS could hold non-finite bit patterns (0 * NaN), so they are skipped
        // (wave-uniform: no lane diverges)
        if (key0 + 32 * ch >= vrows) break;
        short8 pa;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int j = 0; j < 4; ++j) pa[kt * 4 + j] = (short)f2bf(sc[2 * ch + kt][j] * invl);
        const uint16_t* vb0 = Vl + (key0 + 32 * ch + 4 * g + (li >> 2)) * VRS + 4 * (li & 3);
#pragma unroll
        for (int c = 0; c < CT; ++c) {
            const s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v*)(vb0 + c * 16));
            const s4v hi =
                __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v*)(vb0 + 16 * VRS + c * 16));
            const short8 vb = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            oacc[c] = mfma16(pa, vb, oacc[c]);
        }
    }
    // ---- the 4 partial O tiles, summed in wave order, rounded once
    if (wave > 0) {
#pragma unroll
        for (int c = 0; c < CT; ++c) ob[wave - 1][c][lane] = oacc[c];
    }
    __syncthreads();
    if (wave > 0) return;
#pragma unroll
    for (int q = 0; q < W - 1; ++q)
#pragma unroll
        for (int c = 0; c < CT; ++c) oacc[c] += ob[q][c][lane];
    uint16_t* orow[4];
    attn_out_rows(a, b, kvh, row0 + 4 * g, nrows, orow);
#pragma unroll
    for (int c = 0; c < CT; ++c) {
        const int d = c * 16 + li;
        if (d >= HD) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (orow[r]) orow[r][d] = f2bf(oacc[c][r]);
    }
}

// ---------------------------------------------------------------- prefill, one pass, keys split over workgroups
// For the long prefills (Gemma and SigLIP at 448 px, L ~ 1,056): k_attn_fa reads every key's K twice
// and V once per 64 query rows, and with all keys in one workgroup only ~130 workgroups exist, each
// pulling ~1.6 MB through its CU (~30 GB/s per CU: the kernel is bound by that intake, MFMA busy
// < 0.1).  Here a workgroup owns QB = NW x 16 query rows (MQA: the G heads of a KV head are rows of
// the same tiles) and one of `ns` contiguous key ranges; K and V reach LDS by LDS-DMA into an
// ST-slot ring filled by LW loader waves (counted vmcnt, one raw s_barrier per 32-key tile); the NW
// compute waves run S^T = K Q^T, an online softmax and P.V on MFMA.  Each workgroup writes its
// unnormalised O (fp32) and its per-row (max, sum) to scratch; k_attn_fs_combine merges the key
// ranges in a fixed order (ns == 1: the workgroup normalises and stores bf16 itself).
// Rounding: s = bf16(bf16(k.q) * scale) as the reference; p is rounded to bf16 as exp(s - m) with m
// the workgroup's running row max (deferred: raised only when a tile's max passes it by kFsDefer,
// e <= e^8 in between) and normalised in fp32 at the end, where the reference rounds the globally
// normalised p -- the flash-decoding deviation of the decode step.
// LDS images (rows of CR 16-B chunks): K chunk c of key row r at chunk c ^ (r & 15) (conflict-free
// ds_read_b128 of 16 rows x one 16-B k slice); V chunk c at chunk c ^ ((r & 7) << 1) (the
// ds_read_b64_tr_b16 reads of 8 rows x 32 B per half-wave hit 8 distinct 32-B bank groups).  The
// swizzle is applied to each lane's SOURCE address (the LDS-DMA destination is lane-linear); chunks
// past the head dim (HD 72) load a copy of chunk 0 (finite; multiplied by Q's zeroed k range, or
// feeding output columns that are never stored).
template <int HD>
struct FSInfo {
    static constexpr int KS = (HD + 31) / 32;        // 32-deep k-steps of K.Q
    static constexpr int CT = (HD + 15) / 16;        // 16-wide output tiles of P.V
    static constexpr int CH = (HD + 7) / 8;          // 16-B chunks of a head row in HBM
    static constexpr int CR = HD <= 128 ? 16 : 32;   // 16-B chunks of an LDS row
    static constexpr int ROWB = CR * 16;
    static constexpr int TILEB = 32 * ROWB;          // one 32-key K (or V) image
    static constexpr int SLOTB = 2 * TILEB;          // ring slot: K image, then V image
    static constexpr int PCS = SLOTB / 1024;         // 1-KiB LDS-DMA pieces per slot
    static_assert(CR >= 4 * KS && CR >= 2 * CT && CR >= 16, "LDS row holds every k-step and tile");
};
constexpr float kFsDefer = 8.0f;

template <int G, int NMAX>
__device__ __forceinline__ void fs_vm_wait(int n) {  // s_waitcnt vmcnt(G * min(n, NMAX))
    if constexpr (NMAX >= 1) {
        if (n >= NMAX) {
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G * NMAX) : "memory");
            return;
        }
        fs_vm_wait<G, NMAX - 1>(n);
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

// grid (row blocks, n_kv * ns, B); key range sp = blockIdx.y % ns covers tiles [sp * tps, (sp + 1) * tps)
// P2: scale is a power of two (Gemma: 1/16), so bf16(bf16(x) * scale) = bf16(x) * scale (one rounding)
template <int HD, int NW, int LW, int ST, bool P2>
__global__ void __launch_bounds__(64 * (NW + LW), 1) k_attn_fs(AttnArgs a, int ns, int tps) {
    using I = FSInfo<HD>;
    constexpr int KS = I::KS, CT = I::CT, CH = I::CH, CR = I::CR, ROWB = I::ROWB, TILEB = I::TILEB;
    constexpr int SLOTB = I::SLOTB, PCS = I::PCS, GPW = PCS / LW;
    constexpr int QB = NW * 16;
    static_assert(PCS % LW == 0, "whole pieces per loader wave");
    extern __shared__ __attribute__((aligned(16))) uint8_t fs_sm[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int b = blockIdx.z, kvh = blockIdx.y / ns, sp = blockIdx.y % ns;
    const int nt = (a.Lk + 31) / 32;
    const int t0 = sp * tps;
    const int t1 = t0 + tps < nt ? t0 + tps : nt;
    const int ntl = t1 > t0 ? t1 - t0 : 0;
    const uint16_t* kbase = a.k + b * a.k_b_stride + kvh * a.k_head_stride;
    const uint16_t* vbase = a.v + b * a.v_b_stride + kvh * a.v_head_stride;

    if (wave >= NW) {
        // ---------------- loader wave: pieces lw, lw + LW, ... of every slot
        const int lw = wave - NW;
        constexpr int RPP = 1024 / ROWB;  // key rows per piece
        int loff[GPW], prow[GPW], pch[GPW];
        bool pv[GPW];
#pragma unroll
        for (int i = 0; i < GPW; ++i) {
            const int p = lw + LW * i;
            pv[i] = p >= PCS / 2;
            const int q = pv[i] ? p - PCS / 2 : p;
            loff[i] = (pv[i] ? TILEB : 0) + q * 1024;
            const int r = q * RPP + lane / CR, pos = lane % CR;
            const int c = pv[i] ? pos ^ ((r & 7) << 1) : pos ^ (r & 15);
            pch[i] = c < CH ? c : 0;
            prow[i] = r;
        }
        auto issue = [&](int t, int slot) {
#pragma unroll
            for (int i = 0; i < GPW; ++i) {
                int key = t * 32 + prow[i];
                key = key < a.Lk ? key : a.Lk - 1;  // rows past the keys: a valid row, masked (s = -inf)
                const uint16_t* src =
                    (pv[i] ? vbase + (long)key * a.v_row_stride : kbase + (long)key * a.k_row_stride) + pch[i] * 8;
                __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src),
                                                 (__attribute__((address_space(3))) void*)(fs_sm + slot * SLOTB + loff[i]),
                                                 16, 0, 0);
            }
        };
#pragma unroll
        for (int sI = 0; sI < ST - 1; ++sI)
            if (sI < ntl) issue(t0 + sI, sI);
        int slot_next = ST - 1;  // slot of tile it + ST - 1
        for (int it = 0; it < ntl; ++it) {
            // barrier it: tiles it and it + 1 landed (the compute waves multiply K of it + 1 while
            // they finish tile it); the slot refilled after it held tile it - 1, done with at barrier it
            const int issued = ntl < it + ST - 1 ? ntl : it + ST - 1;
            const int need = it + 1 < ntl ? it + 1 : ntl - 1;
            fs_vm_wait<GPW, ST - 3>(issued - need - 1);
            __builtin_amdgcn_s_barrier();
            if (it + ST - 1 < ntl) issue(t0 + it + ST - 1, slot_next);
            slot_next = slot_next + 1 == ST ? 0 : slot_next + 1;
        }
        return;
    }

    // ---------------- compute wave: query rows rbase + li (16 per wave)
    const int g = lane >> 4, li = lane & 15;
    const int nrows = a.Lq * a.G;
    const int rbase = blockIdx.x * QB + wave * 16;
    short8 qf[KS];
    {
        int qi = rbase + li;
        qi = qi < nrows ? qi : nrows - 1;  // rows past the end: a valid row, never stored
        const int qpos = qi / a.G, qhead = kvh * a.G + qi % a.G;
        const uint16_t* qrow = a.q + b * a.q_b_stride + (long)qpos * a.q_row_stride + qhead * a.q_head_stride;
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) qf[kk] = load_frag<HD>(qrow, true, kk, lane);
    }
    f32x4 o[CT];
#pragma unroll
    for (int c = 0; c < CT; ++c) o[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    // row li's running (deferred) max -- finite from the start, so exp(s - m) of a masked key (s = -inf)
    // is 0 and the first tile's rescale factor exp(m - tm) is 0 without a special case -- and this
    // lane's share of the row sum
    float m = -1e30f, l = 0.f;
    // P.V operand: lane reads rows vr0 (lo) and vr0 + 16 (hi), columns 16c + 4 (li & 3) .. + 3
    const int vr0 = 4 * g + (li >> 2);
    const int vsw = (vr0 & 7) << 1;
    // S^T = K Q^T of the tile in `sl`: lane holds keys 16 kt + 4 g + j of query li; even / odd
    // k-steps accumulate in two chains
    auto scores = [&](int sl, f32x4 (&ac)[2][2]) {
        const uint8_t* kb = fs_sm + sl * SLOTB;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) ac[kt][0] = ac[kt][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < KS; ++kk)
#pragma unroll
            for (int kt = 0; kt < 2; ++kt) {
                const int r = kt * 16 + li;
                const short8 kf = *reinterpret_cast<const short8*>(kb + r * ROWB + (((kk * 4 + g) ^ (r & 15)) << 4));
                ac[kt][kk & 1] = mfma16(kf, qf[kk], ac[kt][kk & 1]);
            }
    };
    // s = bf16(bf16(k.q) * scale), keys past Lk masked (the last tile only: wave-uniform branch);
    // returns the tile's max of row li
    auto finish = [&](int t, const f32x4 (&ac)[2][2], float (&sv)[2][4]) -> float {
        float mx = -INFINITY;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float x = rbf(ac[kt][0][j] + ac[kt][1][j]);
                sv[kt][j] = P2 ? x * a.scale : rbf(x * a.scale);
            }
        if (t * 32 + 32 > a.Lk) {
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (t * 32 + kt * 16 + 4 * g + j >= a.Lk) sv[kt][j] = -INFINITY;
        }
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int j = 0; j < 4; ++j) mx = fmaxf(mx, sv[kt][j]);
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        return fmaxf(mx, __shfl_xor(mx, 32, 64));
    };
    // one tile ahead: iteration it multiplies K of tile it + 1 while it runs the softmax and P.V of
    // tile it (the two are independent, so the MFMAs of one overlap the VALU of the other)
    float s[2][4], tm = -INFINITY;
    if (ntl > 0) {
        __builtin_amdgcn_s_barrier();  // barrier 0: tiles 0 and 1 landed
        f32x4 ac[2][2];
        scores(0, ac);
        tm = finish(t0, ac, s);
    }
    int slot = 0;
    for (int it = 0; it < ntl; ++it) {
        if (it > 0) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every read of the slot refilled next is done
            __builtin_amdgcn_s_barrier();                         // tiles it and it + 1 in the ring
        }
        const int nslot = slot + 1 == ST ? 0 : slot + 1;
        f32x4 acn[2][2];
        scores(nslot, acn);  // tile it + 1 (past the last tile: stale LDS, never used)
        // deferred running max: raised (and O, l rescaled) only when a row's tile max passes it by
        // kFsDefer; wave-uniform branch
        if (__ballot(tm > m + kFsDefer)) {
            const float mn = fmaxf(m, tm);
            const float alpha = fa_exp(m - mn);
            l *= alpha;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float ar = __shfl(alpha, 4 * g + r, 64);  // O rows are queries 4g + r
#pragma unroll
                for (int c = 0; c < CT; ++c) o[c][r] *= ar;
            }
            m = mn;
        }
        short8 pa;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float e = fa_exp(s[kt][j] - m);  // masked: exp(-inf) = 0
                l += e;
                pa[kt * 4 + j] = (short)f2bf(e);
            }
        const uint8_t* vb = fs_sm + slot * SLOTB + TILEB;
#pragma unroll
        for (int c = 0; c < CT; ++c) {
            const int cidx = 2 * c + ((li & 3) >> 1);
            const uint8_t* pl = vb + vr0 * ROWB + ((cidx ^ vsw) << 4) + (li & 1) * 8;
            const s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v*)pl);
            const s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v*)(pl + 16 * ROWB));
            const short8 vv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            o[c] = mfma16(pa, vv, o[c]);
        }
        tm = finish(t0 + it + 1, acn, s);
        slot = nslot;
    }
    // row sums: the 4 lane groups of query li, in a fixed order
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    if (ns == 1) {
        const float inv = 1.0f / l;
        uint16_t* orow[4];
        attn_out_rows(a, b, kvh, rbase + 4 * g, nrows, orow);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float ir = __shfl(inv, 4 * g + r, 64);
#pragma unroll
            for (int c = 0; c < CT; ++c) {
                const int d = c * 16 + li;
                if (d < HD && orow[r]) orow[r][d] = f2bf(o[c][r] * ir);
            }
        }
        return;
    }
    // key-split partials: O rows [(b, kvh, sp)][row][HD] fp32, then (m, l) pairs
    const long rec = ((long)(b * a.n_kv + kvh) * ns + sp) * nrows;
    float* part = a.ws;
    float* ml = a.ws + (long)a.B * a.n_kv * ns * nrows * HD;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int row = rbase + 4 * g + r;
        if (row >= nrows) continue;
#pragma unroll
        for (int c = 0; c < CT; ++c) {
            const int d = c * 16 + li;
            if (d < HD) part[(rec + row) * HD + d] = o[c][r];
        }
    }
    if (g == 0 && rbase + li < nrows) {
        ml[(rec + rbase + li) * 2 + 0] = m;
        ml[(rec + rbase + li) * 2 + 1] = l;
    }
}

// merge the key ranges of k_attn_fs in range order: O = sum_sp w_sp O_sp / sum_sp w_sp l_sp,
// w_sp = exp(m_sp - max m); one thread per 8 output columns of a row
template <int HD>
__global__ void __launch_bounds__(256) k_attn_fs_combine(AttnArgs a, int ns) {
    constexpr int C8 = HD / 8;
    const int nrows = a.Lq * a.G;
    const long e = (long)blockIdx.x * 256 + threadIdx.x;
    if (e >= (long)a.B * a.n_kv * nrows * C8) return;
    const int c8 = (int)(e % C8);
    long rr = e / C8;
    const int row = (int)(rr % nrows);
    rr /= nrows;
    const int kvh = (int)(rr % a.n_kv), b = (int)(rr / a.n_kv);
    const float* ml = a.ws + (long)a.B * a.n_kv * ns * nrows * HD;
    const long rec0 = (long)(b * a.n_kv + kvh) * ns * nrows + row;
    float M = -INFINITY;
    for (int q = 0; q < ns; ++q) M = fmaxf(M, ml[(rec0 + (long)q * nrows) * 2]);
    float L = 0.f, acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int q = 0; q < ns; ++q) {
        const long r = rec0 + (long)q * nrows;
        const float mq = ml[r * 2], lq = ml[r * 2 + 1];
        const float w = mq == -INFINITY ? 0.f : fa_exp(mq - M);  // an empty range: O = 0, l = 0
        const f32x4 x0 = *reinterpret_cast<const f32x4*>(a.ws + r * HD + c8 * 8);
        const f32x4 x1 = *reinterpret_cast<const f32x4*>(a.ws + r * HD + c8 * 8 + 4);
        L += w * lq;
#pragma unroll
        for (int j = 0; j < 4; ++j) { acc[j] += w * x0[j]; acc[4 + j] += w * x1[j]; }
    }
    const float inv = 1.0f / L;
    u16x8 ob;
#pragma unroll
    for (int j = 0; j < 8; ++j) ob.v[j] = f2bf(acc[j] * inv);
    const int pos = row / a.G, head = kvh * a.G + row % a.G;
    *reinterpret_cast<u16x8*>(a.o + b * a.o_b_stride + (long)pos * a.o_row_stride + head * a.o_head_stride + c8 * 8) = ob;
}

// key ranges for k_attn_fs.  A workgroup takes the whole LDS (one per CU), so a grid past 256
// workgroups runs in two rounds: split the keys (2, 4, ...) only while the grid stays within one
// round and every range keeps >= 16 tiles (shorter ranges lose more to the combine than they gain);
// scratch for the partials or the split is dropped
static int fs_splits(const AttnArgs& a, int HD, int QB, int want) {
    const int nrows = a.Lq * a.G, nt = (a.Lk + 31) / 32;
    const long blocks = (long)(nrows + QB - 1) / QB * a.n_kv * a.B;
    int ns = 1;
    if (want > 0) ns = want;
    else
        while (blocks * ns * 2 <= 256 && nt / (ns * 2) >= 16) ns *= 2;
    if (ns > nt) ns = nt;
    while (ns > 1 && (!a.ws || (long)a.B * a.n_kv * ns * nrows * (HD + 2) > a.ws_floats)) ns >>= 1;
    return ns < 1 ? 1 : ns;
}

template <int HD, int NW, int LW, int ST, bool P2>
static void launch_fs_t(hipStream_t s, const AttnArgs& a, int ns, int tps, dim3 grid) {
    constexpr size_t lds = (size_t)ST * FSInfo<HD>::SLOTB;
    static_assert(lds <= 160 * 1024, "LDS");
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_attn_fs<HD, NW, LW, ST, P2>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr = true;
    }
    hipLaunchKernelGGL((k_attn_fs<HD, NW, LW, ST, P2>), grid, dim3(64 * (NW + LW)), lds, s, a, ns, tps);
}

template <int HD, int NWQ = 0>
static void launch_fs(hipStream_t s, const AttnArgs& a, int want_ns) {
    // head dim 256: 4 compute waves (their registers fit 2 waves per SIMD with the loaders, not 3) and a
    // 5-slot ring (160 KiB); head dim 72: 8 compute waves, 8 slots.  NWQ > 0: that many compute waves (fewer
    // query rows per workgroup, more workgroups over the same keys: probe variants 81 / 82)
    constexpr int NW = NWQ > 0 ? NWQ : HD == 256 ? 4 : 8, LW = 4, ST = HD == 256 ? 5 : 8;
    const int nrows = a.Lq * a.G, nt = (a.Lk + 31) / 32;
    int ns = fs_splits(a, HD, NW * 16, want_ns);
    const int tps = (nt + ns - 1) / ns;
    ns = (nt + tps - 1) / tps;  // no empty range
    dim3 grid((nrows + NW * 16 - 1) / (NW * 16), a.n_kv * ns, a.B);
    int e2 = 0;
    const bool p2 = std::frexp(a.scale, &e2) == 0.5f;
    if (p2) launch_fs_t<HD, NW, LW, ST, true>(s, a, ns, tps, grid);
    else launch_fs_t<HD, NW, LW, ST, false>(s, a, ns, tps, grid);
    if (ns > 1) {
        const long n8 = (long)a.B * a.n_kv * nrows * (HD / 8);
        hipLaunchKernelGGL(k_attn_fs_combine<HD>, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, s, a, ns);
    }
}

template <int HD, int RG, int KSPL>
static void launch_fa(hipStream_t s, const AttnArgs& a) {
    using I = FAInfo<HD>;
    constexpr size_t lds = (size_t)KSPL * 2 * 32 * (I::KRS + I::VS) * 2 + (size_t)KSPL * RG * 16 * 2 * 4;
    static_assert(lds <= 160 * 1024, "LDS");
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_attn_fa<HD, RG, KSPL, 1>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr = true;
    }
    dim3 grid((a.Lq * a.G + 16 * RG - 1) / (16 * RG), a.n_kv, a.B);
    hipLaunchKernelGGL((k_attn_fa<HD, RG, KSPL, 1>), grid, dim3(64 * RG * KSPL), lds, s, a);
}

// attention variant override (tuning hook pgmi_tune_attention): 0 = the 16-row kernel, 7 = the
// one-pass short-range kernel (HD 72, <= 256 keys), 8 = the
// 16-row kernel with every load up front (HD 256, <= 320 keys), RK = the tiled kernel with RG = R,
// KSPL = K (41, 42, 21, 22; 44 and 24 for HD 72); -1 = the measured choice in attention_prefill.
// Every variant is forced and checked against the oracle by tests/test_gpu_ops.py.
static int g_attn_force = -1;

void attention_force_variant(int v) { g_attn_force = v; }

template <int HD>
static void launch_fa_variant(hipStream_t s, const AttnArgs& a, int rk) {
    switch (rk) {
        case 41: launch_fa<HD, 4, 1>(s, a); return;
        case 21: launch_fa<HD, 2, 1>(s, a); return;
        case 22: launch_fa<HD, 2, 2>(s, a); return;
        case 44: if constexpr (HD == 72) { launch_fa<HD, 4, 4>(s, a); return; } break;
        case 24: if constexpr (HD == 72) { launch_fa<HD, 2, 4>(s, a); return; } break;
        default: break;
    }
    launch_fa<HD, 4, 2>(s, a);  // 42
}

static size_t attn_full_lds(int head_dim, int Lk) {
    const int LkP = (Lk + 31) & ~31;
    const int hdp = (head_dim + 15) / 16 * 16;
    return (size_t)16 * LkP * 4 + (size_t)16 * LkP * 2 + (size_t)2 * 32 * (hdp + 16) * 2;
}

void attention_prefill(hipStream_t s, int head_dim, const AttnArgs& a) {
    int v = g_attn_force;
    if (v < 0) {
        // measured on MI355X (tools/probes/attn_bench.py, round 1), us per call:
        //   SigLIP 224 (256 rows x 16 heads):  16-row 16.4 | RG2xKSPL4 10.8 | RG4xKSPL2 13.5
        //   SigLIP 448 (1024 x 16):            16-row 153.5 | RG4xKSPL4 32.4 | RG4xKSPL2 36.0
        //   Gemma 224 (288 x 8 heads, MQA):    16-row 21.9 | RG4xKSPL2 26.1 | RG2xKSPL2 26.4
        //   Gemma 448 (1056 x 8):              16-row 159.5 | RG4xKSPL2 61.3 | RG2xKSPL2 122.7
        // round 3 (same probe, graph-replayed): the one-pass key-split kernel k_attn_fs (variant 9)
        //   Gemma 224 12.2 (full_pre 15.1) | Gemma 448 31.7 (tiled RG4xKSPL2 52.5) | SigLIP 448 24.4 (31.8);
        //   SigLIP 224 stays on k_attn_short at one image (6.7 against 10.6); at 8 images
        //   (tools/probes/plan_sweep.py --batch 8, whole tower) k_attn_fs: tower 4204 -> 3835 us
        const long rows = (long)a.Lq * a.G * a.n_kv * a.B;
        v = head_dim == 256 ? 9 : (a.Lk <= 256 && rows <= 4096) ? 7 : 9;
        // round 6: Gemma at one 224 px image (288 queries x 8 heads, 288 keys: no key split, 36 workgroups of
        // 4 compute waves) takes 2 compute waves per workgroup, 72 workgroups over the same keys: in situ LM
        // prefill 2,408.7 -> 2,394.0 us (gpurun_out r6g, variant 82; 1 wave, 81: 2,396.0)
        if (head_dim == 256 && (a.Lk + 31) / 32 < 16 && (rows + 31) / 32 <= 256) v = 82;
    }
    if ((v == 81 || v == 82) && head_dim == 256) {  // one pass, 1 / 2 compute waves per workgroup, one key range
        if (v == 81) launch_fs<256, 1>(s, a, 1);
        else launch_fs<256, 2>(s, a, 1);
        return;
    }
    if (v == 9 || v == 91 || v == 92 || v == 94) {  // one pass, keys split over workgroups (auto / 1 / 2 / 4 ranges)
        const int want = v == 9 ? 0 : v - 90;
        if (head_dim == 256) launch_fs<256>(s, a, want);
        else launch_fs<72>(s, a, want);
        return;
    }
    if (v == 7 && head_dim == 72 && a.Lk <= 256) {
        dim3 grid((a.Lq * a.G + 15) / 16, a.n_kv, a.B);
        hipLaunchKernelGGL((k_attn_short<72, 4>), grid, dim3(256), 0, s, a);
        return;
    }
    if (v == 7) v = head_dim == 256 ? 42 : 24;  // forced on a shape it does not cover: the tiled kernel
    if (v == 8 && head_dim == 256 && a.Lk <= 320) {
        // 16 query rows per workgroup, every K/V load issued up front (Lk <= 320)
        const size_t lds = (size_t)16 * ((a.Lk + 31) & ~31) * 2 + (size_t)2 * 32 * (256 + 16) * 2 + 2 * 4 * 16 * 4;
        dim3 grid((a.Lq * a.G + 15) / 16, a.n_kv, a.B);
        hipLaunchKernelGGL((k_attn_full_pre<256, 5, 10>), grid, dim3(256), lds, s, a);
        return;
    }
    if (v == 8) v = 0;
    if (v != 0 || a.Lk > attention_prefill_max_keys(head_dim)) {
        if (head_dim == 256) launch_fa_variant<256>(s, a, v);
        else launch_fa_variant<72>(s, a, v);
        return;
    }
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
    attn_decode_block(a, st, part, max_chunks, blockIdx.x, blockIdx.y, blockIdx.z, lds);
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
