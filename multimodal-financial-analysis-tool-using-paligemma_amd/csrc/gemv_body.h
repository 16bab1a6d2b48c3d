#pragma once
// gemv_body.h -- KV-cached decode projections (batch B <= 8 rows), gfx950.
//
// Decode at batch 1 streams ~5.02 GB of weights per token, so every
// projection of GemmaDecoderLayer (modeling_gemma.py:307-338) is one HBM-bound pass over
// its nn.Linear weight [N][K] (K contiguous, used as stored):
//   - each wave owns RPW "units" (1 row, or a row pair: RoPE's (d, d+128) or GeGLU's
//     (gate n, up n)); lane l covers K elements [8l + 512c, +8) for c < K/512, so one
//     wave-instruction reads 1 KiB contiguous of a row (16 B per lane, non-temporal);
//   - the activation (B x K, bf16) is staged once per workgroup in LDS, with the
//     preceding RMSNorm fused into that prologue (modeling_gemma.py:114-120);
//   - the first unit group's weight loads are issued BEFORE the prologue, and the next
//     group's before the current group's reduction/epilogue;
//   - fp32 accumulation via v_dot2_f32_bf16, one wave reduction per output;
//   - the reference's rounding points live in the epilogues (RoPE: modeling_gemma.py:
//     197-198, KV append :259, residual :327/:336, GeGLU :134, logits :417-418).
#include <type_traits>

#include "coh.h"
#include "common.h"
#include "launch.h"

namespace pgmi {

enum GemvMode : int { GV_QKV = 0, GV_RES = 1, GV_GEGLU = 2, GV_LOGITS = 3, GV_ORES = 4 };

struct GemvArgs {
    const uint16_t* x;       // activation rows [nb][K] (h for the norm'd modes)
    const uint16_t* norm_w;  // RMSNorm weight (nullptr: plain copy)
    float eps;
    const uint16_t* W;       // weight rows
    int n_units;
    int K;
    int nb;                  // valid batch rows (<= template B)
    int I;                   // GeGLU: up rows offset; QKV: number of q heads
    // outputs
    uint16_t* out;           // RES: h in/out [nb][N]; GEGLU: act [nb][I]; QKV: q [nb][nh*256]
    float* logits;           // LOGITS: [nb][N]
    float* pmax;             // LOGITS: per-block partial max [nb][gridDim]
    int* pidx;
    // LOGITS (decode): the last workgroup to finish folds every block's partial into next[b]
    // (torch.argmax first max, inference.py:68) and advances *adv by one step -- the work of
    // k_argmax_finish without its launch.  done: arrival counter, re-armed to 0 by that block.
    unsigned* done;
    int64_t* next;
    StepState* adv;
    int64_t* hist;  // (may be null) also receives next[b]: a multi-step graph's token record (pgmi_decode_steps)
    // QKV
    const uint16_t* cosT;
    const uint16_t* sinT;
    int max_pos;
    const StepState* st;
    uint16_t* kc;
    uint16_t* vc;
    long kv_b_stride;
    int nkv;
    // ORES: decode-attention partials (kernels_attn.hip) combined in the prologue
    const float* part;
    int max_chunks;
    int G;
    uint16_t* o_out;
    // QKV of decode layer 0 (EMB kernels): x is the token's embedding row, bf16(E[id] * normalizer)
    // (modeling_gemma.py:565,368; a pad id gives a zero row), read here instead of from a separate
    // embedding launch; workgroup 0 also stores it to emb_out (the layer's residual h)
    const int64_t* ids;
    const uint16_t* E;
    float normalizer;
    int64_t pad_id;
    uint16_t* emb_out;
    // batched decode (MFMA forms, B >= 3): the post-attention RMSNorm's sum of squares, carried from
    // o_proj to gate|up instead of a k_rows_norm pass.  GV_RES (one K slice) writes each row's partial
    // over its 16-column unit group, [nb][K / 16]; GV_GEGLU (unstaged) reads them, x being the raw h
    float* ssq;
    // batched decode (MFMA forms): the weight matrix's fragment-major image (k_mf_swizzle, built at prepare),
    // read instead of W when set (gate|up: the gate rows' image, then the up rows')
    const uint16_t* Wf;
};

// WK waves split one unit group's K range (WK = 4 for the 16384-wide down_proj), their
// partial sums meet in LDS; 4/WK unit groups per workgroup.
// XREG: the activation lives in registers (lane's own K chunks), the RMSNorm is computed
// per wave (WK == 1: every wave holds the whole row), no LDS staging / barrier; used when
// B * K/(512*WK) chunks fit in 32 VGPRs.  Otherwise the activation is staged in LDS.
template <int B, int KCH, int RPW, int MODE, int WK, bool XREG, int DEPTH = 1, bool EMB = false>
__device__ __forceinline__ void gemv_block(const GemvArgs& a, const int blk, const int nblk, uint16_t* xs) {
    static_assert(!EMB || (MODE == GV_QKV && XREG && WK == 1), "embedding fold: register-held q|k|v input only");
    constexpr int NR = (MODE == GV_QKV || MODE == GV_GEGLU) ? 2 : 1;
    constexpr int KCW = KCH / WK;  // chunks per wave
    constexpr int NL = RPW * NR * KCW;
    constexpr int K = KCH * 512;
    constexpr int GPB = 4 / WK;    // unit groups per block
    // the latency-bound projections (q|k|v, o_proj: 18.9 MB a layer) read their weights with the default
    // cache policy when PGMI_SMALL_NT=0 (probe build): the 4.9 GB of streamed weights stay
    // non-temporal, so the small ones may stay resident in the Infinity Cache across decode steps
#ifndef PGMI_SMALL_NT
#define PGMI_SMALL_NT 1
#endif
    constexpr bool kSmallTemporal = !PGMI_SMALL_NT && (MODE == GV_QKV || MODE == GV_ORES);
    __shared__ float red[4][B];
    __shared__ float kred[WK > 1 ? 4 : 1][RPW * NR * B];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wk = wave % WK, grp = wave / WK;
    // unit groups of this workgroup: interleaved over the grid
    const int stride = nblk * GPB * RPW;
    int bb = blk * GPB * RPW;  // block-uniform loop base
    const int bend = a.n_units;
    int ub = bb + grp * RPW;
    const int kofs = wk * KCW * 512 + 8 * lane;

    auto row_of = [&](int u, int j) -> long {
        if constexpr (MODE == GV_QKV) return (long)((u >> 7) * 256 + (u & 127) + j * 128);
        else if constexpr (MODE == GV_GEGLU) return (long)u + (long)j * a.I;
        else return (long)u;
    };

    // DEPTH register sets of weight rows: groups g+1 .. g+DEPTH-1 stay in flight while group g
    // is reduced (statically indexed: the loop below is unrolled by DEPTH)
    uint4 w[DEPTH][NL];
    auto issue = [&](auto slot, int base) {
        constexpr int SL = decltype(slot)::value;
#pragma unroll
        for (int i = 0; i < RPW; ++i) {
            int u = base + i;
            if (u >= bend) u = bend - 1;  // clamp: duplicate work, result discarded
#pragma unroll
            for (int j = 0; j < NR; ++j) {
                const uint16_t* rp = a.W + row_of(u, j) * K + kofs;
#pragma unroll
                for (int c = 0; c < KCW; ++c)
                    w[SL][(i * NR + j) * KCW + c] = kSmallTemporal ? ldg16(rp + 512 * c) : ldg_nt(rp + 512 * c);
            }
        }
    };
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, DEPTH - 1>;
    // register-held activation (XREG) and its RMSNorm weights: loaded unconditionally (row
    // clamped) so no branch splits the loads; they go out BEFORE the
    // weight stream, so the norm is computed while the weights are in flight (vmcnt is in
    // order: a load issued after the weights could only be consumed after all of them landed)
    // the residual modes never normalise their input (down_proj / o_proj): no norm registers
    constexpr bool NORM = MODE != GV_RES && MODE != GV_ORES;
    uint4 xr[XREG ? B : 1][XREG ? KCW : 1];
    uint4 nw[XREG && NORM ? KCW : 1];
    auto load_x = [&]() {
        if constexpr (XREG && MODE != GV_ORES) {
#pragma unroll
            for (int b = 0; b < B; ++b) {
                const int bq = b < a.nb ? b : a.nb - 1;
                const uint16_t* xrow;
                if constexpr (EMB) {
                    const int64_t id = a.ids[bq];  // wave-uniform: a scalar load
                    xrow = a.E + (id == a.pad_id ? 0 : id) * (long)K;
                } else {
                    xrow = a.x + (long)bq * K;
                }
#pragma unroll
                for (int c = 0; c < KCW; ++c) xr[b][c] = ldx16<false>(xrow + kofs + 512 * c);
            }
            if (NORM && a.norm_w) {
#pragma unroll
                for (int c = 0; c < KCW; ++c) nw[c] = ldg16(a.norm_w + kofs + 512 * c);
            }
        }
    };
    // the latency-bound qkv projection fetches its activation first, so the RMSNorm overlaps
    // the weight flight (measured: the streaming modes lose a little by it -- same-box A/B,
    // tools/probes/decode_kernels.py -- and keep the weights-first order)
    constexpr bool XFIRST = MODE == GV_QKV;
    if constexpr (XFIRST) {
        load_x();
        // unconditional (issue clamps the unit): a branch around the stream would make the
        // compiler's in-order vmcnt model drain it before the activation can be used
        issue(S0{}, ub);
        if constexpr (DEPTH == 2) issue(S1{}, ub + stride);
        asm volatile("" ::: "memory");  // keep the weight stream ahead of the norm (no sinking past it)
    } else {
        issue(S0{}, ub);
        if constexpr (DEPTH == 2) issue(S1{}, ub + stride);
        load_x();
    }

    if constexpr (MODE == GV_ORES) {
        // (G <= 8 query heads of one KV head: PaliGemma's MQA, checked at pgmi_create)
        // x[b][h*256 + d] = bf16(sum_c e^(m_c - M) O_c[h][d] / sum_c e^(m_c - M) l_c), chunks in
        // a fixed order (the flash-decoding combine of k_attn_decode's partials)
        // every thread combines its own 8 outputs from the chunk records directly (stats and
        // partial rows in one round trip, no LDS staging of the weights, no barrier)
        const int nch = (a.st->kv_len + 1 + kAttnChunk - 1) / kAttnChunk;
        constexpr int CMAX = 12;  // chunks held in registers (768 keys); longer caches take two passes
        const int nitems = a.nb * K / 8;
        for (int e8 = tid; e8 < nitems; e8 += 256) {
            const int b = e8 / (K / 8), e = (e8 % (K / 8)) * 8;
            const int h = e >> 8;
            const float* pb = a.part + (long)b * a.max_chunks * kAttnPartStride + h * 256 + (e & 255);
            const float* sp = a.part + (long)b * a.max_chunks * kAttnPartStride + 16 * 256 + h;
            float o[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = 0.f;
            float M = -INFINITY, S = 0.f;
            if (nch <= CMAX) {
                f32x4 x0[CMAX], x1[CMAX];
                float mc[CMAX], lc[CMAX];
                // unconditional loads (chunk index clamped; records past nch are ignored below):
                // a guarded load per chunk compiled to a branch and a wait per chunk
#pragma unroll
                for (int c = 0; c < CMAX; ++c) {
                    const long cs = (long)(c < nch ? c : nch - 1) * kAttnPartStride;
                    x0[c] = ldxf4<false>(pb + cs);
                    x1[c] = ldxf4<false>(pb + cs + 4);
                    mc[c] = ldxf<false>(sp + cs);
                    lc[c] = ldxf<false>(sp + cs + 16);
                }
#pragma unroll
                for (int c = 0; c < CMAX; ++c)
                    if (c < nch) M = fmaxf(M, mc[c]);
#pragma unroll
                for (int c = 0; c < CMAX; ++c)
                    if (c < nch) {
                        const float w = expf(mc[c] - M);
                        S += w * lc[c];
#pragma unroll
                        for (int j = 0; j < 4; ++j) { o[j] += w * x0[c][j]; o[4 + j] += w * x1[c][j]; }
                    }
            } else {
                for (int c = 0; c < nch; ++c) M = fmaxf(M, ldxf<false>(sp + (long)c * kAttnPartStride));
                for (int c = 0; c < nch; ++c) {
                    const float w = expf(ldxf<false>(sp + (long)c * kAttnPartStride) - M);
                    S += w * ldxf<false>(sp + (long)c * kAttnPartStride + 16);
                    const f32x4 x0 = ldxf4<false>(pb + (long)c * kAttnPartStride);
                    const f32x4 x1 = ldxf4<false>(pb + (long)c * kAttnPartStride + 4);
#pragma unroll
                    for (int j = 0; j < 4; ++j) { o[j] += w * x0[j]; o[4 + j] += w * x1[j]; }
                }
            }
            u16x8 ob;
#pragma unroll
            for (int j = 0; j < 8; ++j) ob.v[j] = f2bf(o[j] / S);
            *reinterpret_cast<u16x8*>(xs + b * K + e) = ob;
            if (a.o_out && blk == 0) *reinterpret_cast<u16x8*>(a.o_out + (long)b * K + e) = ob;
        }
        for (int e8 = tid; e8 < (B - a.nb) * K / 8; e8 += 256)
            *reinterpret_cast<uint4*>(xs + a.nb * K + e8 * 8) = make_uint4(0, 0, 0, 0);
        __syncthreads();
    } else if constexpr (XREG) {
#pragma unroll
        for (int b = 0; b < B; ++b)  // rows past nb (clamped loads) contribute zeros
            if (b >= a.nb)
#pragma unroll
                for (int c = 0; c < KCW; ++c) xr[b][c] = make_uint4(0, 0, 0, 0);
        if constexpr (EMB) {
            // x = bf16(E[id] * normalizer) (a pad id: zeros), the residual stream of layer 0
#pragma unroll
            for (int b = 0; b < B; ++b) {
                const bool pad = a.ids[b < a.nb ? b : a.nb - 1] == a.pad_id;
#pragma unroll
                for (int c = 0; c < KCW; ++c) {
                    const uint16_t* e = reinterpret_cast<const uint16_t*>(&xr[b][c]);
                    u16x8 o;
#pragma unroll
                    for (int j = 0; j < 8; ++j) o.v[j] = pad ? (uint16_t)0 : f2bf(bf2f(e[j]) * a.normalizer);
                    xr[b][c] = *reinterpret_cast<const uint4*>(&o);
                    if (blk == 0 && wave == 0 && b < a.nb)
                        *reinterpret_cast<uint4*>(a.emb_out + (long)b * K + kofs + 512 * c) = xr[b][c];
                }
            }
        }
        if (NORM && a.norm_w) {  // WK == 1: the wave holds the whole row
#pragma unroll
            for (int b = 0; b < B; ++b) {
                float ss = 0.f;
#pragma unroll
                for (int c = 0; c < KCW; ++c) {
                    const uint16_t* e = reinterpret_cast<const uint16_t*>(&xr[b][c]);
#pragma unroll
                    for (int j = 0; j < 8; ++j) { const float f = bf2f(e[j]); ss += f * f; }
                }
                ss = wave_sum(ss);
                const float r = 1.0f / sqrtf(ss / (float)K + a.eps);
#pragma unroll
                for (int c = 0; c < KCW; ++c) {
                    const uint16_t* we = reinterpret_cast<const uint16_t*>(&nw[c]);
                    const uint16_t* e = reinterpret_cast<const uint16_t*>(&xr[b][c]);
                    u16x8 o;
#pragma unroll
                    for (int j = 0; j < 8; ++j) o.v[j] = f2bf((bf2f(e[j]) * r) * (1.0f + bf2f(we[j])));
                    xr[b][c] = *reinterpret_cast<const uint4*>(&o);
                }
            }
        }
    } else {
        // ---- prologue: stage (RMSNorm'd) activation rows in LDS
        float ss[B];
#pragma unroll
        for (int b = 0; b < B; ++b) ss[b] = 0.f;
        for (int c = tid * 8; c < K; c += 256 * 8) {
#pragma unroll
            for (int b = 0; b < B; ++b) {
                uint4 v = (b < a.nb) ? ldx16<false>(a.x + (long)b * K + c) : make_uint4(0, 0, 0, 0);
                *reinterpret_cast<uint4*>(xs + b * K + c) = v;
                if (a.norm_w) {
                    const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
                    for (int j = 0; j < 8; ++j) { float f = bf2f(e[j]); ss[b] += f * f; }
                }
            }
        }
        if (a.norm_w) {
#pragma unroll
            for (int b = 0; b < B; ++b) {
                float t = wave_sum(ss[b]);
                if (lane == 0) red[wave][b] = t;
            }
            __syncthreads();
            float r[B];
#pragma unroll
            for (int b = 0; b < B; ++b)
                r[b] = 1.0f / sqrtf((red[0][b] + red[1][b] + red[2][b] + red[3][b]) / (float)K + a.eps);
            for (int c = tid * 8; c < K; c += 256 * 8) {
                uint4 wv = ldg16(a.norm_w + c);
                const uint16_t* we = reinterpret_cast<const uint16_t*>(&wv);
#pragma unroll
                for (int b = 0; b < B; ++b) {
                    uint4 v = *reinterpret_cast<uint4*>(xs + b * K + c);
                    const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
                    u16x8 o;
#pragma unroll
                    for (int j = 0; j < 8; ++j) o.v[j] = f2bf((bf2f(e[j]) * r[b]) * (1.0f + bf2f(we[j])));
                    *reinterpret_cast<u16x8*>(xs + b * K + c) = o;
                }
            }
        }
        __syncthreads();
    }

    int kv_len = 0, pos = 0;
    if constexpr (MODE == GV_QKV) {
        kv_len = a.st->kv_len;
        pos = a.st->position;
        if (pos < 0) pos = 0;
        if (pos > a.max_pos - 1) pos = a.max_pos - 1;  // clamp (modeling_gemma.py:163-165)
    }
    float best[B];
    int besti[B];
#pragma unroll
    for (int b = 0; b < B; ++b) { best[b] = -INFINITY; besti[b] = 0x7fffffff; }

    // ISSUE: start the stream of group +DEPTH in this step.  The loop below peels the last group
    // (DEPTH 1) so the in-loop issue is unconditional: behind a branch the compiler cannot count
    // the loads in flight and waits vmcnt(0) -- for the next group's stream -- at the epilogue's
    // residual read
    auto step = [&](auto slot, auto issue_next) {
        constexpr int SL = decltype(slot)::value;
        constexpr bool ISSUE = decltype(issue_next)::value;
        // epilogue operands of this group (residual h, RoPE cos/sin), queued behind its weights
        float pre[RPW][B][2];
#pragma unroll
        for (int i = 0; i < RPW; ++i) {
            const int u = ub + i < bend ? ub + i : bend - 1;
#pragma unroll
            for (int b = 0; b < B; ++b) {
                const int bq = b < a.nb ? b : a.nb - 1;
                if constexpr (MODE == GV_RES || MODE == GV_ORES) {
                    pre[i][b][0] = bf2f(ldxh<false>(a.out + (long)bq * a.n_units + u));
                } else if constexpr (MODE == GV_QKV) {
                    pre[i][b][0] = bf2f(a.cosT[(long)pos * 128 + (u & 127)]);
                    pre[i][b][1] = bf2f(a.sinT[(long)pos * 128 + (u & 127)]);
                }
            }
        }
        float acc[RPW][NR][B];
#pragma unroll
        for (int i = 0; i < RPW; ++i)
#pragma unroll
            for (int j = 0; j < NR; ++j)
#pragma unroll
                for (int b = 0; b < B; ++b) acc[i][j][b] = 0.f;
#pragma unroll
        for (int c = 0; c < KCW; ++c) {
#pragma unroll
            for (int b = 0; b < B; ++b) {
                uint4 xv;
                if constexpr (XREG) xv = xr[b][c];
                else xv = *reinterpret_cast<const uint4*>(xs + b * K + kofs + 512 * c);
#pragma unroll
                for (int i = 0; i < RPW; ++i)
#pragma unroll
                    for (int j = 0; j < NR; ++j) acc[i][j][b] = dot8(w[SL][(i * NR + j) * KCW + c], xv, acc[i][j][b]);
            }
        }
        const int cur = ub;
        ub += stride;
        bb += stride;
        // the stream of group +DEPTH starts before this group's epilogue, into the freed set
        if constexpr (ISSUE) {
            if constexpr (DEPTH == 1) issue(slot, ub + (DEPTH - 1) * stride);
            else if (ub + (DEPTH - 1) * stride < bend) issue(slot, ub + (DEPTH - 1) * stride);
        }

#pragma unroll
        for (int i = 0; i < RPW; ++i)
#pragma unroll
            for (int j = 0; j < NR; ++j)
#pragma unroll
                for (int b = 0; b < B; ++b) acc[i][j][b] = wave_sum(acc[i][j][b]);
        if constexpr (WK > 1) {
            // combine the WK K-slices of each unit in a fixed order
            if (lane == 0) {
#pragma unroll
                for (int i = 0; i < RPW; ++i)
#pragma unroll
                    for (int j = 0; j < NR; ++j)
#pragma unroll
                        for (int b = 0; b < B; ++b) kred[wave][(i * NR + j) * B + b] = acc[i][j][b];
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < RPW; ++i)
#pragma unroll
                for (int j = 0; j < NR; ++j)
#pragma unroll
                    for (int b = 0; b < B; ++b) {
                        float t = 0.f;
#pragma unroll
                        for (int q = 0; q < WK; ++q) t += kred[grp * WK + q][(i * NR + j) * B + b];
                        acc[i][j][b] = t;
                    }
            __syncthreads();
            if (wk != 0) return;  // slice 0 of each group writes
        }

#pragma unroll
        for (int i = 0; i < RPW; ++i) {
            const int u = cur + i;
            if (u >= bend) break;
#pragma unroll
            for (int b = 0; b < B; ++b) {
                if (b >= a.nb) break;
                if constexpr (MODE == GV_RES || MODE == GV_ORES) {
                    if (lane == 0) {
                        stxh<false>(a.out + (long)b * a.n_units + u, f2bf(rbf(acc[i][0][b]) + pre[i][b][0]));
                    }
                } else if constexpr (MODE == GV_GEGLU) {
                    if (lane == 0) {
                        const float g = rbf(gelu_tanh(rbf(acc[i][0][b])));
                        stxh<false>(a.out + (long)b * a.I + u, f2bf(g * rbf(acc[i][1][b])));
                    }
                } else if constexpr (MODE == GV_LOGITS) {
                    const float v = rbf(acc[i][0][b]);
                    if (lane == 0) a.logits[(long)b * a.n_units + u] = v;
                    if (v > best[b]) { best[b] = v; besti[b] = u; }  // rows visited in increasing order
                } else {  // GV_QKV
                    if (lane == 0) {
                        const int hh = u >> 7, d = u & 127;
                        const float x0 = rbf(acc[i][0][b]), x1 = rbf(acc[i][1][b]);
                        const int nh = a.I;
                        if (hh < nh + a.nkv) {
                            const float c = pre[i][b][0];
                            const float sn = pre[i][b][1];
                            const uint16_t o0 = f2bf(rbf(x0 * c) + rbf(-x1 * sn));
                            const uint16_t o1 = f2bf(rbf(x1 * c) + rbf(x0 * sn));
                            uint16_t* dst;
                            if (hh < nh) {
                                dst = a.out + (long)b * nh * 256 + hh * 256;
                            } else {
                                dst = a.kc + b * a.kv_b_stride + (long)kv_len * (a.nkv * 256) + (hh - nh) * 256;
                            }
                            stxh<false>(dst + d, o0);
                            stxh<false>(dst + d + 128, o1);
                        } else {
                            uint16_t* dst = a.vc + b * a.kv_b_stride + (long)kv_len * (a.nkv * 256) +
                                            (hh - nh - a.nkv) * 256;
                            stxh<false>(dst + d, f2bf(x0));
                            stxh<false>(dst + d + 128, f2bf(x1));
                        }
                    }
                }
            }
        }
    };
    using Yes = std::true_type;
    using No = std::false_type;
    if constexpr (DEPTH == 1) {
        while (bb + stride < bend) step(S0{}, Yes{});  // a next group exists: stream it
        if (bb < bend) step(S0{}, No{});
    } else {
        while (bb < bend) {
            step(S0{}, Yes{});
            if (bb >= bend) break;
            step(S1{}, Yes{});
        }
    }

    if constexpr (MODE == GV_LOGITS) {
        // block-level first-max over the 4 waves, one partial per block
        __shared__ float bv[4][B];
        __shared__ int bi[4][B];
        if (lane == 0) {
#pragma unroll
            for (int b = 0; b < B; ++b) { bv[wave][b] = best[b]; bi[wave][b] = besti[b]; }
        }
        __syncthreads();
        if (tid == 0) {
#pragma unroll
            for (int b = 0; b < B; ++b) {
                if (b >= a.nb) break;
                float m = bv[0][b];
                int mi = bi[0][b];
                for (int q = 1; q < 4; ++q)
                    if (bv[q][b] > m || (bv[q][b] == m && bi[q][b] < mi)) { m = bv[q][b]; mi = bi[q][b]; }
                if (a.done) {  // write-through: the folding block may sit on another XCD
                    stf_coh(a.pmax + (long)b * nblk + blk, m);
                    sti_coh(a.pidx + (long)b * nblk + blk, mi);
                } else {
                    stxf<false>(a.pmax + (long)b * nblk + blk, m);
                    stxi<false>(a.pidx + (long)b * nblk + blk, mi);
                }
            }
        }
        if (a.done) {
            // coh.h protocol: the storing lane drains its stores, then counts; the block whose
            // add came last reads every partial coherently after a barrier.  Two-level count
            // (same-address atomics serialize): block -> shard blk % 32 (own 128-B line), the
            // block completing a shard -> top word done[0]
            constexpr int NSH = 32, STR = 32;
            __shared__ int last;
            if (tid == 0) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const int sh = blk % NSH;
                const unsigned shard_n = (unsigned)((nblk - sh + NSH - 1) / NSH);
                const unsigned n_sh = (unsigned)(nblk < NSH ? nblk : NSH);
                last = 0;
                if (__hip_atomic_fetch_add(a.done + (1 + sh) * STR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1 ==
                    shard_n)
                    last = __hip_atomic_fetch_add(a.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1 == n_sh;
            }
            __syncthreads();
            if (last) {
                for (int b = 0; b < a.nb && b < B; ++b) {
                    float m = -INFINITY;
                    int mi = 0x7fffffff;
                    for (int i = tid; i < nblk; i += blockDim.x) {
                        const float v = ldf_coh(a.pmax + (long)b * nblk + i);
                        const int ix = ldi_coh(a.pidx + (long)b * nblk + i);
                        if (v > m || (v == m && ix < mi)) { m = v; mi = ix; }
                    }
#pragma unroll
                    for (int o = 32; o > 0; o >>= 1) {
                        const float v = __shfl_xor(m, o);
                        const int ix = __shfl_xor(mi, o);
                        if (v > m || (v == m && ix < mi)) { m = v; mi = ix; }
                    }
                    __syncthreads();  // bv/bi reuse across rows
                    if (lane == 0) { bv[wave][0] = m; bi[wave][0] = mi; }
                    __syncthreads();
                    if (tid == 0) {
                        for (int q = 1; q < 4; ++q)
                            if (bv[q][0] > m || (bv[q][0] == m && bi[q][0] < mi)) { m = bv[q][0]; mi = bi[q][0]; }
                        a.next[b] = mi;
                        if (a.hist) a.hist[b] = mi;
                    }
                }
                if (tid == 0) {
                    if (a.adv) {
                        a.adv->kv_len += 1;
                        a.adv->position += 1;
                    }
                }
                if (tid <= NSH) __hip_atomic_store(a.done + tid * STR, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

template <int B, int KCH, int RPW, int MODE, int WK, bool XREG, int DEPTH, bool EMB = false>
__global__ void __launch_bounds__(256) k_gemv(GemvArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint16_t xs[];  // [B][K]
    gemv_block<B, KCH, RPW, MODE, WK, XREG, DEPTH, EMB>(a, blockIdx.x, gridDim.x, xs);
}

}  // namespace pgmi
