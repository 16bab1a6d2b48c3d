// kernels_gemv_mfma.hip -- decode projections for 2..16 sequences in lock-step (BASELINE configs[3]:
// 8 images per GPU), on MFMA.
//
// At batch 1 a decode projection is one HBM pass with v_dot2 (gemv_body.h).  At batch B the
// same pass owes B dot products per weight byte; on v_dot2 that turns the pass VALU-bound (B = 8:
// gate/up 90 us vs 22 us at B = 1).  Here the batch rows are the M side of a v_mfma_f32_16x16x32_bf16
// (rows >= B are zero) and 16 weight rows are the N side, so the pass is back to one read of
// the weights:
//   - one wave owns a 16-unit group (16 weight rows; 16 row pairs for RoPE / GeGLU) over a
//     KW-wide slice of K; WK waves of a workgroup split K and meet in LDS; KS workgroups split
//     it further for the 16384-wide down_proj (fp32 partial slabs, reduced by k_mf_combine);
//   - B operand (weights) straight from HBM in the MFMA layout: lane (n = lane & 15, g = lane >> 4)
//     reads 16 B of row n at k = 32i + 8g, so one load instruction covers 64 contiguous bytes of
//     each of its 16 rows (default cache policy: the other half of each 128-B line follows; PGMI_MF_NT);
//   - A operand (activations, B x K bf16): the wave's K slice held in registers, staged through
//     LDS (row stride K + 8: conflict-free 16-B reads) with the RMSNorm (modeling_gemma.py:114-120)
//     fused in, or read from global (o_proj's and down_proj's inputs);
//   - epilogues and rounding points exactly as gemv_body.h (RoPE + KV append, GeGLU, residual,
//     fp32 logits + per-workgroup first-max argmax partials).
#include <cstdlib>

#include "gemv_body.h"

namespace pgmi {

constexpr int MF_MAXB = 16;

// RMSNorm'd (or plain) activation rows into xs (stride ld).  Every row's chunks are loaded
// before any is reduced (one round trip for the whole [nb][K] block, not one per row).  NBM: rows
// loaded per chunk (unconditionally, rows past nb clamped to the last one); 8 when nb <= 8, so
// batches up to 8 issue half the loads of the 16-row form (mf_stage_rows picks it per launch).
template <int NBM>
__device__ void mf_stage_rows_t(const GemvArgs& a, int K, uint16_t* xs, int ld, float* red, int k0, int ksl) {
    const int tid = threadIdx.x, nt = blockDim.x, lane = tid & 63, wave = tid >> 6, nw = nt >> 6;
    float ss[NBM];
#pragma unroll
    for (int b = 0; b < NBM; ++b) ss[b] = 0.f;
    // K <= 8 x threads (K = 2048 at 256 or 512 threads): one chunk per thread, and its norm weights are
    // fetched with the rows (one round trip, not a second one after the reduction)
    const bool one = (K <= nt * 8);
    const bool has = tid * 8 < K;
    const uint4 wv0 = (one && a.norm_w) ? ldg16(a.norm_w + (has ? tid * 8 : 0)) : make_uint4(0, 0, 0, 0);
    for (int c = tid * 8; c < K; c += nt * 8) {
        uint4 v[NBM];
#pragma unroll
        for (int b = 0; b < NBM; ++b)  // unconditional (clamped row): the loads stay in flight together
            v[b] = ldg16(a.x + (long)(b < a.nb ? b : a.nb - 1) * K + c);
        const bool mine = c >= k0 && c < k0 + ksl;
#pragma unroll
        for (int b = 0; b < NBM; ++b)
            if (b < a.nb) {
                if (mine) *reinterpret_cast<uint4*>(xs + b * ld + (c - k0)) = v[b];
                const uint16_t* e = reinterpret_cast<const uint16_t*>(&v[b]);
#pragma unroll
                for (int j = 0; j < 8; ++j) { const float f = bf2f(e[j]); ss[b] += f * f; }
            }
    }
    if (!a.norm_w) return;
#pragma unroll
    for (int b = 0; b < NBM; ++b)
        if (b < a.nb) {
            const float t = wave_sum(ss[b]);
            if (lane == 0) red[b * 16 + wave] = t;
        }
    __syncthreads();
    float r[NBM];
#pragma unroll
    for (int b = 0; b < NBM; ++b) {
        float t = 0.f;
        if (b < a.nb)
            for (int w = 0; w < nw; ++w) t += red[b * 16 + w];  // fixed order
        r[b] = 1.0f / sqrtf(t / (float)K + a.eps);
    }
    for (int c = one ? tid * 8 : k0 + tid * 8; c < k0 + ksl; c += nt * 8) {
        if (c < k0) continue;
        const uint4 wv = one ? wv0 : ldg16(a.norm_w + c);
        const uint16_t* we = reinterpret_cast<const uint16_t*>(&wv);
#pragma unroll
        for (int b = 0; b < NBM; ++b)
            if (b < a.nb) {
                const uint4 v = *reinterpret_cast<const uint4*>(xs + b * ld + (c - k0));
                const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
                u16x8 o;
#pragma unroll
                for (int j = 0; j < 8; ++j) o.v[j] = f2bf((bf2f(e[j]) * r[b]) * (1.0f + bf2f(we[j])));
                *reinterpret_cast<u16x8*>(xs + b * ld + (c - k0)) = o;
            }
    }
}

__device__ void mf_stage_rows(const GemvArgs& a, int K, uint16_t* xs, int ld, float* red, int k0 = 0, int ksl = -1) {
    if (ksl < 0) ksl = K;  // stage columns [k0, k0 + ksl) at xs column 0; the norm uses the whole row
    if (a.nb <= 8) mf_stage_rows_t<8>(a, K, xs, ld, red, k0, ksl);  // uniform branch: each form drains its own loads
    else mf_stage_rows_t<MF_MAXB>(a, K, xs, ld, red, k0, ksl);
}

// Fragment-major weight image for the batched (MFMA) decode GEMVs, built once at prepare: the 16-row x 32-k
// block (g, kb) of a [rows][K] matrix is stored as the 64 lanes' B fragments in lane order -- lane
// (n = l & 15, g = l >> 4) holds row 16 g_row + n, k = 32 kb + 8 g .. + 8 -- so one load instruction of a
// wave reads 1 KiB contiguous (the row-major image: 16 rows x 64 B, half lines whose other halves come one
// instruction later).  Element offset of (row group gr, k block kb, lane l) = ((gr * K / 32 + kb) * 64 + l) * 8.
// qkv: the q|k|v GEMV's row order instead (k_gemv_mf<GV_QKV>: a 16-row group is 8 rotary pairs of one head).
__device__ __forceinline__ long qkv_row(int u) {
    const int grp_ = u >> 4, nn = u & 15;
    return (long)((grp_ >> 4) * 256 + (grp_ & 15) * 8 + (nn & 7) + (nn >> 3) * 128);
}

__global__ void k_mf_swizzle(const uint16_t* __restrict__ W, int K, long n_chunks, int qkv, uint16_t* __restrict__ out) {
    const long c = (long)blockIdx.x * blockDim.x + threadIdx.x;  // one 16-B chunk per thread
    if (c >= n_chunks) return;
    const int l = (int)(c & 63);
    const long blk = c >> 6, kbs = K / 32;
    const long gr = blk / kbs, kb = blk % kbs;
    const int u = (int)(gr * 16 + (l & 15));
    const long row = qkv ? qkv_row(u) : u, k = kb * 32 + 8 * (l >> 4);
    *reinterpret_cast<uint4*>(out + c * 8) = ldg16(W + row * K + k);
}

void mf_swizzle(hipStream_t s, const uint16_t* W, int rows, int K, uint16_t* out, bool qkv) {
    const long n = (long)rows * K / 8;
    hipLaunchKernelGGL(k_mf_swizzle, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, W, K, n, (int)qkv, out);
}

// MODE: GV_*; NR: weight rows per unit (2: RoPE / GeGLU pairs); KW: K elements per wave; WK:
// waves per unit group (K split inside the workgroup).  grid.x: unit-group slots (grid-stride
// over groups), grid.y: KS (K split over workgroups; GV_RES only, partials to ws).
// PF = 2 (GV_RES, no staging): the streams of a workgroup's next TWO groups are in flight while a
// group multiplies -- two register buffers in ping-pong, every issue unconditional (groups past the
// end read one 64-B line of the matrix: all lanes the same address, results discarded), so the
// compiler's in-order vmcnt keeps the second stream in flight across the first's wait.
// NS (no staging): the q|k|v / gate|up input is already RMSNorm'd (k_rows_norm wrote it), so each wave
// reads its K slice straight from global like the residual projections; or (gate|up, a.ssq) the input is
// h and each wave normalises its slice on load from o_proj's partial sums of squares
// Weight-stream cache policy of the register-streamed MFMA GEMVs.  Each load instruction reads 64-B
// halves of 128-B lines (16 rows x 4 lanes of 16 B), the other half following one instruction later:
// with the default policy the line is kept in L2 for it.  Same-box A/B (B = 8 step, tools/ab_variants.sh
// b8): non-temporal everywhere 1.551 / 1.556 ms, default policy on gate|up only 1.530 / 1.526, on every
// mode 1.472 / 1.475.  Probe builds: -DPGMI_MF_NT=1 non-temporal everywhere, 0 gate|up only.
#ifndef PGMI_MF_NT
#define PGMI_MF_NT 2
#endif
template <int MODE, int NR, int KW, int WK, int PF = 1, bool NS = false, bool SW = false>
__global__ void __launch_bounds__(64 * WK) k_gemv_mf(GemvArgs a, float* __restrict__ ws) {
    constexpr int NKB = KW / 128;          // 128-wide k blocks per wave
    constexpr bool STAGE = (MODE != GV_RES) && !NS;
    // (the fragment-major image, SW: every load reads whole lines once -- non-temporal)
    constexpr bool kNt = SW || PGMI_MF_NT == 1 || (PGMI_MF_NT == 0 && MODE != GV_GEGLU);
    extern __shared__ __attribute__((aligned(16))) uint16_t mfs[];
    __shared__ float red[MF_MAXB * 16];
    __shared__ f32x4 kred[WK][NR][64];
    const int tid = threadIdx.x, lane = tid & 63, wk = tid >> 6;
    const int n = lane & 15, g = lane >> 4;
    const int K = a.K, ld = K + 8;
    const int KS = gridDim.y, ks = blockIdx.y;
    const int k0 = (ks * WK + wk) * KW;
    const int n_groups = (a.n_units + 15) / 16;

    // GV_QKV: unit u = one weight row; a 16-row group is 8 rotary pairs of one head, d in lanes
    // n < 8 and d + 128 in lane n + 8 (the partner value is one lane swap away in the C map), so the
    // 2,560 rows make 160 groups
    static_assert(MODE != GV_QKV || NR == 1, "q|k|v: one weight row per lane");
    static_assert(MODE != GV_ORES, "o_proj at B >= 3: k_attn_combine, then GV_RES");
    auto row_of = [&](int u, int j) -> long {
        if constexpr (MODE == GV_QKV) {
            const int grp_ = u >> 4, nn = u & 15;
            return (long)((grp_ >> 4) * 256 + (grp_ & 15) * 8 + (nn & 7) + (nn >> 3) * 128);
        }
        else if constexpr (MODE == GV_GEGLU) return (long)u + (long)j * a.I;
        else return (long)u;
    };
    uint4 w[NR][NKB][4];
    // SW: the fragment-major image (k_mf_swizzle; n_units % 16 == 0, the up rows' image of n_groups groups
    // after the gate rows'): lane-linear 1-KiB pieces, k block stride 512 elements, read non-temporal
    static_assert(!SW || PF == 1, "fragment-major image: one-deep register streams");
    auto issue = [&](int grp) {
        int u = grp * 16 + n;
        if (u >= a.n_units) u = a.n_units - 1;  // clamp: duplicate row, result discarded
#pragma unroll
        for (int j = 0; j < NR; ++j) {
            const uint16_t* rp = SW ? a.W + (((long)j * n_groups + grp) * (K / 32) + k0 / 32) * 512 + lane * 8
                                    : a.W + row_of(u, j) * K + k0 + 8 * g;
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const long o = SW ? (long)(kb * 4 + i) * 512 : kb * 128 + 32 * i;
                    w[j][kb][i] = kNt ? ldg_nt(rp + o) : ldg16(rp + o);
                }
        }
    };
    if constexpr (PF == 2) {
        static_assert(MODE == GV_RES && NR == 1, "two-deep stream: K-split residual projection only");
        uint4 wb[2][NKB][4];
        auto issue_into = [&](uint4 (&dst)[NKB][4], int gi) {
            const bool live = gi < n_groups;
            const uint16_t* rp = live ? a.W + (long)(gi * 16 + n < a.n_units ? gi * 16 + n : a.n_units - 1) * K + k0 + 8 * g
                                      : a.W;
            const int step = live ? 1 : 0;
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    dst[kb][i] = kNt ? ldg_nt(rp + step * (kb * 128 + 32 * i)) : ldg16(rp + step * (kb * 128 + 32 * i));
        };
        const int G = gridDim.x;
        // activation rows n >= nb re-read row nb - 1 (unconditional loads): they only feed C rows
        // b >= nb, which are never stored
        short8 xr[NKB][4];
        const int xrow = n < a.nb ? n : a.nb - 1;
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                xr[kb][i] = __builtin_bit_cast(short8, ldg16(a.x + (long)xrow * K + k0 + kb * 128 + 32 * i + 8 * g));
        // the activation before the two streams: the first multiply waits for xr and the first
        // stream only (in-order vmcnt), the second stream stays in flight
        issue_into(wb[0], blockIdx.x);
        issue_into(wb[1], blockIdx.x + G);
        auto step = [&](uint4 (&buf)[NKB][4], int cur) {
            f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
                for (int i = 0; i < 4; ++i) acc = mfma16(xr[kb][i], __builtin_bit_cast(short8, buf[kb][i]), acc);
            issue_into(buf, cur + 2 * G);  // this buffer's next stream starts now
            if constexpr (WK > 1) {
                kred[wk][0][lane] = acc;
                __syncthreads();
                if (wk == 0)
#pragma unroll
                    for (int q = 1; q < WK; ++q) acc += kred[q][0][lane];
                __syncthreads();
            }
            const int u = cur * 16 + n;
            if (wk == 0 && cur < n_groups && u < a.n_units)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int b = 4 * g + r;
                    if (b >= a.nb) break;
                    ws[((long)ks * a.nb + b) * a.n_units + u] = acc[r];  // K split only (no load in the loop)
                }
        };
        // pairs of groups per trip; the trip count is uniform over the grid, and a group past the
        // end multiplies the dummy line and stores nothing (no branch around any load)
        for (int g0 = blockIdx.x; g0 - (int)blockIdx.x < n_groups; g0 += 2 * G) {
            step(wb[0], g0);
            step(wb[1], g0 + G);
        }
        return;
    }
    int grp = blockIdx.x;
    // Normalise-on-load (FOLD: gate|up, a.ssq; K = 2048): x = h, RMSNorm'd by each wave for its own K slice
    // from the 16-column partial sums of squares o_proj's epilogue wrote (a.ssq, [nb][K / 16]).  Its
    // loads -- the norm weight (to LDS, nws, not 64 registers per lane beside the weight stream), the raw
    // h slice, the row's partials -- are issued BEFORE the weight stream, so the in-order vmcnt of their
    // waits leaves the stream in flight while the norm is computed.  Rows n >= nb re-read row nb - 1: they
    // only feed C rows b >= nb, which are never stored.
    constexpr bool FOLD = NS && MODE == GV_GEGLU;
    constexpr int KF = 2048, Q4 = KF / 64;
    __shared__ __attribute__((aligned(16))) uint16_t nws[FOLD ? KF : 8];
    const bool fold = FOLD && a.ssq;
    short8 xf[NKB][4];
    uint4 nw0 = make_uint4(0, 0, 0, 0);
    f32x4 sv[FOLD ? Q4 / 4 : 1];
    if (fold) {
        const int row = n < a.nb ? n : a.nb - 1;
        if (tid * 8 < KF) nw0 = ldg16(a.norm_w + tid * 8);
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                xf[kb][i] = __builtin_bit_cast(short8, ldg16(a.x + (long)row * KF + k0 + kb * 128 + 32 * i + 8 * g));
        const f32x4* sp = reinterpret_cast<const f32x4*>(a.ssq + (long)row * (KF / 16) + g * Q4);
#pragma unroll
        for (int c = 0; c < (FOLD ? Q4 / 4 : 1); ++c) sv[c] = sp[c];
    }
    // unfolded, unstaged inputs: this wave's K slice of the rows before the stream, every load unconditional
    // (rows n >= nb re-read row nb - 1: they only feed C rows b >= nb, never stored), so the first MFMA waits
    // for its fragment only
    if (!STAGE && !fold) {
        const int row = n < a.nb ? n : a.nb - 1;
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                xf[kb][i] = __builtin_bit_cast(short8, ldg16(a.x + (long)row * K + k0 + kb * 128 + 32 * i + 8 * g));
    }
    // unconditional (a workgroup past the last group streams that group again, unused): no branch around
    // the stream, so the waits for the loads above are counted past it
    issue(grp < n_groups ? grp : n_groups - 1);
    // RoPE operands of this workgroup's first group, fetched with the weight stream (the epilogue
    // would otherwise pay their round trip after the reduction)
    float cs0 = 0.f, sn0 = 0.f;
    if constexpr (MODE == GV_QKV) {
        int p0 = a.st->position;
        p0 = p0 < 0 ? 0 : (p0 > a.max_pos - 1 ? a.max_pos - 1 : p0);
        const int d0 = (grp & 15) * 8 + (n & 7);
        cs0 = bf2f(a.cosT[(long)p0 * 128 + d0]);
        sn0 = bf2f(a.sinT[(long)p0 * 128 + d0]);
    }
    const int grp0 = grp;

    // ---- activations: this wave's K slice, MFMA A layout (row b = lane & 15)
    if constexpr (STAGE) {
        mf_stage_rows(a, K, mfs, ld, red);
        __syncthreads();
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                xf[kb][i] = n < a.nb ? *reinterpret_cast<const short8*>(mfs + n * ld + k0 + kb * 128 + 32 * i + 8 * g)
                                     : short8{0, 0, 0, 0, 0, 0, 0, 0};
    } else if (fold) {
        // the row's rstd: lane group g sums its quarter of the partials in order, the quarters meet over two
        // lane swaps (the same tree in every lane of the row); then bf16((h * r) * (1 + w)) as k_rows_norm
        if (tid * 8 < KF) *reinterpret_cast<uint4*>(nws + tid * 8) = nw0;
        __syncthreads();
        float ss = 0.f;
#pragma unroll
        for (int c = 0; c < (FOLD ? Q4 / 4 : 1); ++c) { ss += sv[c][0]; ss += sv[c][1]; ss += sv[c][2]; ss += sv[c][3]; }
        ss += __shfl_xor(ss, 16, 64);
        ss += __shfl_xor(ss, 32, 64);
        const float r = 1.0f / sqrtf(ss / (float)KF + a.eps);
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const u16x8 wv = *reinterpret_cast<const u16x8*>(nws + k0 + kb * 128 + 32 * i + 8 * g);
                const u16x8 e = __builtin_bit_cast(u16x8, xf[kb][i]);
                u16x8 o;
#pragma unroll
                for (int j = 0; j < 8; ++j) o.v[j] = f2bf((bf2f(e.v[j]) * r) * (1.0f + bf2f(wv.v[j])));
                xf[kb][i] = __builtin_bit_cast(short8, o);
            }
    }

    int kv_len = 0, pos = 0;
    if constexpr (MODE == GV_QKV) {
        kv_len = a.st->kv_len;
        pos = a.st->position;
        if (pos < 0) pos = 0;
        if (pos > a.max_pos - 1) pos = a.max_pos - 1;  // clamp (modeling_gemma.py:163-165)
    }
    float best[4];
    int besti[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) { best[r] = -INFINITY; besti[r] = 0x7fffffff; }

    // One trip per row group of the workgroup, the last one peeled off: the in-loop issue of the next group's
    // stream is unconditional, so the compiler's in-order vmcnt model stays exact across trips and each MFMA
    // waits for its own fragment (a branch around the issue made every trip wait vmcnt(0) for the whole stream
    // before its first MFMA).  Same box, B = 8 step 1.3341 / 1.3282 / 1.3359 -> 1.3179 / 1.3021 / 1.3054 ms
    // (profiles/r05_b8_peel_ab.txt)
    auto body = [&](auto next_t) {
        constexpr bool NEXT = decltype(next_t)::value;
        f32x4 acc[NR];
#pragma unroll
        for (int j = 0; j < NR; ++j) {
            acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[j] = mfma16(xf[kb][i], __builtin_bit_cast(short8, w[j][kb][i]), acc[j]);
        }
        const int cur = grp;
        if constexpr (NEXT) issue(grp + gridDim.x);  // the next group's stream starts now (it exists)
        grp += gridDim.x;
        if constexpr (WK > 1) {
#pragma unroll
            for (int j = 0; j < NR; ++j) kred[wk][j][lane] = acc[j];
            __syncthreads();
            if (wk == 0) {
#pragma unroll
                for (int j = 0; j < NR; ++j) {
                    acc[j] = kred[0][j][lane];
#pragma unroll
                    for (int q = 1; q < WK; ++q) acc[j] += kred[q][j][lane];
                }
            }
            __syncthreads();
            if (wk != 0) return;
        }
        // C map: col n = unit (cur*16 + n), row b = 4g + r
        const int u = cur * 16 + n;
        if constexpr (MODE == GV_QKV) {
            // the rotary partner of this lane's row is lane n ^ 8's (same rows b)
            f32x4 part;
#pragma unroll
            for (int r = 0; r < 4; ++r) part[r] = __shfl_xor(acc[0][r], 8, 64);
            const int hh = cur >> 4, d = (cur & 15) * 8 + (n & 7), hi = n >> 3;
            const int nh = a.I;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int b = 4 * g + r;
                if (b >= a.nb) break;
                const float x0 = rbf(hi ? part[r] : acc[0][r]), x1 = rbf(hi ? acc[0][r] : part[r]);
                if (hh < nh + a.nkv) {
                    const float c = cur == grp0 ? cs0 : bf2f(a.cosT[(long)pos * 128 + d]);
                    const float sn = cur == grp0 ? sn0 : bf2f(a.sinT[(long)pos * 128 + d]);
                    const uint16_t o = hi ? f2bf(rbf(x1 * c) + rbf(x0 * sn)) : f2bf(rbf(x0 * c) + rbf(-x1 * sn));
                    uint16_t* dst = hh < nh ? a.out + (long)b * nh * 256 + hh * 256
                                            : a.kc + b * a.kv_b_stride + (long)kv_len * (a.nkv * 256) + (hh - nh) * 256;
                    dst[d + hi * 128] = o;
                } else {
                    uint16_t* dst = a.vc + b * a.kv_b_stride + (long)kv_len * (a.nkv * 256) + (hh - nh - a.nkv) * 256;
                    dst[d + hi * 128] = f2bf(hi ? x1 : x0);
                }
            }
            return;
        }
        if constexpr (MODE == GV_RES) {
            if (KS == 1) {
                // h += o_proj(x); with a.ssq, each row's sum of squares of the new h over this group's 16
                // columns (the next RMSNorm's partial, read by gate|up): a fixed butterfly over lanes n
                float q[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int b = 4 * g + r;
                    q[r] = 0.f;
                    if (b < a.nb && u < a.n_units) {
                        const long o = (long)b * a.n_units + u;
                        const uint16_t v = f2bf(rbf(acc[0][r]) + bf2f(a.out[o]));
                        a.out[o] = v;
                        q[r] = bf2f(v) * bf2f(v);
                    }
                }
                if (a.ssq) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
#pragma unroll
                        for (int o = 1; o < 16; o <<= 1) q[r] += __shfl_xor(q[r], o, 64);
                        if (n == 0 && 4 * g + r < a.nb) a.ssq[(long)(4 * g + r) * n_groups + cur] = q[r];
                    }
                }
                return;
            }
        }
        if (u >= a.n_units) return;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int b = 4 * g + r;
            if (b >= a.nb) break;
            if constexpr (MODE == GV_RES) {
                if (KS > 1) ws[((long)ks * a.nb + b) * a.n_units + u] = acc[0][r];
                else a.out[(long)b * a.n_units + u] = f2bf(rbf(acc[0][r]) + bf2f(a.out[(long)b * a.n_units + u]));
            } else if constexpr (MODE == GV_GEGLU) {
                const float gg = rbf(gelu_tanh(rbf(acc[0][r])));
                a.out[(long)b * a.I + u] = f2bf(gg * rbf(acc[1][r]));
            } else if constexpr (MODE == GV_LOGITS) {
                const float v = rbf(acc[0][r]);
                a.logits[(long)b * a.n_units + u] = v;
                if (v > best[r]) { best[r] = v; besti[r] = u; }  // units visited in increasing order
            }
        }
    };
    while (grp + (int)gridDim.x < n_groups) body(std::true_type{});
    if (grp < n_groups) body(std::false_type{});
    if constexpr (MODE == GV_LOGITS) {
        // first max per batch row over this workgroup's units: lanes of one g hold 16 columns
        __shared__ float bv[MF_MAXB];
        __shared__ int bi[MF_MAXB];
        if (wk == 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float m = best[r];
                int mi = besti[r];
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) {
                    const float m2 = __shfl_xor(m, o, 64);
                    const int i2 = __shfl_xor(mi, o, 64);
                    if (m2 > m || (m2 == m && i2 < mi)) { m = m2; mi = i2; }
                }
                if (n == 0) { bv[4 * g + r] = m; bi[4 * g + r] = mi; }
            }
        }
        __syncthreads();
        if (tid < a.nb) {
            a.pmax[(long)tid * gridDim.x + blockIdx.x] = bv[tid];
            a.pidx[(long)tid * gridDim.x + blockIdx.x] = bi[tid];
        }
    }
}

// ---------------------------------------------------------------- LDS-DMA streaming form
// As k_gemv_ms, but the weights reach the MFMA through a per-wave LDS ring filled by LDS-DMA
// (global_load_lds_dwordx4): one instruction moves 4 whole 256-B row segments (1 KiB,
// coalesced), where the MFMA-layout register loads touch 16 rows x 64 B each.  Row r's 16-B
// chunk c lands at chunk (c ^ (r & 15)) of its 256-B LDS row (applied to each lane's SOURCE
// address, the LDS-DMA destination being lane-linear), so the B-fragment ds_read_b128s of 16
// rows x one 16-B k slice are conflict-free.  Each wave owns its ring: completion is its own
// vmcnt, no barrier.
template <int N>
__device__ __forceinline__ void mf_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// LDS-DMA cache policy of the ring's weight stream: non-temporal (aux 2).  Its 256-B row segments are whole
// lines read once; same-box A/B (B = 8 step, the batched lm_head's ring): default policy 1.4723 / 1.4730 ms,
// non-temporal 1.4580 / 1.4565 ms.  Probe build -DPGMI_ML_AUX=0 for the default policy.
#ifndef PGMI_ML_AUX
#define PGMI_ML_AUX 2
#endif
template <int MODE, int NR, int KSL, int D>
__global__ void __launch_bounds__(256, 1) k_gemv_ml(GemvArgs a, float* __restrict__ ws) {
    constexpr int NKB = KSL / 128;
    constexpr int SLOT = NR * 16 * 256;  // bytes of one k block of the wave's rows
    constexpr int PER = NR * 4;          // LDS-DMA instructions per k block
    static_assert((D - 1) * PER <= 63, "ring shape");
    extern __shared__ __attribute__((aligned(16))) uint8_t mls[];
    __shared__ float red[MF_MAXB * 16];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n = lane & 15, g = lane >> 4;
    const int K = a.K, ld = KSL + 8;
    const int KS = gridDim.y, ks = blockIdx.y;
    const int k0 = ks * KSL;
    const int n_groups = (a.n_units + 15) / 16;
    const int wpb = blockDim.x >> 6;  // streaming waves per workgroup (4; 1 for short row counts)
    const int gstride = gridDim.x * wpb;
    uint16_t* xs = reinterpret_cast<uint16_t*>(mls);
    uint8_t* ring = mls + (((size_t)a.nb * ld * 2 + 127) & ~(size_t)127) + (size_t)wave * D * SLOT;

    auto row_of = [&](int u, int j) -> long {
        if constexpr (MODE == GV_GEGLU) return (long)u + (long)j * a.I;
        else return (long)u;
    };
    // LDS-DMA of k block kb of group grp into slot: instruction q (of PER) covers rows
    // 4(q % 4) .. +3 of row set j = q / 4; lane -> row 4(q%4) + (lane >> 4), position lane & 15
    const int prow = lane >> 4, ppos = lane & 15;
    // k-block order rotated per group (rot = group % NKB): concurrent waves read different
    // offsets of their rows instead of all streaming the same 256-B column of rows 4 KiB apart
    auto rot_of = [&](int grp) { return grp % NKB; };
    auto issue = [&](int grp, int kb, int slot) {
        kb += rot_of(grp);
        if (kb >= NKB) kb -= NKB;
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int j = q / 4, r = 4 * (q % 4) + prow;
            int u = grp * 16 + r;
            if (u >= a.n_units) u = a.n_units - 1;
            const int c = ppos ^ r;  // source chunk landing at position ppos of row r
            const uint16_t* src = a.W + row_of(u, j) * K + k0 + kb * 128 + c * 8;
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src),
                                             (__attribute__((address_space(3))) void*)(ring + slot * SLOT + q * 1024), 16, 0,
                                             PGMI_ML_AUX);
        }
    };
    int grp = blockIdx.x * wpb + wave;
    // the ring's first D blocks go out before the activation staging: the two round trips
    // overlap (the staging's own waits drain the ring too, so the main loop starts with every
    // counted LDS-DMA retired)
    if (grp < n_groups) {
#pragma unroll
        for (int d = 0; d < D; ++d) issue(grp, d, d);
    }
    if (a.norm_w) {
        mf_stage_rows(a, K, xs, ld, red, k0, KSL);
    } else {
        for (int c = tid * 8; c < KSL; c += blockDim.x * 8) {
            uint4 v[MF_MAXB];
#pragma unroll
            for (int b = 0; b < MF_MAXB; ++b)  // unconditional (clamped row): one round trip
                v[b] = ldg16(a.x + (long)(b < a.nb ? b : a.nb - 1) * K + k0 + c);
#pragma unroll
            for (int b = 0; b < MF_MAXB; ++b)
                if (b < a.nb) *reinterpret_cast<uint4*>(xs + b * ld + c) = v[b];
        }
    }
    mf_vmcnt<0>();
    __syncthreads();
    const int xrow = n < a.nb ? n : 0;
    const uint16_t* xa = xs + xrow * ld + 8 * g;
    const bool xz = n >= a.nb;
    int slot0 = 0;  // ring slot of this group's block 0 (the stream runs on across groups)

    float best[4];
    int besti[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) { best[r] = -INFINITY; besti[r] = 0x7fffffff; }

    for (; grp < n_groups; grp += gstride) {
        const int nxt = grp + gstride;
        const bool more = nxt < n_groups;
        const int rot = rot_of(grp);
        f32x4 acc[NR];
#pragma unroll
        for (int j = 0; j < NR; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) {
            const int slot = (slot0 + kb) % D;
            // block kb landed: the younger D-1 blocks may still be in flight (only while they exist)
            if (kb + D <= NKB || more) mf_vmcnt<(D - 1) * PER>();
            else mf_vmcnt<0>();
            const uint8_t* sb = ring + slot * SLOT + n * 256;
            short8 wf[NR][4];
#pragma unroll
            for (int j = 0; j < NR; ++j)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    wf[j][i] = *reinterpret_cast<const short8*>(sb + j * 4096 + (((4 * i + g) ^ n) << 4));
            short8 xv[4];
            const int kr = kb + rot < NKB ? kb + rot : kb + rot - NKB;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                xv[i] = *reinterpret_cast<const short8*>(xa + kr * 128 + 32 * i);
                if (xz) xv[i] = short8{0, 0, 0, 0, 0, 0, 0, 0};
            }
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the slot's reads are done
            if (kb + D < NKB) issue(grp, kb + D, slot);
            else if (more) issue(nxt, kb + D - NKB, slot);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < NR; ++j) acc[j] = mfma16(xv[i], wf[j][i], acc[j]);
        }
        slot0 = (slot0 + NKB) % D;
        const int u = grp * 16 + n;
        if (u >= a.n_units) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int b = 4 * g + r;
            if (b >= a.nb) break;
            if constexpr (MODE == GV_RES) {
                if (KS > 1) ws[((long)ks * a.nb + b) * a.n_units + u] = acc[0][r];
                else a.out[(long)b * a.n_units + u] = f2bf(rbf(acc[0][r]) + bf2f(a.out[(long)b * a.n_units + u]));
            } else if constexpr (MODE == GV_GEGLU) {
                const float gg = rbf(gelu_tanh(rbf(acc[0][r])));
                a.out[(long)b * a.I + u] = f2bf(gg * rbf(acc[1][r]));
            } else {  // GV_LOGITS
                const float v = rbf(acc[0][r]);
                a.logits[(long)b * a.n_units + u] = v;
                if (v > best[r]) { best[r] = v; besti[r] = u; }
            }
        }
    }
    if constexpr (MODE == GV_LOGITS) {
        __shared__ float bv[4][MF_MAXB];
        __shared__ int bi[4][MF_MAXB];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float m = best[r];
            int mi = besti[r];
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) {
                const float m2 = __shfl_xor(m, o, 64);
                const int i2 = __shfl_xor(mi, o, 64);
                if (m2 > m || (m2 == m && i2 < mi)) { m = m2; mi = i2; }
            }
            if (n == 0) { bv[wave][4 * g + r] = m; bi[wave][4 * g + r] = mi; }
        }
        __syncthreads();
        if (tid < a.nb) {
            float m = bv[0][tid];
            int mi = bi[0][tid];
            for (int q = 1; q < wpb; ++q)  // the workgroup's streaming waves, in a fixed order
                if (bv[q][tid] > m || (bv[q][tid] == m && bi[q][tid] < mi)) { m = bv[q][tid]; mi = bi[q][tid]; }
            a.pmax[(long)tid * gridDim.x + blockIdx.x] = m;
            a.pidx[(long)tid * gridDim.x + blockIdx.x] = mi;
        }
    }
}

// flash-decoding combine of k_attn_decode's partials -> o (bf16 [nb][G*256]), one thread per
// 8 outputs, chunk records in a fixed order (gemv_body.h's GV_ORES prologue, once per output).
// As that prologue: up to CMAX chunk records are loaded unconditionally up front (chunk index
// clamped, records past nch ignored), so the combine costs one memory round trip instead of one
// per chunk; 64-thread workgroups spread the 2,048 threads of B = 8 over 32 CUs.
__global__ void __launch_bounds__(64) k_attn_combine(GemvArgs a, uint16_t* __restrict__ o, int K) {
    const int e8 = blockIdx.x * 64 + threadIdx.x;
    if (e8 >= a.nb * K / 8) return;
    const int nch = (a.st->kv_len + 1 + kAttnChunk - 1) / kAttnChunk;
    const int b = e8 / (K / 8), e = (e8 % (K / 8)) * 8;
    const int h = e >> 8;
    const float* pb = a.part + (long)b * a.max_chunks * kAttnPartStride + h * 256 + (e & 255);
    const float* sp = a.part + (long)b * a.max_chunks * kAttnPartStride + 16 * 256 + h;
    float M = -INFINITY, S = 0.f, acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    constexpr int CMAX = 12;  // chunks held in registers (768 keys); longer caches take the loop
    if (nch <= CMAX) {
        f32x4 x0[CMAX], x1[CMAX];
        float mc[CMAX], lc[CMAX];
#pragma unroll
        for (int c = 0; c < CMAX; ++c) {
            const long cs = (long)(c < nch ? c : nch - 1) * kAttnPartStride;
            x0[c] = *reinterpret_cast<const f32x4*>(pb + cs);
            x1[c] = *reinterpret_cast<const f32x4*>(pb + cs + 4);
            mc[c] = sp[cs];
            lc[c] = sp[cs + 16];
        }
#pragma unroll
        for (int c = 0; c < CMAX; ++c)
            if (c < nch) M = fmaxf(M, mc[c]);
#pragma unroll
        for (int c = 0; c < CMAX; ++c)
            if (c < nch) {
                const float wgt = expf(mc[c] - M);
                S += wgt * lc[c];
#pragma unroll
                for (int j = 0; j < 4; ++j) { acc[j] += wgt * x0[c][j]; acc[4 + j] += wgt * x1[c][j]; }
            }
    } else {
        for (int c = 0; c < nch; ++c) M = fmaxf(M, sp[(long)c * kAttnPartStride]);
        for (int c = 0; c < nch; ++c) {
            const float wgt = expf(sp[(long)c * kAttnPartStride] - M);
            S += wgt * sp[(long)c * kAttnPartStride + 16];
            const f32x4 x0 = *reinterpret_cast<const f32x4*>(pb + (long)c * kAttnPartStride);
            const f32x4 x1 = *reinterpret_cast<const f32x4*>(pb + (long)c * kAttnPartStride + 4);
#pragma unroll
            for (int j = 0; j < 4; ++j) { acc[j] += wgt * x0[j]; acc[4 + j] += wgt * x1[j]; }
        }
    }
    u16x8 ob;
#pragma unroll
    for (int j = 0; j < 8; ++j) ob.v[j] = f2bf(acc[j] / S);
    *reinterpret_cast<u16x8*>(o + (long)b * K + e) = ob;
}

// h[b][n] = bf16(bf16(sum_ks ws[ks][b][n]) + h[b][n]), fixed ks order
// (KS <= 8: the eight slab loads and the residual load are issued unconditionally up front -- slab
// index clamped, slabs past KS left out of the sum by a select after the loads -- so the combine is
// one memory round trip, not one per slab; the sum keeps the slab order)
__global__ void k_mf_combine(const float* __restrict__ ws, int KS, int nb, int N, uint16_t* __restrict__ h) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nb * N) return;
    const long slab = (long)nb * N;
    float s;
    if (KS <= 8) {
        float p[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) p[q] = ws[(long)(q < KS ? q : 0) * slab + i];
        s = p[0];
#pragma unroll
        for (int q = 1; q < 8; ++q) s = q < KS ? s + p[q] : s;
    } else {
        s = ws[i];
        for (int q = 1; q < KS; ++q) s += ws[(long)q * slab + i];
    }
    h[i] = f2bf(rbf(s) + bf2f(h[i]));
}

// One workgroup per batch row: RMSNorm (modeling_gemma.py:114-120) of x -> out, the rows the
// unstaged batched projections read.  Every thread's chunks are loaded before the reduction.
__global__ void __launch_bounds__(256) k_rows_norm(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                   float eps, int K, uint16_t* __restrict__ out) {
    __shared__ float red[4];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint16_t* xr = x + (long)b * K;
    float ss = 0.f;
    for (int c = tid * 8; c < K; c += 256 * 8) {
        const uint4 v = ldg16(xr + c);
        const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
        for (int j = 0; j < 8; ++j) { const float f = bf2f(e[j]); ss += f * f; }
    }
    ss = wave_sum(ss);
    if (lane == 0) red[wave] = ss;
    __syncthreads();
    const float r = 1.0f / sqrtf((red[0] + red[1] + red[2] + red[3]) / (float)K + eps);
    for (int c = tid * 8; c < K; c += 256 * 8) {
        const uint4 v = ldg16(xr + c), wv = ldg16(w + c);
        const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
        const uint16_t* we = reinterpret_cast<const uint16_t*>(&wv);
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o.v[j] = f2bf((bf2f(e[j]) * r) * (1.0f + bf2f(we[j])));
        *reinterpret_cast<u16x8*>(out + (long)b * K + c) = o;
    }
}

// k_mf_combine (KS <= 8) with the next RMSNorm fused: one workgroup per batch row, h = bf16(bf16(sum_ks ws[ks])
// + h) (fixed ks order, the slab loads issued up front as k_mf_combine), then (w != nullptr) hn =
// RMSNorm(h) -- the next layer's normalised input, so its q|k|v projection stages nothing
__global__ void __launch_bounds__(256) k_mf_combine_norm(const float* __restrict__ ws, int KS, int N,
                                                         uint16_t* __restrict__ h, const uint16_t* __restrict__ w,
                                                         float eps, uint16_t* __restrict__ hn) {
    __shared__ float red[4];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const long slab = (long)gridDim.x * N;
    float ss = 0.f;
    // N = 2048: one chunk of 8 per thread, kept in registers for the norm (no re-read of h); wider rows re-read
    u16x8 keep{};
    for (int c = tid * 8; c < N; c += 256 * 8) {
        const long i0 = (long)b * N + c;
        f32x4 p[8][2];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const long o = (long)(q < KS ? q : 0) * slab + i0;
            p[q][0] = *reinterpret_cast<const f32x4*>(ws + o);
            p[q][1] = *reinterpret_cast<const f32x4*>(ws + o + 4);
        }
        const uint4 hv = ldg16(h + i0);
        const uint16_t* he = reinterpret_cast<const uint16_t*>(&hv);
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float t = p[0][j >> 2][j & 3];
#pragma unroll
            for (int q = 1; q < 8; ++q) t = q < KS ? t + p[q][j >> 2][j & 3] : t;
            o.v[j] = f2bf(rbf(t) + bf2f(he[j]));
            const float f = bf2f(o.v[j]);
            ss += f * f;
        }
        *reinterpret_cast<u16x8*>(h + i0) = o;
        keep = o;
    }
    if (!w) return;
    ss = wave_sum(ss);
    if (lane == 0) red[wave] = ss;
    __syncthreads();
    const float r = 1.0f / sqrtf((red[0] + red[1] + red[2] + red[3]) / (float)N + eps);
    for (int c = tid * 8; c < N; c += 256 * 8) {
        const uint4 wv = ldg16(w + c);
        const uint4 v = N <= 256 * 8 ? __builtin_bit_cast(uint4, keep) : ldg16(h + (long)b * N + c);  // own stores
        const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
        const uint16_t* we = reinterpret_cast<const uint16_t*>(&wv);
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o.v[j] = f2bf((bf2f(e[j]) * r) * (1.0f + bf2f(we[j])));
        *reinterpret_cast<u16x8*>(hn + (long)b * N + c) = o;
    }
}

void rows_norm(hipStream_t s, const uint16_t* x, const uint16_t* w, float eps, int nb, int K, uint16_t* out) {
    hipLaunchKernelGGL(k_rows_norm, dim3(nb), dim3(256), 0, s, x, w, eps, K, out);
}

// smallest lock-step batch whose decode projections run on MFMA (B <= 2: the v_dot2 GEMVs of gemv_body.h)
int gemv_mf_min_batch() { return 3; }

template <int MODE, int NR, int KW, int WK, int PF = 1, bool NS = false, bool SW = false>
static void launch_mf(hipStream_t s, const GemvArgs& a, int blocks, int KS, float* ws) {
    const size_t lds = (MODE == GV_RES || NS) ? 0 : (size_t)a.nb * (a.K + 8) * sizeof(uint16_t);
    static size_t attr = 0;
    if (lds > attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemv_mf<MODE, NR, KW, WK, PF, NS, SW>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr = lds;
    }
    hipLaunchKernelGGL((k_gemv_mf<MODE, NR, KW, WK, PF, NS, SW>), dim3(blocks, KS), dim3(64 * WK), lds, s, a, ws);
}

static int groups_of(int units) { return (units + 15) / 16; }

// waves: streaming waves per workgroup (GV_LOGITS keeps 4: its block reduction is laid out for 4 waves)
template <int MODE, int NR, int KSL, int D>
static void launch_ml(hipStream_t s, const GemvArgs& a, int blocks, int KS, float* ws, int waves = 4) {
    const size_t lds = (((size_t)a.nb * (KSL + 8) * 2 + 127) & ~(size_t)127) + (size_t)waves * D * NR * 16 * 256;
    static size_t attr = 0;
    if (lds > attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemv_ml<MODE, NR, KSL, D>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr = lds;
    }
    hipLaunchKernelGGL((k_gemv_ml<MODE, NR, KSL, D>), dim3(blocks, KS), dim3(64 * waves), lds, s, a, ws);
}

// workgroups of 4 streaming waves: every group once, capped at `cap` workgroups (grid-stride)
static int ms_blocks(int units, int cap) {
    const int wg = (groups_of(units) + 3) / 4;
    return wg < cap ? wg : cap;
}

// q|k|v: one weight row per lane, rotary pairs across lanes n / n + 8 (one shuffle in the
// epilogue): 160 workgroups of 8 waves splitting K = 2048 (the pair-per-lane form made 80, and a
// 4-way K split over workgroups with a separate RoPE kernel measured slower)
void gemv_mf_qkv(hipStream_t s, const GemvArgs& a, float* /*ws*/) {
    GemvArgs r = a;
    r.n_units = 2 * a.n_units;
    if (a.Wf) {  // the fragment-major weight image in the GEMV's row order (the decode step passes it)
        r.W = a.Wf;
        if (a.norm_w) launch_mf<GV_QKV, 1, 256, 8, 1, false, true>(s, r, groups_of(r.n_units), 1, nullptr);
        else launch_mf<GV_QKV, 1, 256, 8, 1, true, true>(s, r, groups_of(r.n_units), 1, nullptr);
        return;
    }
    if (a.norm_w) launch_mf<GV_QKV, 1, 256, 8>(s, r, groups_of(r.n_units), 1, nullptr);
    else launch_mf<GV_QKV, 1, 256, 8, 1, true>(s, r, groups_of(r.n_units), 1, nullptr);  // input already normed
}

void gemv_mf_geglu(hipStream_t s, const GemvArgs& a) {  // K = 2048, gate|up row pairs
    // register-streamed MFMA form: 4 waves split K (512 each); over the row-major weights 512 workgroups (2 per CU) dealing the
    // 1,024 row groups grid-stride, so each stages its 8 normalised rows for two groups; same-box A/B
    // (tools/b8_ab.sh) B = 8 step 1.737 -> 1.681 ms against the one-workgroup-per-CU LDS-DMA ring
    // (k_gemv_ml, 4 waves x 3-deep rings); 256 / 384 / 1,024 workgroups and 2 or 8 K-split waves
    // measured slower (1.746-2.051 ms); the unstaged form re-swept in round 4 (profiles/r04_gu_blocks_ab.txt:
    // 512 best against 384 / 768 / 1,024)
    // (a.ssq: x = h, normalised on load from o_proj's partial sums of squares -- unstaged, norm_w read)
    // a.Wf: the fragment-major weight image (1-KiB lane-linear loads; the decode step passes it)
    const bool staged = a.norm_w && !a.ssq;
    if (a.Wf) {
        GemvArgs r = a;
        r.W = a.Wf;
        // 256 workgroups (one per CU, four groups each): same box, B = 8 step 1.3358-1.3376 ms at 512,
        // 1.3300-1.3344 at 256, 1.3564-1.3573 at 384, 1.3667-1.3672 at 1,024 (profiles/r05_b8_grid_ab.txt).
        // Normalise-on-load form: 8 waves splitting K (256 each) once the loop was peeled -- same box, B = 8 step
        // 1.3082 / 1.3089 / 1.3083 -> 1.3000 / 1.3002 / 1.2963 ms against 4 x 512 (512 workgroups 1.313, two-deep
        // register streams 1.320, profiles/r05_b8_gu_waves_ab.txt)
        if (staged) launch_mf<GV_GEGLU, 2, 512, 4, 1, false, true>(s, r, 256, 1, nullptr);
        else launch_mf<GV_GEGLU, 2, 256, 8, 1, true, true>(s, r, 256, 1, nullptr);
        return;
    }
    if (staged) launch_mf<GV_GEGLU, 2, 512, 4>(s, a, 512, 1, nullptr);
    else launch_mf<GV_GEGLU, 2, 512, 4, 1, true>(s, a, 512, 1, nullptr);  // input already normed
}

// o_proj: combine the attention partials once (-> o, bf16 [nb][K]), then the residual GEMV
void gemv_mf_ores(hipStream_t s, const GemvArgs& a, uint16_t* o) {
    const int K = a.K;
    hipLaunchKernelGGL(k_attn_combine, dim3((a.nb * K / 8 + 63) / 64), dim3(64), 0, s, a, o, K);
    GemvArgs r = a;
    r.x = o;
    r.norm_w = nullptr;
    // 128 workgroups of 8 waves splitting K (the q|k|v form) instead of 64 two-wave LDS-ring workgroups:
    // B = 8 step 1.751-1.760 -> 1.718-1.721 ms (same-box A/B).  (The same form for the K = 16384 down
    // projection, 1,024 workgroups, measured slower: 1.79 ms.)
    if (a.Wf) {  // the fragment-major weight image (the decode step passes it)
        r.W = a.Wf;
        launch_mf<GV_RES, 1, 256, 8, 1, false, true>(s, r, groups_of(a.n_units), 1, nullptr);
        return;
    }
    launch_mf<GV_RES, 1, 256, 8>(s, r, groups_of(a.n_units), 1, nullptr);
}

int gemv_mf_logits(hipStream_t s, const GemvArgs& a, int max_blocks) {  // K = 2048
    // (the register-streamed form at 512 / 1,024 / 2,048 workgroups measured no faster: 1.741-1.768 ms; again in
    // round 5 with the peeled loop: B = 8 step 1.283 -> 1.330-1.341 ms, profiles/r05_b8_lm_mf_ab.txt)
    const int blocks = ms_blocks(a.n_units, max_blocks < 256 ? max_blocks : 256);
    launch_ml<GV_LOGITS, 1, 2048, 6>(s, a, blocks, 1, nullptr);
    return blocks;
}

// the K = 16384 down projection of the batched decode step with the next RMSNorm fused into its
// combine: h (a.out) += down(x); hn = RMSNorm(h) with norm_w (nullptr: h only)
void gemv_mf_res_norm(hipStream_t s, const GemvArgs& a, float* ws, const uint16_t* norm_w, float eps, uint16_t* hn) {
    const int KS = a.K / 2048;  // <= 8 (checked by the caller: gemv_res_norm)
    if (a.Wf) {
        // the fragment-major image (the decode step passes it), one-deep streams: same box, B = 8 step
        // 1.3461-1.3489 -> 1.3336-1.3339 ms against the two-deep row-major form below (the image with the
        // two-deep streams read slower: profiles/r05_b8_fragment_image_ab.txt); 32 x 8 workgroups (64 / 16 x 8:
        // 1.3574-1.3617 / 1.3514-1.3518 against 1.3374-1.3376, profiles/r05_b8_grid_ab.txt); 8 waves of 256
        // per K slice once the loop was peeled: 1.3003 / 1.2990 / 1.3016 -> 1.2855 / 1.2853 / 1.2807 ms against
        // 4 waves of 512 (16 / 64 x 8 workgroups of 8 waves: 1.33 / 1.29; q|k|v and o_proj with 16 waves no faster;
        // profiles/r05_b8_down_waves_ab.txt)
        GemvArgs r = a;
        r.W = a.Wf;
        launch_mf<GV_RES, 1, 256, 8, 1, false, true>(s, r, 32, KS, ws);
    } else {
        launch_mf<GV_RES, 1, 512, 4, 2>(s, a, 32, KS, ws);
    }
    hipLaunchKernelGGL(k_mf_combine_norm, dim3(a.nb), dim3(256), 0, s, ws, KS, a.n_units, a.out, norm_w, eps, hn);
}

// residual projections; ws: fp32 scratch of KS x nb x N floats for the K split of K = 16384
void gemv_mf_res(hipStream_t s, const GemvArgs& a, float* ws) {
    if (a.K == 2048) {
        launch_ml<GV_RES, 1, 2048, 6>(s, a, ms_blocks(a.n_units, 256), 1, nullptr);
        return;
    }
    if (a.K % 2048 == 0 && ws) {  // K slices of 2048 over grid.y, fp32 partials, fixed-order combine
        const int KS = a.K / 2048;
        // register-streamed MFMA form, 4 waves x 512 of each 2,048-wide K slice, 32 x 8 workgroups
        // (every row group of a slice once): B = 8 step 1.737 -> 1.704 ms against the LDS-DMA ring
        // (64 / 128 x 8 workgroups: 1.710 / 1.744)
        launch_mf<GV_RES, 1, 512, 4, 2>(s, a, 32, KS, ws);
        const int nn = a.nb * a.n_units;
        hipLaunchKernelGGL(k_mf_combine, dim3((nn + 255) / 256), dim3(256), 0, s, ws, KS, a.nb, a.n_units, a.out);
        return;
    }
    const int G = groups_of(a.n_units);
    launch_mf<GV_RES, 1, 128, 1>(s, a, G, a.K / 128, ws);  // generic K (multiple of 128)
    const int nn = a.nb * a.n_units;
    hipLaunchKernelGGL(k_mf_combine, dim3((nn + 255) / 256), dim3(256), 0, s, ws, a.K / 128, a.nb, a.n_units, a.out);
}

}  // namespace pgmi
