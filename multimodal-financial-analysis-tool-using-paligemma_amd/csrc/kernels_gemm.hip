// kernels_gemm.hip -- MFMA bf16 GEMM for the prefill path (gfx950, v_mfma_f32_16x16x32_bf16).
//
// C[M,N] = A[M,K] . W[N,K]^T with both operands K-contiguous (nn.Linear layout, so the
// reference's weights are used as stored).  Covers every nn.Linear / Conv2d of the
// prefill (modeling_siglip.py:45-51,92-95,154-155; modeling_gemma.py:129-131,220-223,
// 391,433) with the reference's rounding points fused into the epilogue.
//
// Tile: BM x BN x 64 over a grid of waves (below); A/B tiles staged global -> registers ->
// LDS (double buffered, one barrier per k-tile, next tile's global loads in flight during
// the MFMAs).  LDS rows
// are padded to 72 bf16 (144 B) so the 16 rows a ds_read_b128 lane group touches land
// on distinct banks.  Split-K (grid.z) writes fp32 partial slabs that a separate
// epilogue kernel reduces in a fixed order (bitwise reproducible).
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include <hip/hip_ext.h>

#include "common.h"
#include "launch.h"

#include <cstdlib>
#include <type_traits>

namespace pgmi {

constexpr int BK = 64;
constexpr int LDSK = 72;  // padded row (elements)

// Probe builds only (tools/build_variant.sh "-DPGMI_GEMM_DIAG=n"; never set in the product build): bit 0 = the
// panel kernels' compute waves read their fragments but issue no MFMA, bit 1 = the LDS-DMA stages issue no
// loads (the waits then pass at once) -- what the k-loop costs without the matrix work / without the intake
#ifndef PGMI_GEMM_DIAG
#define PGMI_GEMM_DIAG 0
#endif
template <int TM, int TN, int NB>
__device__ __forceinline__ void diag_consume(const short8 (&fa)[TM], const short8 (&fb)[NB][TN]) {
#pragma unroll
    for (int i = 0; i < TM; ++i) asm volatile("" ::"v"(fa[i]));
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(fb[b][j]));
}

template <int EPI>
__device__ __forceinline__ void epi_store(const EpiArgs& ea, int m, int n, float acc, float acc2) {
    switch (EPI) {
        case EPI_STORE: ea.out[(long)m * ea.ldo + n] = f2bf(acc); break;
        case EPI_BIAS: ea.out[(long)m * ea.ldo + n] = f2bf(acc + bf2f(ea.bias[n])); break;
        case EPI_BIAS_GELU: ea.out[(long)m * ea.ldo + n] = f2bf(gelu_tanh(rbf(acc + bf2f(ea.bias[n])))); break;
        case EPI_BIAS_RES:
            ea.out[(long)m * ea.ldo + n] = f2bf(rbf(acc + bf2f(ea.bias[n])) + bf2f(ea.res[(long)m * ea.ldr + n]));
            break;
        case EPI_RES: ea.out[(long)m * ea.ldo + n] = f2bf(rbf(acc) + bf2f(ea.res[(long)m * ea.ldr + n])); break;
        case EPI_BIAS_POS:
            ea.out[(long)m * ea.ldo + n] =
                f2bf(rbf(acc + bf2f(ea.bias[n])) + bf2f(ea.pos[(long)(m % ea.npos) * ea.ldo + n]));
            break;
        case EPI_F32: ea.out_f32[(long)m * ea.ldo + n] = rbf(acc); break;
        case EPI_GEGLU: ea.out[(long)m * ea.ldo + n] = f2bf(rbf(gelu_tanh(rbf(acc))) * rbf(acc2)); break;
        default: break;  // EPI_ROPE: rope_apply
    }
}

// EPI_ROPE column map: a tile's logical column lr (wave lr / 32, 16-column tile (lr / 16) % 2, lane
// lr % 16) reads weight row d or d + 128 of the same head, so the two tiles of a wave hold a rotary
// pair (d, d + 128) in the same lane.  BN must divide 256 (a tile never straddles a head).
__device__ __forceinline__ int rope_row(int n, int BN) {
    const int h = n >> 8, u = n & 255, lr = u % BN;
    return (h << 8) + ((lr >> 4) & 1) * 128 + (u / BN) * (BN / 2) + (lr >> 5) * 16 + (lr & 15);
}

// Epilogue of a wave's TM x TN MFMA tiles (C map of 16x16x32: column nb + 16 j + (lane & 15), rows
// mb + 16 i + 4 (lane >> 4) + r).  Every operand the epilogue reads -- bias per column, residual /
// position rows per element -- is loaded first from a clamped (always valid) address (epi_load),
// and only the stores sit under the bounds guard (epi_apply): a guarded load makes hipcc branch
// around it and wait vmcnt(0) per element (one dependent round trip per output).  In a kernel
// whose waves also issue LDS-DMA, hipcc waits vmcnt(0) after every ordinary load anyway, so
// k_gemm_p issues epi_load before its ring starts (the values wait in registers).
template <int EPI, int TM, int TN>
struct EpiOps {
    static constexpr bool HB = EPI == EPI_BIAS || EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_RES || EPI == EPI_BIAS_POS;
    static constexpr bool HX = EPI == EPI_BIAS_RES || EPI == EPI_RES || EPI == EPI_BIAS_POS;
    float bv[HB ? TN : 1];
    float xv[HX ? TM : 1][HX ? TN : 1][4];
};

template <int EPI, int TM, int TN>
__device__ __forceinline__ void epi_load(const EpiArgs& ea, int M, int N, int mb, int nb, int lane,
                                         EpiOps<EPI, TM, TN>& e) {
    using E = EpiOps<EPI, TM, TN>;
    int ncl[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = nb + j * 16 + (lane & 15);
        ncl[j] = n < N ? n : N - 1;
        if constexpr (E::HB) e.bv[j] = bf2f(ea.bias[ncl[j]]);
    }
    if constexpr (E::HX) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                int m = mb + i * 16 + (lane >> 4) * 4 + r;
                m = m < M ? m : M - 1;
                const uint16_t* row;
                if constexpr (EPI == EPI_BIAS_POS) row = ea.pos + (long)(m % ea.npos) * ea.ldo;
                else row = ea.res + (long)m * ea.ldr;
#pragma unroll
                for (int j = 0; j < TN; ++j) e.xv[i][j][r] = bf2f(row[ncl[j]]);
            }
    }
}

template <int EPI, int TM, int TN>
__device__ __forceinline__ void epi_apply(const EpiArgs& ea, int M, int N, int mb, int nb, int lane,
                                          EpiOps<EPI, TM, TN>& e, const f32x4 (&acc)[TM][TN],
                                          const f32x4 (&acc2)[TM][TN]) {
    // every operand passes through an empty asm before the first store: the loads are waited for
    // once, here, and the stores below are not mistaken for loads still in flight (on gfx9 vmcnt
    // counts stores too, so a wait placed between two stores would also wait for the first)
    using E = EpiOps<EPI, TM, TN>;
    if constexpr (E::HB) {
#pragma unroll
        for (int j = 0; j < TN; ++j) asm volatile("" : "+v"(e.bv[j]));
    }
    if constexpr (E::HX) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) asm volatile("" : "+v"(e.xv[i][j][r]));
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = nb + j * 16 + (lane & 15);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = mb + i * 16 + (lane >> 4) * 4 + r;
                const float a = acc[i][j][r];
                float o = 0.f;
                if constexpr (EPI == EPI_STORE) o = a;
                else if constexpr (EPI == EPI_BIAS) o = a + e.bv[j];
                else if constexpr (EPI == EPI_BIAS_GELU) o = gelu_tanh(rbf(a + e.bv[j]));
                else if constexpr (EPI == EPI_BIAS_RES) o = rbf(a + e.bv[j]) + e.xv[i][j][r];
                else if constexpr (EPI == EPI_RES) o = rbf(a) + e.xv[i][j][r];
                else if constexpr (EPI == EPI_BIAS_POS) o = rbf(a + e.bv[j]) + e.xv[i][j][r];
                else if constexpr (EPI == EPI_GEGLU) o = rbf(gelu_tanh(rbf(a))) * rbf(acc2[i][j][r]);
                if (m < M && n < N) {
                    if constexpr (EPI == EPI_F32) ea.out_f32[(long)m * ea.ldo + n] = rbf(a);
                    else ea.out[(long)m * ea.ldo + n] = f2bf(o);
                }
            }
        }
}

template <int EPI, int TM, int TN>
__device__ __forceinline__ void epi_tile(const EpiArgs& ea, int M, int N, int mb, int nb, int lane,
                                         const f32x4 (&acc)[TM][TN], const f32x4 (&acc2)[TM][TN]) {
    EpiOps<EPI, TM, TN> e;
    epi_load<EPI, TM, TN>(ea, M, N, mb, nb, lane, e);
    epi_apply<EPI, TM, TN>(ea, M, N, mb, nb, lane, e, acc, acc2);
}

// EPI_ROPE epilogue of a wave's TM x 2 tiles (rope_row column map: the lane's tiles j = 0 / 1 are the
// rotary pair (d, d + 128) of head h).  q|k|v round to bf16 first (the projections' outputs), then
// q/k rotate with three roundings (modeling_gemma.py:197-198) exactly as k_rope_kv; v is copied.
// rope_load reads the rows' positions (one batch), then their cos / sin (one batch); the kernels
// call it before their k loops, so the two dependent round trips overlap the GEMM, and rope_apply
// passes the values through one empty asm before its first store.
template <int TM>
struct RopeOps {
    float cs[TM][4], sn[TM][4];
    int h, d;
};

template <int TM, int BN>
__device__ __forceinline__ void rope_load(const EpiArgs& ea, int M, int mb, int nbw, int lane, RopeOps<TM>& e) {
    const int pr = rope_row(nbw + (lane & 15), BN);
    e.h = pr >> 8;
    e.d = pr & 255;  // < 128
    long pv[TM][4];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            int m = mb + i * 16 + (lane >> 4) * 4 + r;
            m = m < M ? m : M - 1;
            pv[i][r] = ea.rpos[m];
        }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) asm volatile("" : "+v"(pv[i][r]));
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            long p = pv[i][r];
            p = p < 0 ? 0 : (p > ea.max_pos - 1 ? ea.max_pos - 1 : p);
            e.cs[i][r] = bf2f(ea.cosT[p * 128 + e.d]);
            e.sn[i][r] = bf2f(ea.sinT[p * 128 + e.d]);
        }
}

template <int TM>
__device__ __forceinline__ void rope_apply(const EpiArgs& ea, int M, int mb, int lane, RopeOps<TM>& e,
                                           const f32x4 (&acc)[TM][2]) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            asm volatile("" : "+v"(e.cs[i][r]));
            asm volatile("" : "+v"(e.sn[i][r]));
        }
    const int h = e.h, d = e.d;
    const bool rot = h < ea.nh + ea.nkv;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = mb + i * 16 + (lane >> 4) * 4 + r;
            if (m >= M) continue;
            const float x0 = rbf(acc[i][0][r]), x1 = rbf(acc[i][1][r]);
            const int b = m / ea.L, l = m - b * ea.L;
            if (rot) {
                const float c = e.cs[i][r], sv = e.sn[i][r];
                const uint16_t o0 = f2bf(rbf(x0 * c) + rbf(-x1 * sv));
                const uint16_t o1 = f2bf(rbf(x1 * c) + rbf(x0 * sv));
                uint16_t* dst;
                if (h < ea.nh) dst = ea.q_out + (long)m * (ea.nh * 256) + h * 256;
                else dst = ea.kc + b * ea.kv_b_stride + (long)(ea.kv_start + l) * (ea.nkv * 256) + (h - ea.nh) * 256;
                dst[d] = o0;
                dst[d + 128] = o1;
            } else {
                uint16_t* dst =
                    ea.vc + b * ea.kv_b_stride + (long)(ea.kv_start + l) * (ea.nkv * 256) + (h - ea.nh - ea.nkv) * 256;
                dst[d] = f2bf(x0);
                dst[d + 128] = f2bf(x1);
            }
        }
}

// SPLIT: write raw fp32 partials to ws[z][M][N] (z = blockIdx.z) instead of the epilogue.
// Wave grid WGM x WGN; each wave owns TM x TN 16x16 MFMA tiles, so BM = WGM*TM*16 and
// BN = WGN*TN*16.  Small-M prefill GEMMs (M = 256 vision rows, 288 text rows) use one
// workgroup per BN columns covering ALL rows (WGM = 4 or 6, WGN = 1): every weight byte is
// read from HBM once, the activation panel is re-read from L2.
template <int WGM, int WGN, int TM, int TN, int EPI, bool SPLIT>
__global__ void __launch_bounds__(64 * WGM * WGN) k_gemm(const uint16_t* __restrict__ A, int lda,
                                                         const uint16_t* __restrict__ W, int ldw, int M, int N, int K,
                                                         int kt_per_split, EpiArgs ea, float* __restrict__ ws,
                                                         long up_off) {
    constexpr bool DUAL = (EPI == EPI_GEGLU);
    constexpr int NT = 64 * WGM * WGN;
    constexpr int BM = WGM * TM * 16, BN = WGN * TN * 16;
    constexpr int ACH = (BM * 8 + NT - 1) / NT;  // 16-B chunks of the A tile per thread
    constexpr int BCH = (BN * 8 + NT - 1) / NT;
    constexpr int NB = DUAL ? 2 : 1;
    extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
    uint16_t* As = smem;                         // [2][BM][LDSK]
    uint16_t* Bs = smem + 2 * BM * LDSK;         // [2][NB][BN][LDSK]

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave / WGN, wc = wave % WGN;
    const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
    const int nkt_total = (K + BK - 1) / BK;
    const int kt0 = blockIdx.z * kt_per_split;
    int kt1 = kt0 + kt_per_split;
    if (kt1 > nkt_total) kt1 = nkt_total;
    const int nkt = kt1 - kt0;

    f32x4 acc[NB][TM][TN];
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // two register stages (named, statically indexed) + two LDS buffers: the global loads of
    // k-tile t+2 are in flight while tile t is multiplied and tile t+1 is written to LDS
    uint4 ra0[ACH], rb0[NB][BCH], ra1[ACH], rb1[NB][BCH];
    auto gload = [&](int kt, uint4 (&ra)[ACH], uint4 (&rb)[NB][BCH]) {
        const int kbase = kt * BK;
#pragma unroll
        for (int i = 0; i < ACH; ++i) {
            const int c = tid + NT * i, r = c >> 3, kc = (c & 7) * 8;
            const int gm = m0 + r, gk = kbase + kc;
            ra[i] = (c < BM * 8 && gm < M && gk < K) ? ldg16(A + (long)gm * lda + gk) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
            for (int i = 0; i < BCH; ++i) {
                const int c = tid + NT * i, r = c >> 3, kc = (c & 7) * 8;
                const int gn = n0 + r, gk = kbase + kc;
                rb[b][i] = (c < BN * 8 && gn < N && gk < K) ? ldg16(W + b * up_off + (long)gn * ldw + gk)
                                                             : make_uint4(0, 0, 0, 0);
            }
    };
    auto lstore = [&](int buf, const uint4 (&ra)[ACH], const uint4 (&rb)[NB][BCH]) {
#pragma unroll
        for (int i = 0; i < ACH; ++i) {
            const int c = tid + NT * i, r = c >> 3, kc = (c & 7) * 8;
            if (c < BM * 8) *reinterpret_cast<uint4*>(As + (buf * BM + r) * LDSK + kc) = ra[i];
        }
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
            for (int i = 0; i < BCH; ++i) {
                const int c = tid + NT * i, r = c >> 3, kc = (c & 7) * 8;
                if (c < BN * 8) *reinterpret_cast<uint4*>(Bs + ((buf * NB + b) * BN + r) * LDSK + kc) = rb[b][i];
            }
    };
    auto compute = [&](int buf) {
#pragma unroll
        for (int kk = 0; kk < BK / 32; ++kk) {
            const int kof = kk * 32 + 8 * (lane >> 4);
            short8 af[TM], bfr[NB][TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
                af[i] = *reinterpret_cast<const short8*>(As + (buf * BM + (wr * TM + i) * 16 + (lane & 15)) * LDSK + kof);
#pragma unroll
            for (int b = 0; b < NB; ++b)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    bfr[b][j] = *reinterpret_cast<const short8*>(
                        Bs + ((buf * NB + b) * BN + (wc * TN + j) * 16 + (lane & 15)) * LDSK + kof);
#pragma unroll
            for (int b = 0; b < NB; ++b)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) acc[b][i][j] = mfma16(af[i], bfr[b][j], acc[b][i][j]);
        }
    };

    if (nkt > 0) gload(kt0, ra0, rb0);
    if (nkt > 1) gload(kt0 + 1, ra1, rb1);
    if (nkt > 0) lstore(0, ra0, rb0);
    __syncthreads();
    // iteration t: issue loads of t+2 into the register set that held t, multiply buffer t&1,
    // write tile t+1 (loaded one iteration earlier) into the other buffer, barrier
    for (int t = 0; t < nkt; t += 2) {
        if (t + 2 < nkt) gload(kt0 + t + 2, ra0, rb0);
        compute(0);
        if (t + 1 < nkt) lstore(1, ra1, rb1);
        __syncthreads();
        if (t + 1 >= nkt) break;
        if (t + 3 < nkt) gload(kt0 + t + 3, ra1, rb1);
        compute(1);
        if (t + 2 < nkt) lstore(0, ra0, rb0);
        __syncthreads();
    }

    // C/D map of 16x16x32: col = lane & 15, row = (lane >> 4) * 4 + r
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + (wc * TN + j) * 16 + (lane & 15);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + (wr * TM + i) * 16 + (lane >> 4) * 4 + r;
                if (m < M && n < N) {
                    if constexpr (SPLIT) {
                        ws[((long)blockIdx.z * M + m) * N + n] = acc[0][i][j][r];
                    } else {
                        epi_store<EPI>(ea, m, n, acc[0][i][j][r], DUAL ? acc[NB - 1][i][j][r] : 0.f);
                    }
                }
            }
        }
}

// split-K reduction in fixed z order + epilogue (4 consecutive outputs per thread)
template <int EPI>
__global__ void k_splitk_epi(const float* __restrict__ ws, int S, int M, int N, EpiArgs ea) {
    const long total = (long)M * N;
    for (long i4 = blockIdx.x * (long)blockDim.x + threadIdx.x; i4 * 4 < total; i4 += (long)gridDim.x * blockDim.x) {
        const long i = i4 * 4;
        f32x4 a = {0.f, 0.f, 0.f, 0.f};
        for (int z = 0; z < S; ++z) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(ws + (long)z * total + i);
            a += v;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) epi_store<EPI>(ea, (int)((i + j) / N), (int)((i + j) % N), a[j], 0.f);
    }
}

// ---------------------------------------------------------------- panel GEMM (LDS-DMA ring)
// One 256-thread workgroup (one wave per SIMD, 1 workgroup per CU) owns BM = 2*TM*16 rows x
// BN = 2*TN*16 columns (per B operand; NB = 2 for the dual gate/up GEMM).  Both operands go
// global -> LDS by LDS-DMA (global_load_lds_dwordx4, 1 KiB = 8 rows x 128 B per wave
// instruction) into an ST-slot ring of 64-deep k-tiles; the loads of tile t+ST-1 are issued
// right after the barrier that retires tile t and stay in flight across the next barriers
// (counted vmcnt, raw s_barrier).  LDS rows are 128 B with the 16-B chunk index XOR-ed by
// (row & 7): the swizzle is applied to each lane's SOURCE address (LDS-DMA destinations are
// lane-linear), and the matching XOR on the ds_read_b128 fragment reads makes them
// bank-conflict free.  K tails (K % 64, e.g. SigLIP fc2 K = 4304) read a zero block.
// Waves form a 2 x 2 grid; wave (wm, wn) owns TM x TN (x NB) 16x16 MFMA tiles.
__device__ __attribute__((aligned(16))) uint4 g_zero_chunk[1] = {{0u, 0u, 0u, 0u}};

// s_waitcnt vmcnt(G * n) for a runtime n in [0, NMAX] (the count must be an immediate)
template <int G, int NMAX>
__device__ __forceinline__ void vm_wait_tiles(int n) {
    if constexpr (NMAX >= 1) {
        if (n >= NMAX) {
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G * NMAX) : "memory");
            return;
        }
        vm_wait_tiles<G, NMAX - 1>(n);
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

// XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs (linear block id lin = x +
// y * gridDim.x -> XCD lin % 8; observed placement, used for speed only), and each XCD has its own
// L2.  The (column tile nt, K slice z, row tile mt) triples are listed column-tile-major -- the row
// tiles of one (nt, z) weight panel adjacent -- and the list is cut into 8 contiguous runs, one per
// XCD (run x = the blocks lin % 8 == x, in order).  So the n_mt workgroups that read one weight panel
// sit on one XCD and its L2 serves the panel to all but the first; only panels at a run boundary
// are fetched by two XCDs.
//
// Round 4: when the grid splits into 8 equal blocks of bm row tiles x bn column tiles x bs K slices
// (the host's xcd_block picks the shape that minimises the bytes each XCD must bring into its L2 --
// bs/S of K x (bm row panels + bn weight panels) -- and passes it as `code`: bm | bn << 6 | bs << 14;
// bit 30 is k_gemm_w's weight cache policy), XCD x takes block x instead of a run: the batched prefill
// GEMMs otherwise read the whole activation panel on every XCD (8-image down projection: 718 MB per
// launch fetched for ≈180 MB of operands).  Inside a block the row tiles of one weight panel stay adjacent.
__host__ __device__ __forceinline__ void xcd_tile_of(int lin, int gx, int S, int n_mt, int code, int& mt, int& nt,
                                                     int& z) {
    const int xb = code & 0x3FFFF;
    const int G = gx * S;
    const int x = lin & 7, j = lin >> 3;
    if (xb) {
        const int bm = xb & 63, bn = (xb >> 6) & 255, bs = xb >> 14;
        const int n_nt = G / (n_mt * S);
        const int gm = n_mt / bm, gn = n_nt / bn;
        const int xm = x % gm, xn = (x / gm) % gn, xs = x / (gm * gn);
        const int jm = j % bm, js = (j / bm) % bs, jn = j / (bm * bs);
        mt = xm * bm + jm;
        z = xs * bs + js;
        nt = xn * bn + jn;
        return;
    }
    const int q = G >> 3, r = G & 7;
    const int idx = x * q + (x < r ? x : r) + j;
    mt = idx % n_mt;
    z = (idx / n_mt) % S;
    nt = idx / (n_mt * S);
}

__device__ __forceinline__ void xcd_tile(int n_mt, int code, int& mt, int& nt, int& z) {
    xcd_tile_of(blockIdx.x + blockIdx.y * gridDim.x, gridDim.x, gridDim.y, n_mt, code, mt, nt, z);
}

template <int NW, int WM, int TM, int TN, int NB, int ST, int EPI, bool SPLIT>
__global__ void __launch_bounds__(64 * NW, 1) k_gemm_p(const uint16_t* __restrict__ A, int lda,
                                                   const uint16_t* __restrict__ W, int ldw, int M, int N, int K,
                                                   int kt_per_split, EpiArgs ea, float* __restrict__ ws, long up_off,
                                                   int n_mt, int code) {
    constexpr int WN = NW / WM;
    constexpr int BM = WM * TM * 16, BN = WN * TN * 16;
    constexpr int APC = BM / 8, BPC = NB * BN / 8;  // 1-KiB pieces per k-tile
    constexpr int PCS = APC + BPC;
    // LDS-DMA instructions per wave per k-tile; with 8 waves the last few waves re-load a piece
    // (same bytes to the same LDS address) so every wave issues GPW and one vmcnt count fits all
    constexpr int GPW = (PCS + NW - 1) / NW;
    constexpr int ABYTES = BM * 128;
    constexpr int SBYTES = (BM + NB * BN) * 128;    // one ring slot
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_p[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    static_assert(NW == 4 || NW == 8, "4 or 8 waves");
    const int wm = wave / WN, wn = wave % WN;
    // tile coordinates: the row tiles of one weight panel on one XCD (xcd_tile)
    int mt, nt, z;
    xcd_tile(n_mt, code, mt, nt, z);
    const int m0 = mt * BM, n0 = nt * BN;
    const int nkt_total = (K + 63) / 64;
    const int kt0 = z * kt_per_split;
    int kt1 = kt0 + kt_per_split;
    if (kt1 > nkt_total) kt1 = nkt_total;
    const int nkt = kt1 - kt0;

    // per-lane source rows of this wave's pieces (piece p = wave + NW i)
    const uint16_t* src[GPW];
    int gk[GPW];    // element offset of the lane's chunk inside a 64-wide k-tile
    int loff[GPW];  // piece offset in a ring slot (wave-uniform)
    const int prow = lane >> 3;
    const int pchunk = lane & 7;
#pragma unroll
    for (int i = 0; i < GPW; ++i) {
        int p = wave + NW * i;
        if (p >= PCS) p -= PCS;  // padding: repeat a piece
        loff[i] = p * 1024;
        int row;
        const uint16_t* base;
        long ld;
        if (p < APC) {
            row = m0 + p * 8 + prow;
            if (row > M - 1) row = M - 1;  // rows past M: valid memory, results never stored
            base = A;
            ld = lda;
        } else {
            const int q = p - APC;
            const int bo = q / (BN / 8);
            row = n0 + (q % (BN / 8)) * 8 + prow;
            if constexpr (EPI == EPI_ROPE) row = rope_row(row, BN);
            if (row > N - 1) row = N - 1;
            base = W + bo * up_off;
            ld = ldw;
        }
        // lane (row r, LDS chunk c) fetches global chunk c ^ (r & 7)
        gk[i] = (pchunk ^ (row & 7)) * 8;
        src[i] = base + (long)row * ld + gk[i];
    }
    // slot image is piece-linear: A pieces first, then B pieces (piece p at p KiB)
#define PGMI_LDS_AT(slot, i) ((__attribute__((address_space(3))) void*)(smem_p + (slot) * SBYTES + loff[i]))
    const uint16_t* zero = reinterpret_cast<const uint16_t*>(g_zero_chunk);
    auto issue = [&](int kt, int slot) {
        if constexpr (PGMI_GEMM_DIAG & 2) return;
        const int kel = kt * 64;
        if (kel + 64 <= K) {
#pragma unroll
            for (int i = 0; i < GPW; ++i)
                __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src[i] + kel), PGMI_LDS_AT(slot, i), 16, 0, 0);
        } else {  // K tail: chunks at or past K read zeros (K % 8 == 0)
#pragma unroll
            for (int i = 0; i < GPW; ++i) {
                const uint16_t* g = (kel + gk[i] < K) ? src[i] + kel : zero;
                __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(g), PGMI_LDS_AT(slot, i), 16, 0, 0);
            }
        }
    };

    f32x4 acc[NB][TM][TN];
#pragma unroll
    for (int bb = 0; bb < NB; ++bb)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[bb][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int swz = lane & 7;  // fragment rows are 16-aligned + (lane & 15): row & 7 == lane & 7
    const int arow0 = (wm * TM * 16 + (lane & 15)) * 128;
    const int brow0 = ABYTES + (wn * TN * 16 + (lane & 15)) * 128;
    // fragments of one 32-deep k step (kk = 0, 1 of a 64-deep tile), two register sets
    short8 fa0[TM], fb0[NB][TN], fa1[TM], fb1[NB][TN];
#define PGMI_SB() __builtin_amdgcn_sched_barrier(0)
#define PGMI_READ_FRAGS(FA, FB, SLOT, KK)                                                                   \
    do {                                                                                                    \
        const uint8_t* sb_ = smem_p + (SLOT) * SBYTES;                                                      \
        const int ch_ = ((((KK) * 4) + (lane >> 4)) ^ swz) << 4;                                            \
        _Pragma("unroll") for (int i_ = 0; i_ < TM; ++i_) FA[i_] =                                          \
            *reinterpret_cast<const short8*>(sb_ + arow0 + i_ * 16 * 128 + ch_);                            \
        _Pragma("unroll") for (int b_ = 0; b_ < NB; ++b_) _Pragma("unroll") for (int j_ = 0; j_ < TN; ++j_) \
            FB[b_][j_] = *reinterpret_cast<const short8*>(sb_ + brow0 + (b_ * BN + j_ * 16) * 128 + ch_);   \
    } while (0)
#define PGMI_MFMAS(FA, FB)                                                                                  \
    do {                                                                                                    \
        if constexpr (PGMI_GEMM_DIAG & 1) { diag_consume<TM, TN, NB>(FA, FB); break; }                      \
        _Pragma("unroll") for (int b_ = 0; b_ < NB; ++b_) _Pragma("unroll") for (int i_ = 0; i_ < TM; ++i_) \
            _Pragma("unroll") for (int j_ = 0; j_ < TN; ++j_) acc[b_][i_][j_] =                              \
                mfma16(FA[i_], FB[b_][j_], acc[b_][i_][j_]);                                                \
    } while (0)

    // epilogue operands first (see epi_load): held in registers through the k loop
    const int epi_mb = m0 + wm * TM * 16, epi_nb = n0 + wn * TN * 16;
    EpiOps<EPI, TM, TN> epi_ops;
    if constexpr (!SPLIT) epi_load<EPI, TM, TN>(ea, M, N, epi_mb, epi_nb, lane, epi_ops);
    RopeOps<EPI == EPI_ROPE ? TM : 1> rope_ops;
    if constexpr (!SPLIT && EPI == EPI_ROPE) rope_load<TM, BN>(ea, M, epi_mb, epi_nb, lane, rope_ops);

    // ring: tiles t+1 .. t+ST-1 in flight or landed while tile t is multiplied.  Per tile:
    //   read kk=1 fragments | MFMAs kk=0 | retire tile t+1, barrier, refill the slot tile t
    //   lived in with tile t+ST | read tile t+1's kk=0 fragments | MFMAs kk=1
    // so every fragment read is covered by a block of MFMAs and the LDS-DMA of a tile has
    // ST-1 tiles of MFMAs to land.
#pragma unroll
    for (int sI = 0; sI < ST; ++sI)
        if (sI < nkt) issue(kt0 + sI, sI);
    if (nkt > 0) {
        vm_wait_tiles<GPW, ST - 1>((nkt < ST ? nkt : ST) - 1);
        __builtin_amdgcn_s_barrier();
        PGMI_READ_FRAGS(fa0, fb0, 0, 0);
    }
    int slot = 0;
    for (int t = 0; t < nkt; ++t) {
        // the kk=0 fragments (read behind the previous MFMA block) have landed; a real s_waitcnt
        // (not asm) so the compiler's counter model knows nothing older is outstanding and does
        // not drain the kk=1 reads below before the first MFMA
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
        PGMI_READ_FRAGS(fa1, fb1, slot, 1);
        PGMI_SB();
        PGMI_MFMAS(fa0, fb0);
        PGMI_SB();
        if (t + 1 < nkt) {
            // tiles issued so far: min(nkt, t + ST); tile t+1 must have landed
            const int ahead = (nkt - t - 2) < (ST - 2) ? (nkt - t - 2) : (ST - 2);
            vm_wait_tiles<GPW, ST - 2>(ahead);
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): kk=1 reads done before the slot is refilled
        __builtin_amdgcn_s_barrier();
        PGMI_SB();
        if (t + ST < nkt) issue(kt0 + t + ST, slot);
        const int nslot = slot + 1 == ST ? 0 : slot + 1;
        if (t + 1 < nkt) PGMI_READ_FRAGS(fa0, fb0, nslot, 0);
        PGMI_SB();
        PGMI_MFMAS(fa1, fb1);
        PGMI_SB();
        slot = nslot;
    }
#undef PGMI_READ_FRAGS
#undef PGMI_MFMAS
#undef PGMI_SB

    // C/D map of 16x16x32: col = lane & 15, row = (lane >> 4) * 4 + r
    if constexpr (SPLIT) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int n = n0 + (wn * TN + j) * 16 + (lane & 15);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int m = m0 + (wm * TM + i) * 16 + (lane >> 4) * 4 + r;
                    if (m < M && n < N) ws[((long)z * M + m) * N + n] = acc[0][i][j][r];
                }
            }
    } else if constexpr (EPI == EPI_ROPE) {
        rope_apply<TM>(ea, M, epi_mb, lane, rope_ops, acc[0]);
    } else {
        epi_apply<EPI, TM, TN>(ea, M, N, epi_mb, epi_nb, lane, epi_ops, acc[0], acc[NB - 1]);
    }
}

// ---------------------------------------------------------------- warp-specialised panel GEMM
// k_gemm_p's tiles, LDS image and fragment reads, with the two roles split over the waves of the
// workgroup: NW compute waves (the WM x WN wave grid) only read fragments and run MFMAs; LW loader
// waves only issue the LDS-DMA of the ring (k_gemm_p's waves issue both, and an LDS-DMA issue stalls
// its wave for ~60-185 cycles per KiB beside MFMAs -- at the prefill's M = 256..288 panels that
// stall, not the matrix pipe, set the k-step time).  One raw s_barrier per k-tile: before barrier t
// every loader has counted its own DMA of tile t as landed (vmcnt), after it the loaders refill the
// slot of tile t-1 (whose fragments every compute wave read before reaching barrier t).
template <int NW, int WM, int TM, int TN, int NB, int ST, int LW, int EPI, bool SPLIT, bool RL = false>
__global__ void __launch_bounds__(64 * (NW + LW), 1) k_gemm_w(const uint16_t* __restrict__ A, int lda,
                                                          const uint16_t* __restrict__ W, int ldw, int M, int N, int K,
                                                          int kt_per_split, EpiArgs ea, float* __restrict__ ws,
                                                          long up_off, int n_mt, int code) {
    constexpr int WN = NW / WM;
    constexpr int BM = WM * TM * 16, BN = WN * TN * 16;
    constexpr int APC = BM / 8, BPC = NB * BN / 8;  // 1-KiB pieces per k-tile
    constexpr int PCS = APC + BPC;
    constexpr int GPW = (PCS + LW - 1) / LW;        // LDS-DMA instructions per loader wave per k-tile
    constexpr int ABYTES = BM * 128;
    constexpr int SBYTES = (BM + NB * BN) * 128;
    static_assert(ST >= 2, "ring of at least two slots");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_w[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int mt, nt, z;
    xcd_tile(n_mt, code, mt, nt, z);
    const int m0 = mt * BM, n0 = nt * BN;
    const int nkt_total = (K + 63) / 64;
    const int kt0 = z * kt_per_split;
    int kt1 = kt0 + kt_per_split;
    if (kt1 > nkt_total) kt1 = nkt_total;
    const int nkt = kt1 > kt0 ? kt1 - kt0 : 0;

    if (wave >= NW) {
        // ---------------- loader wave
        const int lw = wave - NW;
        const uint16_t* src[GPW];
        int gk[GPW], loff[GPW];
        const int prow = lane >> 3, pchunk = lane & 7;
#pragma unroll
        for (int i = 0; i < GPW; ++i) {
            int p = lw + LW * i;
            if (p >= PCS) p -= PCS;  // padding: repeat a piece (same bytes to the same LDS address)
            loff[i] = p * 1024;
            int row;
            const uint16_t* base;
            long ld;
            if (p < APC) {
                row = m0 + p * 8 + prow;
                if (row > M - 1) row = M - 1;
                base = A;
                ld = lda;
            } else {
                const int q = p - APC;
                const int bo = q / (BN / 8);
                row = n0 + (q % (BN / 8)) * 8 + prow;
                if constexpr (EPI == EPI_ROPE) row = rope_row(row, BN);
                if (row > N - 1) row = N - 1;
                base = W + bo * up_off;
                ld = ldw;
            }
            gk[i] = (pchunk ^ (row & 7)) * 8;
            src[i] = base + (long)row * ld + gk[i];
        }
        const uint16_t* zero = reinterpret_cast<const uint16_t*>(g_zero_chunk);
        // one row tile (n_mt == 1, flagged in bit 30 of code by launch_w): every weight byte is read by one
        // workgroup once, so those pieces stream non-temporal; the activation panel, which every workgroup
        // re-reads, keeps the default policy.  Same box (tools/archive/gpu_r4l.sh, the M = 288 gate|up): 43.1 / 43.8 /
        // 43.3 -> 41.2 / 41.7 / 41.4 us in situ, 224 px prefill 3.80 -> 3.77-3.79 ms
        const bool wnt = (code >> 30) & 1;
        auto issue = [&](int kt, int slot) {
            if constexpr (PGMI_GEMM_DIAG & 2) return;
            const int kel = kt * 64;
            if (kel + 64 <= K) {
#pragma unroll
                for (int i = 0; i < GPW; ++i) {
                    const int p = lw + LW * i < PCS ? lw + LW * i : lw + LW * i - PCS;
                    if (wnt && p >= APC)
                        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src[i] + kel),
                                                         (__attribute__((address_space(3))) void*)(smem_w + slot * SBYTES + loff[i]),
                                                         16, 0, 2);
                    else
                        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src[i] + kel),
                                                         (__attribute__((address_space(3))) void*)(smem_w + slot * SBYTES + loff[i]),
                                                         16, 0, 0);
                }
            } else {
#pragma unroll
                for (int i = 0; i < GPW; ++i) {
                    const uint16_t* g = (kel + gk[i] < K) ? src[i] + kel : zero;
                    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(g),
                                                     (__attribute__((address_space(3))) void*)(smem_w + slot * SBYTES + loff[i]),
                                                     16, 0, 0);
                }
            }
        };
#pragma unroll
        for (int sI = 0; sI < ST - 1; ++sI)
            if (sI < nkt) issue(kt0 + sI, sI);
        int slot_next = ST - 1;  // slot of tile t + ST - 1
        for (int t = 0; t < nkt; ++t) {
            const int issued = (nkt < t + ST - 1) ? nkt : t + ST - 1;
            vm_wait_tiles<GPW, ST - 2>(issued - t - 1);  // tile t landed
            __builtin_amdgcn_s_barrier();
            if (t + ST - 1 < nkt) issue(kt0 + t + ST - 1, slot_next);
            slot_next = slot_next + 1 == ST ? 0 : slot_next + 1;
        }
        return;
    }

    // ---------------- compute wave
    const int wm = wave / WN, wn = wave % WN;
    RopeOps<EPI == EPI_ROPE ? TM : 1> rope_ops;
    if constexpr (!SPLIT && EPI == EPI_ROPE) rope_load<TM, BN>(ea, M, m0 + wm * TM * 16, n0 + wn * TN * 16, lane, rope_ops);
    f32x4 acc[NB][TM][TN];
#pragma unroll
    for (int bb = 0; bb < NB; ++bb)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[bb][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int swz = lane & 7;
    const int arow0 = (wm * TM * 16 + (lane & 15)) * 128;
    const int brow0 = ABYTES + (wn * TN * 16 + (lane & 15)) * 128;
#ifndef PGMI_GEMM_W_PIPE
#define PGMI_GEMM_W_PIPE 1
#endif
    // (two fragment sets: taller wave tiles than TM 9 spill at three waves per SIMD)
    // (and not when the accumulators plus two fragment sets pass ~200 registers: W144q's 144 accumulators)
    constexpr bool PIPE = !RL && PGMI_GEMM_W_PIPE && TM <= 9 && EPI != EPI_ROPE &&  // (RoPE: its operands spill)
                          2 * (TM + NB * TN) * 4 + NB * TM * TN * 4 <= 200;
    if constexpr (RL) {
    // In-wave reload (round 6, the RL configurations: one compute wave per SIMD with a wide wave tile, so each
    // fragment read feeds 2 NB TN MFMAs): one set of A fragments, each row tile's reloaded for the next 32-deep
    // step right behind the MFMAs that read it, and two sets of B fragments (the next step's read first), so
    // the step's later rows multiply while the next step's fragments land -- a single wave overlaps its own LDS
    // reads with its MFMAs, which k_gemm_w's lock-stepped pairs of waves did not (the M = 288 gate|up's
    // diagnostic builds: 33.5 us with no LDS-DMA at all for 15.4 us of MFMA issue).  Per tile t:
    //   (t, 0) landed | read B (t, 1) | rows: MFMA (t, 0), read A (t, 1) | lgkmcnt(0), barrier t + 1 (tile t's
    //   reads are done: the loaders refill its slot) | read B (t + 1, 0) | rows: MFMA (t, 1), read A (t + 1, 0)
    static_assert(EPI != EPI_ROPE, "in-wave reload: no RoPE epilogue");
    short8 fa[TM], fbA[NB][TN], fbB[NB][TN];
#define PGMI_R_CH(KK) (((((KK) * 4) + (lane >> 4)) ^ swz) << 4)
#define PGMI_R_A(I, SB, KK) fa[I] = *reinterpret_cast<const short8*>((SB) + arow0 + (I) * 16 * 128 + PGMI_R_CH(KK))
#define PGMI_R_B(FB, SB, KK)                                                                                \
    do {                                                                                                    \
        _Pragma("unroll") for (int b_ = 0; b_ < NB; ++b_) _Pragma("unroll") for (int j_ = 0; j_ < TN; ++j_) \
            FB[b_][j_] = *reinterpret_cast<const short8*>((SB) + brow0 + (b_ * BN + j_ * 16) * 128 + PGMI_R_CH(KK)); \
    } while (0)
#define PGMI_R_ROW(I, FB)                                                                                   \
    do {                                                                                                    \
        if constexpr (PGMI_GEMM_DIAG & 1) {                                                                 \
            asm volatile("" ::"v"(fa[I]));                                                                  \
        } else {                                                                                            \
            _Pragma("unroll") for (int b_ = 0; b_ < NB; ++b_) _Pragma("unroll") for (int j_ = 0; j_ < TN; ++j_) \
                acc[b_][I][j_] = mfma16(fa[I], FB[b_][j_], acc[b_][I][j_]);                                 \
        }                                                                                                   \
    } while (0)
#define PGMI_R_DIAGB(FB)                                                                                    \
    do {                                                                                                    \
        if constexpr (PGMI_GEMM_DIAG & 1) {                                                                 \
            _Pragma("unroll") for (int b_ = 0; b_ < NB; ++b_) _Pragma("unroll") for (int j_ = 0; j_ < TN; ++j_) \
                asm volatile("" ::"v"(FB[b_][j_]));                                                         \
        }                                                                                                   \
    } while (0)
    int slot = 0;
    if (nkt > 0) {
        __builtin_amdgcn_s_barrier();  // tile 0 is in slot 0
#pragma unroll
        for (int i = 0; i < TM; ++i) PGMI_R_A(i, smem_w, 0);
        PGMI_R_B(fbA, smem_w, 0);
    }
    // every tile but the last (no branch inside the step: a step with and one without the reloads as two arms
    // of one loop body made hipcc copy the accumulators between register assignments and spill)
    for (int t = 0; t + 1 < nkt; ++t) {
        const uint8_t* sb = smem_w + slot * SBYTES;
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): (t, 0)'s fragments
        __builtin_amdgcn_sched_barrier(0);
        PGMI_R_B(fbB, sb, 1);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            PGMI_R_ROW(i, fbA);
            PGMI_R_A(i, sb, 1);
            __builtin_amdgcn_sched_barrier(0);  // the reload stays behind the MFMAs that read fa[i]
        }
        PGMI_R_DIAGB(fbA);
        __builtin_amdgcn_s_waitcnt(0xC07F);  // (t, 1)'s fragments: every read of tile t has landed
        __builtin_amdgcn_sched_barrier(0);
        slot = slot + 1 == ST ? 0 : slot + 1;
        const uint8_t* nb = smem_w + slot * SBYTES;
        __builtin_amdgcn_s_barrier();        // tile t + 1 landed; the loaders may refill tile t's slot
        __builtin_amdgcn_sched_barrier(0);
        PGMI_R_B(fbA, nb, 0);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            PGMI_R_ROW(i, fbB);
            PGMI_R_A(i, nb, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
        PGMI_R_DIAGB(fbB);
    }
    if (nkt > 0) {  // the last tile
        const uint8_t* sb = smem_w + slot * SBYTES;
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
        PGMI_R_B(fbB, sb, 1);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            PGMI_R_ROW(i, fbA);
            PGMI_R_A(i, sb, 1);
            __builtin_amdgcn_sched_barrier(0);
        }
        PGMI_R_DIAGB(fbA);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < TM; ++i) PGMI_R_ROW(i, fbB);
        PGMI_R_DIAGB(fbB);
    }
#undef PGMI_R_CH
#undef PGMI_R_A
#undef PGMI_R_B
#undef PGMI_R_ROW
#undef PGMI_R_DIAGB
    } else if constexpr (PIPE) {
    // Fragment reads pipelined across the barrier (k_gemm_p's schedule): per tile t,
    //   read kk=1 fragments of t | MFMAs kk=0 | lgkmcnt(0), barrier t+1 (tile t+1 landed; the loaders
    //   may now refill t's slot: its fragments are all in registers) | read kk=0 fragments of t+1 |
    //   MFMAs kk=1 of t
    // so the LDS latency of a tile's first fragments hides behind the previous tile's second MFMA
    // block, and a wave's barrier wait overlaps nothing but its own issued reads.  The loader side is
    // unchanged: nkt barriers in all (one before the loop, one inside each iteration but the last).
    short8 fa0[TM], fb0[NB][TN], fa1[TM], fb1[NB][TN];
#define PGMI_W_READ(FA, FB, SB, KK)                                                                        \
    do {                                                                                                   \
        const int ch_ = ((((KK) * 4) + (lane >> 4)) ^ swz) << 4;                                           \
        _Pragma("unroll") for (int i_ = 0; i_ < TM; ++i_) FA[i_] =                                         \
            *reinterpret_cast<const short8*>((SB) + arow0 + i_ * 16 * 128 + ch_);                          \
        _Pragma("unroll") for (int b_ = 0; b_ < NB; ++b_) _Pragma("unroll") for (int j_ = 0; j_ < TN; ++j_) \
            FB[b_][j_] = *reinterpret_cast<const short8*>((SB) + brow0 + (b_ * BN + j_ * 16) * 128 + ch_); \
    } while (0)
#define PGMI_W_MFMA(FA, FB)                                                                                \
    do {                                                                                                   \
        if constexpr (PGMI_GEMM_DIAG & 1) { diag_consume<TM, TN, NB>(FA, FB); break; }                     \
        _Pragma("unroll") for (int b_ = 0; b_ < NB; ++b_) _Pragma("unroll") for (int i_ = 0; i_ < TM; ++i_) \
            _Pragma("unroll") for (int j_ = 0; j_ < TN; ++j_) acc[b_][i_][j_] =                             \
                mfma16(FA[i_], FB[b_][j_], acc[b_][i_][j_]);                                               \
    } while (0)
    int slot = 0;
    if (nkt > 0) {
        __builtin_amdgcn_s_barrier();  // tile 0 is in slot 0
        PGMI_W_READ(fa0, fb0, smem_w, 0);
    }
    for (int t = 0; t < nkt; ++t) {
        const uint8_t* sb = smem_w + slot * SBYTES;
        // the kk=0 fragments (read behind the previous MFMA block) have landed: a real s_waitcnt (not asm), so
        // the compiler's counter model knows nothing older is outstanding and does not drain the kk=1 reads
        // below before the first MFMA (without it the loop-carried reads made it emit lgkmcnt(0) there, and
        // the kk=1 fragment reads ran exposed instead of under the kk=0 MFMAs)
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
        PGMI_W_READ(fa1, fb1, sb, 1);
        __builtin_amdgcn_sched_barrier(0);
        PGMI_W_MFMA(fa0, fb0);
        __builtin_amdgcn_sched_barrier(0);
        slot = slot + 1 == ST ? 0 : slot + 1;
        if (t + 1 < nkt) {
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): tile t's fragments are in registers
            __builtin_amdgcn_s_barrier();        // tile t+1 is in slot `slot`
            __builtin_amdgcn_sched_barrier(0);
            PGMI_W_READ(fa0, fb0, smem_w + slot * SBYTES, 0);
        } else {
            // last tile: its kk=1 fragments must be in.  Waiting here (not at the join below) keeps the
            // counter model exact on both paths, so the kk=1 MFMAs of the other tiles do not wait for the
            // next tile's kk=0 reads issued after the barrier (the merged state made hipcc emit lgkmcnt(1))
            __builtin_amdgcn_s_waitcnt(0xC07F);
        }
        __builtin_amdgcn_sched_barrier(0);
        PGMI_W_MFMA(fa1, fb1);
        __builtin_amdgcn_sched_barrier(0);
    }
#undef PGMI_W_READ
#undef PGMI_W_MFMA
    } else {
    short8 fa[TM], fb[NB][TN];
    int slot = 0;
    for (int t = 0; t < nkt; ++t) {
        __builtin_amdgcn_s_barrier();  // tile t is in slot `slot`
        const uint8_t* sb = smem_w + slot * SBYTES;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int ch = (((kk * 4) + (lane >> 4)) ^ swz) << 4;
#pragma unroll
            for (int i = 0; i < TM; ++i) fa[i] = *reinterpret_cast<const short8*>(sb + arow0 + i * 16 * 128 + ch);
#pragma unroll
            for (int bb = 0; bb < NB; ++bb)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    fb[bb][j] = *reinterpret_cast<const short8*>(sb + brow0 + (bb * BN + j * 16) * 128 + ch);
#pragma unroll
            for (int bb = 0; bb < NB; ++bb)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) acc[bb][i][j] = mfma16(fa[i], fb[bb][j], acc[bb][i][j]);
        }
        slot = slot + 1 == ST ? 0 : slot + 1;
    }
    }
    if constexpr (SPLIT) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int n = n0 + (wn * TN + j) * 16 + (lane & 15);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int m = m0 + (wm * TM + i) * 16 + (lane >> 4) * 4 + r;
                    if (m < M && n < N) ws[((long)z * M + m) * N + n] = acc[0][i][j][r];
                }
            }
    } else if constexpr (EPI == EPI_ROPE) {
        rope_apply<TM>(ea, M, m0 + wm * TM * 16, lane, rope_ops, acc[0]);
    } else {
        epi_tile<EPI, TM, TN>(ea, M, N, m0 + wm * TM * 16, n0 + wn * TN * 16, lane, acc[0], acc[NB - 1]);
    }
}

// ---------------------------------------------------------------- 8-phase GEMM (large M)
// BM x 256 x 64 tiles (BM = 32 TM: 256 at TM 8), one 512-thread workgroup per CU, 8 waves in a
// 2 (M) x 4 (N) grid, each wave TM x 4 MFMA tiles (TM x 2 gate + TM x 2 up for the dual GeGLU GEMM).
// A wave's output splits into 4 quadrants (row half qa x column half qb); the LDS image of a K-tile
// is cut the same way into 4 half-tiles -- A_qa = the qa-th row half of BOTH wave rows, B_qb = the
// qb-th column half of all 4 wave columns -- so each phase reads exactly one A half and / or one B
// half.  Two K-tiles per iteration, 8 phases (quadrant order (0,0) (0,1) (1,1) (1,0): every phase
// but the first reuses the other operand's fragments from registers), each phase
//   ds_read its fragments | LDS-DMA one half-tile of a later K-tile | [vmcnt] | s_barrier |
//   lgkmcnt(0) | 16 MFMAs (setprio 1) | s_barrier
// with the two wave rows staggered by one barrier (ping-pong: one wave of each SIMD in its MFMA
// cluster while the other reads and stages) and four half-tiles in flight across every barrier:
// cdna_hip_programming.md's 256^2 8-phase template, restated for this LDS image, with B0's
// fragments kept in registers across the tile (one fewer fragment read per K-tile).
// LDS rows are 128 B with the 16-B chunk XOR-swizzled by (row & 7) on the DMA's source address.
template <int TM, int EPI, bool SPLIT>
__global__ void __launch_bounds__(512, 1) k_gemm_8p(const uint16_t* __restrict__ A, int lda,
                                                    const uint16_t* __restrict__ W, int ldw, int M, int N, int K,
                                                    int kt_per_split, EpiArgs ea, float* __restrict__ ws, long up_off,
                                                    int n_mt, int code) {
    static_assert(TM % 2 == 0, "row halves of whole 16-row tiles");
    constexpr bool DUAL = (EPI == EPI_GEGLU);
    constexpr int H = TM / 2;                 // row tiles per quadrant
    constexpr int BM = 32 * TM;
    constexpr int HAR = 16 * TM;              // rows of an A half image (H tiles of each wave row)
    constexpr int HAB = HAR * 128, HBB = 128 * 128;
    constexpr int PA = HAR / 8, PB = 16;      // 1-KiB pieces per half
    constexpr int GA = (PA + 7) / 8, GB = PB / 8;
    constexpr int TB = 2 * HAB + 2 * HBB;     // one K-tile buffer: A0 A1 B0 B1
    extern __shared__ __attribute__((aligned(16))) uint8_t sm8[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    int mt, nt, z;
    xcd_tile(n_mt, code, mt, nt, z);
    const int m0 = mt * BM, n0 = nt * (DUAL ? 128 : 256);
    const int nkt_total = K / 64;
    const int kt0 = z * kt_per_split;
    const int kt1 = kt0 + kt_per_split < nkt_total ? kt0 + kt_per_split : nkt_total;
    const int nkt = kt1 - kt0;
    if (nkt <= 0) return;

    // per-lane DMA sources (k = 0 of the tile's columns); piece p = wave + 8 i, pieces past the half
    // repeat an earlier one (same bytes to the same LDS address)
    const uint16_t* sa[2][GA];
    int la[GA];
    const uint16_t* sb[2][GB];
    int lb[GB];
    const int prow = lane >> 3, pch = lane & 7;
#pragma unroll
    for (int i = 0; i < GA; ++i) {
        int pc = wave + 8 * i;
        if (pc >= PA) pc -= PA;
        la[i] = pc * 1024;
        const int ir = pc * 8 + prow;
        const int wr = ir / (8 * TM), r = ir % (8 * TM);
#pragma unroll
        for (int qa = 0; qa < 2; ++qa) {
            int row = m0 + wr * 16 * TM + qa * 8 * TM + r;
            row = row < M ? row : M - 1;
            sa[qa][i] = A + (long)row * lda + ((pch ^ (ir & 7)) << 3);
        }
    }
#pragma unroll
    for (int i = 0; i < GB; ++i) {
        const int pc = wave + 8 * i;
        lb[i] = pc * 1024;
        const int ir = pc * 8 + prow;
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
            const uint16_t* wb = W;
            int row;
            if constexpr (DUAL) {
                row = n0 + (ir >> 5) * 32 + (ir & 31);  // gate rows (qb 0) / the same up rows (qb 1)
                if (qb) wb = W + up_off;
            } else {
                row = n0 + (ir >> 5) * 64 + qb * 32 + (ir & 31);
            }
            row = row < N ? row : N - 1;
            sb[qb][i] = wb + (long)row * ldw + ((pch ^ (ir & 7)) << 3);
        }
    }
#define PGMI_8P_LDS(off) ((__attribute__((address_space(3))) void*)(sm8 + (off)))
    auto stageA = [&](int qa, int kt, int buf) {
        if constexpr (PGMI_GEMM_DIAG & 2) return;
        kt = kt < kt1 ? kt : kt1 - 1;  // past the range: valid bytes into a buffer never read again
        const int kel = kt * 64;
        const int base = buf * TB + qa * HAB;
#pragma unroll
        for (int i = 0; i < GA; ++i)
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(sa[qa][i] + kel), PGMI_8P_LDS(base + la[i]), 16, 0, 0);
    };
    auto stageB = [&](int qb, int kt, int buf) {
        if constexpr (PGMI_GEMM_DIAG & 2) return;
        kt = kt < kt1 ? kt : kt1 - 1;
        const int kel = kt * 64;
        const int base = buf * TB + 2 * HAB + qb * HBB;
#pragma unroll
        for (int i = 0; i < GB; ++i)
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(sb[qb][i] + kel), PGMI_8P_LDS(base + lb[i]), 16, 0, 0);
    };
#undef PGMI_8P_LDS

    f32x4 acc[TM][4];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    short8 fa[H][2], fb[2][2][2];             // fb[qb]: B0's fragments stay live from phase 1 to 4
    const int sw = lane & 7;
    const int arow = (wm * 8 * TM + (lane & 15)) * 128;  // + i * 16 rows
    const int brow = (wn * 32 + (lane & 15)) * 128;      // + jj * 16 rows
    auto readA = [&](int qa, int buf) {
        const uint8_t* b = sm8 + buf * TB + qa * HAB + arow;
#pragma unroll
        for (int i = 0; i < H; ++i)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
                fa[i][kk] = *reinterpret_cast<const short8*>(b + i * 16 * 128 + (((kk * 4 + (lane >> 4)) ^ sw) << 4));
    };
    auto readB = [&](auto qb_c, int buf) {
        constexpr int QB = decltype(qb_c)::value;
        const uint8_t* b = sm8 + buf * TB + 2 * HAB + QB * HBB + brow;
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
                fb[QB][jj][kk] = *reinterpret_cast<const short8*>(b + jj * 16 * 128 + (((kk * 4 + (lane >> 4)) ^ sw) << 4));
    };
    auto mfmas = [&](auto qa_c, auto qb_c) {
        constexpr int QA = decltype(qa_c)::value, QB = decltype(qb_c)::value;
        if constexpr (PGMI_GEMM_DIAG & 1) {
#pragma unroll
            for (int i = 0; i < H; ++i)
#pragma unroll
                for (int kk = 0; kk < 2; ++kk) asm volatile("" ::"v"(fa[i][kk]), "v"(fb[QB][0][kk]), "v"(fb[QB][1][kk]));
            return;
        }
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int i = 0; i < H; ++i)
#pragma unroll
                for (int jj = 0; jj < 2; ++jj)
                    acc[QA * H + i][QB * 2 + jj] = mfma16(fa[i][kk], fb[QB][jj][kk], acc[QA * H + i][QB * 2 + jj]);
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    static_assert(GA == GB, "one vmcnt for every half-tile");
#define PGMI_8P_SB() __builtin_amdgcn_sched_barrier(0)
#define PGMI_8P_TAIL(QAC, QBC, DO)                                      \
    do {                                                                \
        __builtin_amdgcn_s_barrier();                                   \
        __builtin_amdgcn_s_waitcnt(0xC07F); /* lgkmcnt(0) */            \
        PGMI_8P_SB();                                                   \
        __builtin_amdgcn_s_setprio(1);                                  \
        if (DO) mfmas(QAC{}, QBC{});                                    \
        __builtin_amdgcn_s_setprio(0);                                  \
        PGMI_8P_SB();                                                   \
        __builtin_amdgcn_s_barrier();                                   \
    } while (0)
    // the half-tile the next phase reads was issued four half-tiles (three phases) before this wait
#define PGMI_8P_VMCNT() asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * GA) : "memory")

    // Phase p reads (buffer of its K-tile): 1: A0 B0, 2: B1, 3: A1, 4: none (A1 and the kept B0).
    // Wave row 1 runs one barrier behind wave row 0 (one extra s_barrier up front, matched by wave
    // row 0 after the loop), so on every SIMD one wave multiplies while its partner reads and
    // stages.  Under that stagger a read of phase p is retired only by the barrier closing phase
    // p + 1 for the leading row: a half is restaged two phases after its last read, in the order
    // A0 B0 B1 A1, one half per phase; it is read one phase after the vmcnt + barrier retiring it.
    // prologue: K-tile kt0 whole into buffer 0, kt0 + 1's A0 B0 into buffer 1
    stageA(0, kt0, 0);
    stageB(0, kt0, 0);
    stageB(1, kt0, 0);
    stageA(1, kt0, 0);
    stageA(0, kt0 + 1, 1);
    stageB(0, kt0 + 1, 1);
    PGMI_8P_VMCNT();
    __builtin_amdgcn_s_barrier();
    if (wm == 1) __builtin_amdgcn_s_barrier();
    for (int t = 0; t < nkt; t += 2) {
        const int T = kt0 + t;
        const bool has1 = t + 1 < nkt;
        // ---- K-tile T from buffer 0
        readA(0, 0); readB(I0{}, 0); PGMI_8P_SB(); stageB(1, T + 1, 1); PGMI_8P_VMCNT(); PGMI_8P_TAIL(I0, I0, true);
        readB(I1{}, 0); PGMI_8P_SB(); stageA(1, T + 1, 1); PGMI_8P_VMCNT();              PGMI_8P_TAIL(I0, I1, true);
        readA(1, 0); PGMI_8P_SB(); stageA(0, T + 2, 0);                                  PGMI_8P_TAIL(I1, I1, true);
        PGMI_8P_SB(); stageB(0, T + 2, 0); PGMI_8P_VMCNT();                              PGMI_8P_TAIL(I1, I0, true);
        // ---- K-tile T + 1 from buffer 1 (absent past an odd tile count: the phases keep their
        // barriers and stages, the MFMAs are skipped)
        readA(0, 1); readB(I0{}, 1); PGMI_8P_SB(); stageB(1, T + 2, 0); PGMI_8P_VMCNT(); PGMI_8P_TAIL(I0, I0, has1);
        readB(I1{}, 1); PGMI_8P_SB(); stageA(1, T + 2, 0); PGMI_8P_VMCNT();              PGMI_8P_TAIL(I0, I1, has1);
        readA(1, 1); PGMI_8P_SB(); stageA(0, T + 3, 1);                                  PGMI_8P_TAIL(I1, I1, has1);
        PGMI_8P_SB(); stageB(0, T + 3, 1); PGMI_8P_VMCNT();                              PGMI_8P_TAIL(I1, I0, has1);
    }
    if (wm == 0) __builtin_amdgcn_s_barrier();  // the lagging row's last barrier
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the clamped tail stages have landed
#undef PGMI_8P_TAIL
#undef PGMI_8P_VMCNT
#undef PGMI_8P_SB

    // ---- epilogue: acc[i][j] = rows m0 + wm*16*TM + 16 i, columns (qb = j / 2, jj = j % 2)
    const int mb = m0 + wm * 16 * TM;
    f32x4 a0[TM][2], a1[TM][2];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
            a0[i][jj] = acc[i][jj];
            a1[i][jj] = acc[i][2 + jj];
        }
    if constexpr (SPLIT) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int n = n0 + wn * 64 + j * 16 + (lane & 15);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int m = mb + i * 16 + (lane >> 4) * 4 + r;
                    if (m < M && n < N) ws[((long)z * M + m) * N + n] = acc[i][j][r];
                }
            }
    } else if constexpr (DUAL) {
        epi_tile<EPI, TM, 2>(ea, M, N, mb, n0 + wn * 32, lane, a0, a1);
    } else {
        epi_tile<EPI, TM, 2>(ea, M, N, mb, n0 + wn * 64, lane, a0, a0);
        epi_tile<EPI, TM, 2>(ea, M, N, mb, n0 + wn * 64 + 32, lane, a1, a1);
    }
}

// (PGMI_GEMM_KERNELS_ONLY: the kernel templates alone, for single-instantiation ISA / register checks)
#ifndef PGMI_GEMM_KERNELS_ONLY
// Tile configurations (wave grid, per-wave MFMA tiles).  BM = WGM*TM*16, BN = WGN*TN*16.
enum Cfg : int {
    C288x64 = 0,   // 6x1 waves, 3x4 tiles  (text rows: M = 288 = 18 x 16)
    C288x32 = 1,   // 6x1 waves, 3x2 tiles
    C256x64 = 2,   // 4x1 waves, 4x4 tiles  (vision rows: M = 256)
    C256x32 = 3,   // 4x1 waves, 4x2 tiles
    C128x128 = 4,  // 2x2 waves, 4x4 tiles  (large M)
    C128x64 = 5,   // 2x2 waves, 4x2 tiles
    // panel GEMM (k_gemm_p, LDS-DMA ring): BM x BN output columns (dual gate/up: BN/2 columns x 2)
    P288w = 6,     // TM 9,  BN 128, 3 slots
    P256w = 7,     // TM 8,  BN 128, 3 slots
    P352w = 8,     // TM 11, BN 128, 2 slots  (448 px text rows: M = 1056 = 3 x 352)
    P288n = 9,     // TM 9,  BN 64,  3 slots
    P256n = 10,    // TM 8,  BN 64,  3 slots
    P128w = 11,    // TM 4,  BN 128, 3 slots
    P288t = 12,    // TM 9,  BN 32,  4 slots  (2x2 waves, 1 column fragment each)
    P256t = 13,    // 4x1 waves, TM 4, BN 32, 4 slots
    P64x64 = 14,   // TM 2, BN 64,  6 slots   (small GEMMs: every CU busy, little A per CU)
    P128x64 = 15,  // TM 4, BN 64,  6 slots
    P64x128 = 16,  // TM 2, BN 128, 6 slots
    P128x128 = 17, // TM 4, BN 128, 5 slots
    P64x64d = 18,  // TM 2, BN 64,  10 slots
    P128x64d = 19, // 4x1 waves, TM 2, BN 64, 6 slots
    // 8 waves (2 per SIMD: one wave's LDS-DMA issue stalls overlap its partner's MFMAs)
    Q288w = 20,    // 2x4 waves, TM 9,  BN 128, 3 slots
    Q352w = 21,    // 2x4 waves, TM 11, BN 128, 2 slots
    Q256w = 22,    // 2x4 waves, TM 8,  BN 128, 3 slots
    Q288x256 = 23, // 2x4 waves, TM 9,  BN 256, 2 slots
    // shallow rings (2-3 workgroups per CU: more k-tiles in flight per CU for the small GEMMs)
    P64x64s3 = 24, // TM 2, BN 64, 3 slots
    P64x64s4 = 25, // TM 2, BN 64, 4 slots
    P32x64s4 = 26, // TM 1, BN 64, 4 slots
    P64x32s4 = 27, // TM 2, BN 32, 4 slots
    P96x64s4 = 28, // TM 3, BN 64, 4 slots (M = 288 = 3 x 96)
    P96x64s3 = 29, // TM 3, BN 64, 3 slots
    // warp-specialised (k_gemm_w): compute waves + 4 LDS-DMA loader waves
    W288w = 30,    // 2x4 compute waves, TM 9,  BN 128, 3 slots
    W288n = 31,    // 2x4 compute waves, TM 9,  BN 64,  3 slots
    W64x64 = 32,   // 2x2 compute waves, TM 2,  BN 64,  6 slots
    W352w = 33,    // 2x4 compute waves, TM 11, BN 128, 2 slots
    W128x128 = 34, // 2x4 compute waves, TM 4,  BN 128, 4 slots
    W128x64 = 35,  // 2x2 compute waves, TM 4,  BN 64,  5 slots
    // 8-phase (k_gemm_8p): 2x4 waves, BN 256 (dual: 128 gate + 128 up), two K-tile buffers
    E256 = 36,     // TM 8: 256 rows
    E192 = 37,     // TM 6: 192 rows
    // round 6: k_gemm_w's in-wave reload mode (W288w's tiles; bit-identical results)
    R288w = 38,    // 2x4 compute waves, TM 9, BN 128 (dual 64 + 64), 3 slots
    kNumCfg = 39,
};
static_assert(kNumCfg == kGemmCfgs, "launch.h kGemmCfgs");

struct Plan {
    Cfg cfg;
    int bm, bn, split;
};

static int g_force_cfg = -1, g_force_split = 0;  // tuning override (pgmi_tune_gemm)

void gemm_force_plan(int cfg, int split) {
    g_force_cfg = cfg;
    g_force_split = split;
}

// per-shape plan overrides (tuning hook pgmi_tune_gemm_shape): in-situ sweeps of one GEMM of a
// forward while the others keep their measured plans
struct ShapePlan {
    int M, N, K;
    bool dual;
    int cfg, split;
};
static ShapePlan g_shape_plans[16];
static int g_n_shape_plans = 0;

int gemm_force_shape(int M, int N, int K, int dual, int cfg, int split) {
    for (int i = 0; i < g_n_shape_plans; ++i)
        if (g_shape_plans[i].M == M && g_shape_plans[i].N == N && g_shape_plans[i].K == K &&
            g_shape_plans[i].dual == (dual != 0)) {
            g_shape_plans[i] = g_shape_plans[--g_n_shape_plans];
            break;
        }
    if (cfg < 0) return 0;
    if (g_n_shape_plans >= 16) return -1;
    g_shape_plans[g_n_shape_plans++] = {M, N, K, dual != 0, cfg, split < 1 ? 1 : split};
    return 0;
}

static Plan choose(int M, int N, int K, bool dual) {
    if (g_force_cfg >= 0) {
        static const int bms[] = {288, 288, 256, 256, 128, 128, 288, 256, 352, 288, 256, 128, 288, 256, 64, 128, 64, 128, 64, 128, 288, 352, 256, 288, 64, 64, 32, 64, 96, 96, 288, 288, 64, 352, 128, 128, 256, 192, 288};
        static const int bns[] = {64, 32, 64, 32, 128, 64, 128, 128, 128, 64, 64, 128, 32, 32, 64, 64, 128, 128, 64, 64, 128, 128, 128, 256, 64, 64, 64, 32, 64, 64, 128, 64, 64, 128, 128, 64, 256, 256, 128};
        const int c = g_force_cfg;
        const int bn = (dual && c >= P288w) ? bns[c] / 2 : bns[c];
        return {(Cfg)c, bms[c], bn, dual && c < P288w ? 1 : (g_force_split > 0 ? g_force_split : 1)};
    }
    // Measured on MI355X (tools/gemm_sweep.py; GPU time of graph-replayed calls, round 1): the
    // PaliGemma prefill shapes at 224 px (M = 256 vision / 288 text rows) and 448 px (1024 /
    // 1056 rows).  Small GEMMs want every CU busy with little A per CU (64 x 64 tiles, 6-slot
    // ring, no split: the epilogue stays in the GEMM); the dual gate/up and K = 16384 down
    // projections want full-M panels that read each weight byte once.
    struct Entry { int M, N, K; bool dual; Cfg cfg; int split; };
    static const Entry table[] = {
        // round 2: tools/gemm_sweep.py --cold (every call reads its weights from HBM, as the layer
        // loop does); W* = warp-specialised (k_gemm_w), P*s* = shallow rings
        {288, 2560, 2048, false, W64x64, 1},    // text q|k|v            10.8 us
        // text rows, round 3 in situ (tools/probes/plan_sweep.py --target lm: the generate loop's whole
        // language-model prefill timed per candidate, split partials reduced by the residual + RMSNorm)
        {288, 2048, 2048, false, W128x128, 4},  // text o_proj           LM -45 us vs W64x64 unsplit
        {288, 16384, 2048, true, R288w, 1},     // text gate|up (GeGLU)  LM -27 us vs W288w (round 3, W288n); round 6:
                                                // the in-wave reload form of the same tiles, bit-identical, isolated
                                                // 47.2 -> 40.5 us (cold), in situ -7 us per LM prefill (gpurun_out r6i)
        {288, 2048, 16384, false, W288n, 8},    // text down             round 6 in situ: LM -26 / -50 us vs W128x128
                                                // split 4 on two boxes (gpurun_out r6b / r6e; round 3 had the opposite)
        // vision rows: round 3, in situ (tools/probes/plan_sweep.py: the whole tower timed per
        // candidate; split-K partials of out_proj / fc2 are reduced by the residual + LayerNorm kernel)
        {256, 3456, 1152, false, P64x64s4, 1},  // vision q|k|v          tower -17 us vs W64x64
        {256, 1152, 1152, false, P64x64s4, 3},  // vision out_proj       tower -38 us vs P32x64s4 unsplit
        {256, 4304, 1152, false, P96x64s4, 1},  // vision fc1 (+GELU)    11.0 us (exp/rcp GELU; was 16.4)
        {256, 1152, 4304, false, P96x64s4, 4},  // vision fc2            tower -19 us vs P64x64s4 split 3
        {256, 1152, 640, false, P64x32s4, 1},   // patch embedding        5.3 us (was 6.6 on P64x64)
        {256, 2048, 1152, false, P32x64s4, 1},  // multimodal projector   7.6 us
        {1056, 2560, 2048, false, W128x128, 1}, // 448 px text q|k|v     21.3 us (P96x64s3 24.0 in the same sweep)
        {1056, 2048, 2048, false, W128x128, 1}, // 448 px text o_proj    19.5 us (P96x64s3 23.9)
        {1056, 16384, 2048, true, E192, 1},     // 448 px gate|up       135.5 us (W352w 149.8); in situ LM 5688 -> 5538 us
        {1056, 2048, 16384, false, E192, 5},    // 448 px down          (W288w split 4 79.1 us); in situ 5688 -> 5539 us;
                                                // round 4 in situ (profiles/r04_plan_sweeps.txt): split 5 (240 WGs) 5294 -> 5271 us
        {1024, 3456, 1152, false, W128x128, 1}, // 448 px vision q|k|v   18.3 us (was 24.6)
        {1024, 1152, 1152, false, P96x64s4, 1}, // 448 px vision out     10.6 us (P32x64s4 13.7)
        {1024, 4304, 1152, false, W288w, 1},    // 448 px vision fc1     25.1 us (exp/rcp GELU; was 29.5)
        {1024, 1152, 4304, false, W128x128, 3}, // 448 px vision fc2     in situ tower 2965 -> 2904 us vs W288w split 4
        // configs[3]: 8 images per GPU as one batch (vision 2048 rows, text 2304 rows), cold sweep
        {2048, 3456, 1152, false, W288w, 1},    // vision q|k|v          31.2 us (was 46.8)
        {2048, 1152, 1152, false, W128x128, 1}, // vision out_proj       22.3 us (was 31.6)
        {2048, 4304, 1152, false, W352w, 1},    // vision fc1            48.6 us (was 91.5)
        {2048, 1152, 4304, false, W288w, 2},    // vision fc2            47.3 us (was 72.2)
        {2048, 2048, 1152, false, W128x128, 1}, // projector             19.1 us (was 23.8)
        {2304, 2560, 2048, false, Q256w, 1},    // text q|k|v            in situ LM 9047 -> 8902 us vs W288w + RoPE
                                                // epilogue (61 us in situ: 160 workgroups); RoPE by k_rope_kv
        {2304, 2048, 2048, false, W288n, 1},    // text o_proj           35.4 us (was 62.1)
        {2304, 16384, 2048, true, E256, 1},     // text gate|up         261.8 us (W288w 301.8); in situ LM 10064 -> 9435 us
        {2304, 2048, 16384, false, W288w, 2},   // text down            153.9 us (was 298.6)
    };
    static const int bms[] = {288, 288, 256, 256, 128, 128, 288, 256, 352, 288, 256, 128, 288, 256, 64, 128, 64, 128, 64, 128, 288, 352, 256, 288, 64, 64, 32, 64, 96, 96, 288, 288, 64, 352, 128, 128, 256, 192, 288};
    static const int bns[] = {64, 32, 64, 32, 128, 64, 128, 128, 128, 64, 64, 128, 32, 32, 64, 64, 128, 128, 64, 64, 128, 128, 128, 256, 64, 64, 64, 32, 64, 64, 128, 64, 64, 128, 128, 64, 256, 256, 128};
    auto mk = [&](Cfg c, int split) -> Plan { return {c, bms[c], dual ? bns[c] / 2 : bns[c], dual ? 1 : split}; };
    for (int i = 0; i < g_n_shape_plans; ++i) {
        const ShapePlan& o = g_shape_plans[i];
        if (o.M == M && o.N == N && o.K == K && o.dual == dual) return mk((Cfg)o.cfg, o.split);
    }
    for (const Entry& e : table)
        if (e.M == M && e.N == N && e.K == K && e.dual == dual) return mk(e.cfg, e.split);
    // lock-step decode batches as GEMMs (M <= 16 rows; tools/gemm_sweep.py b8_*
    // in isolation: gate|up 64x128 tiles 24.2 us, down 64x64 split 8 18.1 us)
    if (M <= 16) {
        if (dual) return mk(P64x128, 1);
        if (K >= 8192) return mk(P64x64, 8);
    }
    // other shapes (batched prefill: M = B x 256 / 288 rows; other image sizes)
    if (dual) return mk(M <= 288 || M >= 2048 ? W288w : W352w, 1);
    if (K >= 8192) return mk(M <= 288 ? W288n : W288w, M <= 288 ? 8 : M <= 1056 ? 4 : 2);
    const long t64 = (long)((M + 63) / 64) * ((N + 63) / 64);
    if (t64 <= 256) return mk(P64x64, 1);
    const long t128 = (long)((M + 127) / 128) * ((N + 127) / 128);
    Plan p = mk(P128w, 1);
    const int nkt = (K + 63) / 64;
    while (t128 * p.split < 200 && p.split < 4 && nkt / (p.split * 2) >= 4) p.split *= 2;
    return p;
}

size_t gemm_ws_bytes(int M, int N, int K) {
    Plan p = choose(M, N, K, false);
    return p.split > 1 ? (size_t)p.split * M * N * sizeof(float) : 0;
}

// host: the XCD block shape for xcd_tile's `code` argument, or 0 for the run order -- used only when
// it cuts the bytes the 8 XCDs must fetch into their L2s by at least 20 %.  Memoised per launch shape
// behind a mutex (contexts may be driven from several host threads).
static int xcd_block_pick(int n_mt, int n_nt, int S, int BM, int BN, int K);
static int xcd_block(int n_mt, int n_nt, int S, int BM, int BN, int K) {
    static std::mutex mu;
    static std::map<std::tuple<int, int, int, int, int, int>, int> memo;
    const auto key = std::make_tuple(n_mt, n_nt, S, BM, BN, K);
    std::lock_guard<std::mutex> lock(mu);
    auto it = memo.find(key);
    if (it != memo.end()) return it->second;
    const int code = xcd_block_pick(n_mt, n_nt, S, BM, BN, K);
    memo[key] = code;
    return code;
}

static int xcd_block_pick(int n_mt, int n_nt, int S, int BM, int BN, int K) {
    const long G = (long)n_mt * n_nt * S;
    // measured (same box, tools/archive/gpu_r4c.sh): 8-image prefill 12.88 -> 12.59 ms, 448 px flat, but the
    // 224 px tower 1.46 -> 1.53 ms (its split-K fc2 picked a block order that reads fewer bytes and
    // runs slower): the block order is used for the batched prefills' activation panels (>= 2048 rows)
    if ((long)n_mt * BM < 2048) return 0;
    if (G % 8 != 0 || n_mt >= 64 * 8 || G > 65536) return 0;
    const double ks = (double)K / S * 2.0;  // bytes per row of one K slice
    // the run order: XCD x reads the (mt, z) row panels and (nt, z) weight panels of its run
    const long q = G / 8;
    double run = 0.0;
    for (int x = 0; x < 8; ++x) {
        long na = 0, nb = 0;
        std::vector<char> sa((size_t)n_mt * S, 0), sb((size_t)n_nt * S, 0);
        for (long idx = x * q; idx < (x + 1) * q; ++idx) {
            const int mt = (int)(idx % n_mt), z = (int)((idx / n_mt) % S), nt = (int)(idx / ((long)n_mt * S));
            if (!sa[(size_t)mt * S + z]++) ++na;
            if (!sb[(size_t)nt * S + z]++) ++nb;
        }
        run += ks * ((double)na * BM + (double)nb * BN);
    }
    double best = 0.8 * run;
    int code = 0;
    for (int bm = 1; bm <= n_mt && bm < 64; ++bm) {
        if (n_mt % bm) continue;
        for (int bn = 1; bn <= n_nt && bn < 256; ++bn) {
            if (n_nt % bn) continue;
            for (int bs = 1; bs <= S && bs < 16; ++bs) {
                if (S % bs || (n_mt / bm) * (n_nt / bn) * (S / bs) != 8) continue;
                const double bytes = 8.0 * bs * ks * ((double)bm * BM + (double)bn * BN);
                if (bytes < best) { best = bytes; code = bm | (bn << 6) | (bs << 14); }
            }
        }
    }
    return code;
}

// in-situ timing probe (pgmi_prefill_probe): when a pair of events is armed, the next GEMM kernel is
// launched with hipExtLaunchKernelGGL, whose events take that kernel's own start and end -- a time
// free of the host's launch pace and of the stream's other packets; the pair is used once.  Per host
// thread: the engine arms the pair right before the GEMM call that takes it, on the same thread.
static thread_local hipEvent_t g_probe_ev0 = nullptr, g_probe_ev1 = nullptr;
void gemm_probe_events(hipEvent_t start, hipEvent_t stop) {
    g_probe_ev0 = start;
    g_probe_ev1 = stop;
}
#define PGMI_GEMM_LAUNCH(KERN, GRID, BLOCK, LDS, S, ...)                                                  \
    do {                                                                                                \
        if (g_probe_ev0) {                                                                              \
            hipExtLaunchKernelGGL(KERN, GRID, BLOCK, LDS, S, g_probe_ev0, g_probe_ev1, 0, __VA_ARGS__); \
            g_probe_ev0 = g_probe_ev1 = nullptr;                                                        \
        } else {                                                                                        \
            hipLaunchKernelGGL(KERN, GRID, BLOCK, LDS, S, __VA_ARGS__);                                 \
        }                                                                                               \
    } while (0)

template <int WGM, int WGN, int TM, int TN, int EPI>
static void launch_t(hipStream_t s, const uint16_t* A, int lda, const uint16_t* W, int ldw, int M, int N, int K,
                     const EpiArgs& ea, float* ws, int split, long up_off) {
    constexpr int NB = (EPI == EPI_GEGLU) ? 2 : 1;  // EPI < 0: partials only
    constexpr int BM = WGM * TM * 16, BN = WGN * TN * 16, NT = 64 * WGM * WGN;
    const size_t lds = (size_t)(2 * BM * LDSK + 2 * NB * BN * LDSK) * sizeof(uint16_t);
    const int nkt = (K + BK - 1) / BK;
    const int per = (nkt + split - 1) / split;
    dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM, split);
    static bool attr_set = false;
    if (!attr_set) {
        if constexpr (EPI >= 0)
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm<WGM, WGN, TM, TN, EPI, false>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm<WGM, WGN, TM, TN, EPI_STORE, true>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr_set = true;
    }
    if constexpr (EPI < 0) {
        PGMI_GEMM_LAUNCH((k_gemm<WGM, WGN, TM, TN, EPI_STORE, true>), grid, dim3(NT), lds, s, A, lda, W, ldw, M, N,
                           K, per, ea, ws, up_off);
        return;
    } else if (split == 1) {
        PGMI_GEMM_LAUNCH((k_gemm<WGM, WGN, TM, TN, EPI, false>), grid, dim3(NT), lds, s, A, lda, W, ldw, M, N, K,
                           per, ea, ws, up_off);
    } else {
        PGMI_GEMM_LAUNCH((k_gemm<WGM, WGN, TM, TN, EPI_STORE, true>), grid, dim3(NT), lds, s, A, lda, W, ldw, M, N,
                           K, per, ea, ws, up_off);
        long total4 = ((long)M * N + 3) / 4;
        long blocks = (total4 + 255) / 256;
        if (blocks > 4096) blocks = 4096;
        hipLaunchKernelGGL((k_splitk_epi<EPI>), dim3((unsigned)blocks), dim3(256), 0, s, ws, split, M, N, ea);
    }
}

#undef PGMI_LDS_AT

// panel GEMM launcher: WM x (4/WM) waves, TNW = 16-column fragments per wave (per B operand
// for plain GEMMs; the dual GEMM splits them over gate and up); EPI < 0: partials only
template <int NW, int WM, int TM, int TNW, int ST, int EPI>
static void launch_p(hipStream_t s, const uint16_t* A, int lda, const uint16_t* W, int ldw, int M, int N, int K,
                     const EpiArgs& ea, float* ws, int split, long up_off) {
    constexpr bool DUAL = (EPI == EPI_GEGLU);
    constexpr int NB = DUAL ? 2 : 1;
    constexpr int TN = DUAL ? (TNW >= 2 ? TNW / 2 : 1) : TNW;  // the dual GEMM keeps the B rows per slot
    constexpr int BM = WM * TM * 16, BN = (NW / WM) * TN * 16;
    constexpr int STQ = (size_t)ST * (BM + NB * BN) * 128 <= 163840 ? ST : ST - 1;  // fit 160 KiB
    constexpr size_t lds = (size_t)STQ * (BM + NB * BN) * 128;
    static_assert(lds <= 163840, "LDS ring exceeds 160 KiB");
    constexpr int EK = EPI < 0 ? EPI_STORE : EPI;
    const int nkt = (K + 63) / 64;
    const int per = (nkt + split - 1) / split;
    const int n_mt = (M + BM - 1) / BM, n_nt = (N + BN - 1) / BN;
    dim3 grid(n_mt * n_nt, split);
    const int code = xcd_block(n_mt, n_nt, split, BM, NB * BN, K);
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm_p<NW, WM, TM, TN, NB, STQ, EK, false>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm_p<NW, WM, TM, TN, NB, STQ, EK, true>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr_set = true;
    }
    if (EPI < 0 || split > 1) {
        PGMI_GEMM_LAUNCH((k_gemm_p<NW, WM, TM, TN, NB, STQ, EK, true>), grid, dim3(64 * NW), lds, s, A, lda, W, ldw, M, N, K, per,
                           ea, ws, up_off, n_mt, code);
        if (EPI >= 0) {
            long total4 = ((long)M * N + 3) / 4;
            long blocks = (total4 + 255) / 256;
            if (blocks > 4096) blocks = 4096;
            hipLaunchKernelGGL((k_splitk_epi<EK>), dim3((unsigned)blocks), dim3(256), 0, s, ws, split, M, N, ea);
        }
    } else {
        PGMI_GEMM_LAUNCH((k_gemm_p<NW, WM, TM, TN, NB, STQ, EK, false>), grid, dim3(64 * NW), lds, s, A, lda, W, ldw, M, N, K,
                           per, ea, ws, up_off, n_mt, code);
    }
}

// warp-specialised launcher: as launch_p, NW compute waves (grid WM x NW/WM) + LW loader waves (RL: in-wave reload)
template <int NW, int WM, int TM, int TNW, int ST, int LW, int EPI, bool RL = false>
static void launch_w(hipStream_t s, const uint16_t* A, int lda, const uint16_t* W, int ldw, int M, int N, int K,
                     const EpiArgs& ea, float* ws, int split, long up_off) {
    constexpr bool DUAL = (EPI == EPI_GEGLU);
    constexpr int NB = DUAL ? 2 : 1;
    constexpr int TN = DUAL ? (TNW >= 2 ? TNW / 2 : 1) : TNW;
    constexpr int BM = WM * TM * 16, BN = (NW / WM) * TN * 16;
    constexpr size_t lds = (size_t)ST * (BM + NB * BN) * 128;
    static_assert(lds <= 163840, "LDS ring exceeds 160 KiB");
    constexpr int EK = EPI < 0 ? EPI_STORE : EPI;
    const int nkt = (K + 63) / 64;
    const int per = (nkt + split - 1) / split;
    const int n_mt = (M + BM - 1) / BM, n_nt = (N + BN - 1) / BN;
    dim3 grid(n_mt * n_nt, split);
    const int code = xcd_block(n_mt, n_nt, split, BM, NB * BN, K) | (n_mt == 1 ? 1 << 30 : 0);
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm_w<NW, WM, TM, TN, NB, ST, LW, EK, false, RL>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm_w<NW, WM, TM, TN, NB, ST, LW, EK, true, RL>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr_set = true;
    }
    const dim3 block(64 * (NW + LW));
    if (EPI < 0 || split > 1) {
        PGMI_GEMM_LAUNCH((k_gemm_w<NW, WM, TM, TN, NB, ST, LW, EK, true, RL>), grid, block, lds, s, A, lda, W, ldw, M, N, K,
                           per, ea, ws, up_off, n_mt, code);
        if (EPI >= 0) {
            long total4 = ((long)M * N + 3) / 4;
            long blocks = (total4 + 255) / 256;
            if (blocks > 4096) blocks = 4096;
            hipLaunchKernelGGL((k_splitk_epi<EK>), dim3((unsigned)blocks), dim3(256), 0, s, ws, split, M, N, ea);
        }
    } else {
        PGMI_GEMM_LAUNCH((k_gemm_w<NW, WM, TM, TN, NB, ST, LW, EK, false, RL>), grid, block, lds, s, A, lda, W, ldw, M, N, K,
                           per, ea, ws, up_off, n_mt, code);
    }
}

// 8-phase launcher (K % 64 == 0); EPI < 0: partials only
template <int TM, int EPI>
static void launch_8p(hipStream_t s, const uint16_t* A, int lda, const uint16_t* W, int ldw, int M, int N, int K,
                      const EpiArgs& ea, float* ws, int split, long up_off) {
    constexpr bool DUAL = (EPI == EPI_GEGLU);
    constexpr int BM = 32 * TM, BNO = DUAL ? 128 : 256;
    constexpr size_t lds = (size_t)2 * (2 * 16 * TM * 128 + 2 * 128 * 128);
    static_assert(lds <= 163840, "LDS exceeds 160 KiB");
    constexpr int EK = EPI < 0 ? EPI_STORE : EPI;
    const int nkt = K / 64;
    const int per = (nkt + split - 1) / split;
    const int n_mt = (M + BM - 1) / BM, n_nt = (N + BNO - 1) / BNO;
    dim3 grid(n_mt * n_nt, split);
    const int code = xcd_block(n_mt, n_nt, split, BM, DUAL ? 2 * BNO : BNO, K);
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm_8p<TM, EK, false>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm_8p<TM, EK, true>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr_set = true;
    }
    if (EPI < 0 || split > 1) {
        PGMI_GEMM_LAUNCH((k_gemm_8p<TM, EK, true>), grid, dim3(512), lds, s, A, lda, W, ldw, M, N, K, per, ea, ws,
                           up_off, n_mt, code);
        if (EPI >= 0) {
            long total4 = ((long)M * N + 3) / 4;
            long blocks = (total4 + 255) / 256;
            if (blocks > 4096) blocks = 4096;
            hipLaunchKernelGGL((k_splitk_epi<EK>), dim3((unsigned)blocks), dim3(256), 0, s, ws, split, M, N, ea);
        }
    } else {
        PGMI_GEMM_LAUNCH((k_gemm_8p<TM, EK, false>), grid, dim3(512), lds, s, A, lda, W, ldw, M, N, K, per, ea, ws,
                           up_off, n_mt, code);
    }
}

template <int EPI>
static void launch_pcfg(hipStream_t s, const uint16_t* A, int lda, const uint16_t* W, int ldw, int M, int N, int K,
                        const EpiArgs& ea, float* ws, const Plan& p, long up_off) {
#define P_(wm, tm, tn, st) launch_p<4, wm, tm, tn, st, EPI>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off)
#define P8_(wm, tm, tn, st) launch_p<8, wm, tm, tn, st, EPI>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off)
    switch (p.cfg) {
        case P288w: P_(2, 9, 4, 3); break;
        case P256w: P_(2, 8, 4, 3); break;
        case P352w: P_(2, 11, 4, 2); break;
        case P288n: P_(2, 9, 2, 3); break;
        case P256n: P_(2, 8, 2, 4); break;
        case P128w: P_(2, 4, 4, 3); break;
        case P288t: P_(2, 9, 1, 4); break;
        case P256t: P_(4, 4, 2, 4); break;
        case P64x64: P_(2, 2, 2, 6); break;
        case P128x64: P_(2, 4, 2, 6); break;
        case P64x128: P_(2, 2, 4, 6); break;
        case P128x128: P_(2, 4, 4, 5); break;
        case P64x64d: P_(2, 2, 2, 10); break;
        case P128x64d: P_(4, 2, 4, 6); break;
        case Q288w: P8_(2, 9, 2, 3); break;
        case Q352w: P8_(2, 11, 2, 2); break;
        case Q256w: P8_(2, 8, 2, 3); break;
        case Q288x256: P8_(2, 9, 4, 2); break;
        case P64x64s3: P_(2, 2, 2, 3); break;
        case P64x64s4: P_(2, 2, 2, 4); break;
        case P32x64s4: P_(2, 1, 2, 4); break;
        case P64x32s4: P_(2, 2, 1, 4); break;
        case P96x64s4: P_(2, 3, 2, 4); break;
        case P96x64s3: P_(2, 3, 2, 3); break;
        case W288w: launch_w<8, 2, 9, 2, 3, 4, EPI>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off); break;
        case W288n: launch_w<8, 2, 9, 1, 3, 4, EPI>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off); break;
        case W64x64: launch_w<4, 2, 2, 2, 6, 4, EPI>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off); break;
        case W352w: launch_w<8, 2, 11, 2, 2, 4, EPI>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off); break;
        case W128x128: launch_w<8, 2, 4, 2, 4, 4, EPI>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off); break;
        case W128x64: launch_w<4, 2, 4, 2, 5, 4, EPI>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off); break;
        case E256: launch_8p<8, EPI>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off); break;
        case E192: launch_8p<6, EPI>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off); break;
        case R288w: launch_w<8, 2, 9, 2, 3, 4, EPI, true>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off); break;
        default: break;
    }
#undef P_
#undef P8_
}

template <int EPI>
static void launch_e(hipStream_t s, const uint16_t* A, int lda, const uint16_t* W, int ldw, int M, int N, int K,
                     const EpiArgs& ea, float* ws, const Plan& p, long up_off) {
    switch (p.cfg) {
        case C288x64: launch_t<6, 1, 3, 4, EPI>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off); break;
        case C288x32: launch_t<6, 1, 3, 2, EPI>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off); break;
        case C256x64: launch_t<4, 1, 4, 4, EPI>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off); break;
        case C256x32: launch_t<4, 1, 4, 2, EPI>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off); break;
        case C128x128: launch_t<2, 2, 4, 4, EPI>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off); break;
        case C128x64: launch_t<2, 2, 4, 2, EPI>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off); break;
        default: launch_pcfg<EPI>(s, A, lda, W, ldw, M, N, K, ea, ws, p, up_off); break;
    }
}

int gemm(hipStream_t s, const uint16_t* A, int lda, const uint16_t* W, int ldw, int M, int N, int K, Epi epi,
         const EpiArgs& ea, float* ws, size_t ws_bytes, int up_offset_rows, bool defer) {
    Plan p = choose(M, N, K, epi == EPI_GEGLU);
    if ((p.cfg == E256 || p.cfg == E192) && K % 64 != 0) p.cfg = P128w;  // the 8-phase kernel has no K tail
    if (p.split > 1 && (size_t)p.split * M * N * sizeof(float) > ws_bytes) p.split = 1;
    if (p.split > 1 && N % 4 != 0) p.split = 1;  // the split-K epilogue works on 4 outputs per thread
    const long up_off = (long)up_offset_rows * ldw;
    if (defer && p.split > 16) p.split = 16;  // the consumers (splitk_res_norm, rope_kv) reduce at most 16 slabs
    if (p.split > 1) {
        // every K range non-empty (a forced split can exceed what K allows: the 8-phase kernel
        // leaves an empty range's partial slab unwritten, and any empty range is wasted work);
        // the consumers reduce the split returned here
        const int nkt = (K + BK - 1) / BK;
        const int per = (nkt + p.split - 1) / p.split;
        p.split = (nkt + per - 1) / per;
    }
    if (defer && p.split > 1) {
        // partial slabs only: the consumer kernel (splitk_res_norm / rope_kv_append) reduces them
        switch (p.cfg) {
            case C288x64: launch_t<6, 1, 3, 4, -1>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off); break;
            case C288x32: launch_t<6, 1, 3, 2, -1>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off); break;
            case C256x64: launch_t<4, 1, 4, 4, -1>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off); break;
            case C256x32: launch_t<4, 1, 4, 2, -1>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off); break;
            case C128x128: launch_t<2, 2, 4, 4, -1>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off); break;
            case C128x64: launch_t<2, 2, 4, 2, -1>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off); break;
            default: launch_pcfg<-1>(s, A, lda, W, ldw, M, N, K, ea, ws, p, up_off); break;
        }
        return p.split;
    }
    switch (epi) {
        case EPI_STORE: launch_e<EPI_STORE>(s, A, lda, W, ldw, M, N, K, ea, ws, p, up_off); break;
        case EPI_BIAS: launch_e<EPI_BIAS>(s, A, lda, W, ldw, M, N, K, ea, ws, p, up_off); break;
        case EPI_BIAS_GELU: launch_e<EPI_BIAS_GELU>(s, A, lda, W, ldw, M, N, K, ea, ws, p, up_off); break;
        case EPI_BIAS_RES: launch_e<EPI_BIAS_RES>(s, A, lda, W, ldw, M, N, K, ea, ws, p, up_off); break;
        case EPI_RES: launch_e<EPI_RES>(s, A, lda, W, ldw, M, N, K, ea, ws, p, up_off); break;
        case EPI_BIAS_POS: launch_e<EPI_BIAS_POS>(s, A, lda, W, ldw, M, N, K, ea, ws, p, up_off); break;
        case EPI_F32: launch_e<EPI_F32>(s, A, lda, W, ldw, M, N, K, ea, ws, p, up_off); break;
        case EPI_GEGLU: launch_e<EPI_GEGLU>(s, A, lda, W, ldw, M, N, K, ea, ws, p, up_off); break;
        case EPI_ROPE: return 0;  // gemm_qkv_rope only
    }
    return 1;
}

bool gemm_qkv_rope(hipStream_t s, const uint16_t* A, int lda, const uint16_t* W, int ldw, int M, int N, int K,
                   const EpiArgs& ea) {
    if (N % 256 != 0 || N != (ea.nh + 2 * ea.nkv) * 256) return false;
    const Plan p = choose(M, N, K, false);
    if (p.split != 1) return false;
    // configurations with two 16-column tiles per wave and a tile width dividing 256
#define P_(wm, tm, st) launch_p<4, wm, tm, 2, st, EPI_ROPE>(s, A, lda, W, ldw, M, N, K, ea, nullptr, 1, 0)
#define W_(nw, tm, st) launch_w<nw, 2, tm, 2, st, 4, EPI_ROPE>(s, A, lda, W, ldw, M, N, K, ea, nullptr, 1, 0)
    switch (p.cfg) {
        case P288n: P_(2, 9, 3); break;
        case P64x64: P_(2, 2, 6); break;
        case P128x64: P_(2, 4, 6); break;
        case P64x64s3: P_(2, 2, 3); break;
        case P64x64s4: P_(2, 2, 4); break;
        case P32x64s4: P_(2, 1, 4); break;
        case P96x64s4: P_(2, 3, 4); break;
        case P96x64s3: P_(2, 3, 3); break;
        case W288w: W_(8, 9, 3); break;
        case W64x64: W_(4, 2, 6); break;
        case W352w: W_(8, 11, 2); break;
        case W128x128: W_(8, 4, 4); break;
        case W128x64: launch_w<4, 2, 4, 2, 5, 4, EPI_ROPE>(s, A, lda, W, ldw, M, N, K, ea, nullptr, 1, 0); break;
        default: return false;
    }
#undef P_
#undef W_
    return true;
}

// host replica of a launch's tile order (pgmi_debug_gemm_tiles: the CPU test that every workgroup of the
// grid gets a distinct (row tile, column tile, K slice)); returns the XCD block code the launch would use
int gemm_tile_order(int n_mt, int n_nt, int S, int BM, int BN, int K, int* mt, int* nt, int* z) {
    const int code = xcd_block(n_mt, n_nt, S, BM, BN, K);
    const int gx = n_mt * n_nt;
    for (int lin = 0; lin < gx * S; ++lin) xcd_tile_of(lin, gx, S, n_mt, code, mt[lin], nt[lin], z[lin]);
    return code;
}

#endif  // PGMI_GEMM_KERNELS_ONLY

}  // namespace pgmi
