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
#include "common.h"
#include "launch.h"

namespace pgmi {

constexpr int BK = 64;
constexpr int LDSK = 72;  // padded row (elements)

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

// Tile configurations (wave grid, per-wave MFMA tiles).  BM = WGM*TM*16, BN = WGN*TN*16.
enum Cfg : int {
    C288x64 = 0,   // 6x1 waves, 3x4 tiles  (text rows: M = 288 = 18 x 16)
    C288x32 = 1,   // 6x1 waves, 3x2 tiles
    C256x64 = 2,   // 4x1 waves, 4x4 tiles  (vision rows: M = 256)
    C256x32 = 3,   // 4x1 waves, 4x2 tiles
    C128x128 = 4,  // 2x2 waves, 4x4 tiles  (large M)
    C128x64 = 5,   // 2x2 waves, 4x2 tiles
};

struct Plan {
    Cfg cfg;
    int bm, bn, split;
};

static int g_force_cfg = -1, g_force_split = 0;  // tuning override (pgmi_tune_gemm)

void gemm_force_plan(int cfg, int split) {
    g_force_cfg = cfg;
    g_force_split = split;
}

static Plan choose(int M, int N, int K, bool dual) {
    if (g_force_cfg >= 0) {
        static const int bms[] = {288, 288, 256, 256, 128, 128}, bns[] = {64, 32, 64, 32, 128, 64};
        return {(Cfg)g_force_cfg, bms[g_force_cfg], bns[g_force_cfg], dual ? 1 : (g_force_split > 0 ? g_force_split : 1)};
    }
    // Measured on MI355X (tools/gemm_sweep.py, prefill shapes M = 256 / 288): the 2x2-wave
    // 128x64 tile with split-K wins for the projection GEMMs; the 288-row panel (weights read
    // once, A re-read from L2) wins for the dual gate/up GEMM and the K = 16384 down projection.
    const int nkt = (K + BK - 1) / BK;
    Plan p;
    const bool small_m = M <= 288;
    if (small_m && dual) {
        p = {M <= 256 ? C256x64 : C288x64, M <= 256 ? 256 : 288, 64, 1};
    } else if (small_m && K >= 8192) {
        p = {M <= 256 ? C256x64 : C288x64, M <= 256 ? 256 : 288, 64, 1};
    } else if (dual) {
        p = {C128x128, 128, 128, 1};
        return p;
    } else {
        p = {C128x64, 128, 64, 1};
        if (!small_m && (long)((M + 127) / 128) * ((N + 127) / 128) >= 256) p = {C128x128, 128, 128, 1};
    }
    if (dual) return p;
    const long tiles = (long)((M + p.bm - 1) / p.bm) * ((N + p.bn - 1) / p.bn);
    while (tiles * p.split < 200 && p.split < 8 && nkt / (p.split * 2) >= 2) p.split *= 2;
    return p;
}

size_t gemm_ws_bytes(int M, int N, int K) {
    Plan p = choose(M, N, K, false);
    return p.split > 1 ? (size_t)p.split * M * N * sizeof(float) : 0;
}

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
        hipLaunchKernelGGL((k_gemm<WGM, WGN, TM, TN, EPI_STORE, true>), grid, dim3(NT), lds, s, A, lda, W, ldw, M, N,
                           K, per, ea, ws, up_off);
        return;
    } else if (split == 1) {
        hipLaunchKernelGGL((k_gemm<WGM, WGN, TM, TN, EPI, false>), grid, dim3(NT), lds, s, A, lda, W, ldw, M, N, K,
                           per, ea, ws, up_off);
    } else {
        hipLaunchKernelGGL((k_gemm<WGM, WGN, TM, TN, EPI_STORE, true>), grid, dim3(NT), lds, s, A, lda, W, ldw, M, N,
                           K, per, ea, ws, up_off);
        long total4 = ((long)M * N + 3) / 4;
        long blocks = (total4 + 255) / 256;
        if (blocks > 4096) blocks = 4096;
        hipLaunchKernelGGL((k_splitk_epi<EPI>), dim3((unsigned)blocks), dim3(256), 0, s, ws, split, M, N, ea);
    }
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
    }
}

int gemm(hipStream_t s, const uint16_t* A, int lda, const uint16_t* W, int ldw, int M, int N, int K, Epi epi,
         const EpiArgs& ea, float* ws, size_t ws_bytes, int up_offset_rows, bool defer) {
    Plan p = choose(M, N, K, epi == EPI_GEGLU);
    if (p.split > 1 && (size_t)p.split * M * N * sizeof(float) > ws_bytes) p.split = 1;
    if (p.split > 1 && N % 4 != 0) p.split = 1;  // the split-K epilogue works on 4 outputs per thread
    const long up_off = (long)up_offset_rows * ldw;
    if (defer && p.split > 1) {
        // partial slabs only: the consumer kernel (splitk_res_norm / rope_kv_append) reduces them
        switch (p.cfg) {
            case C288x64: launch_t<6, 1, 3, 4, -1>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off); break;
            case C288x32: launch_t<6, 1, 3, 2, -1>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off); break;
            case C256x64: launch_t<4, 1, 4, 4, -1>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off); break;
            case C256x32: launch_t<4, 1, 4, 2, -1>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off); break;
            case C128x128: launch_t<2, 2, 4, 4, -1>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off); break;
            case C128x64: launch_t<2, 2, 4, 2, -1>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off); break;
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
    }
    return 1;
}

}  // namespace pgmi
