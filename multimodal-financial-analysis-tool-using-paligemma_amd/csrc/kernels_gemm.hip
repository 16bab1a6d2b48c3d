// kernels_gemm.hip -- MFMA bf16 GEMM for the prefill path (gfx950, v_mfma_f32_16x16x32_bf16).
//
// C[M,N] = A[M,K] . W[N,K]^T with both operands K-contiguous (nn.Linear layout, so the
// reference's weights are used as stored).  Covers every nn.Linear / Conv2d of the
// prefill (modeling_siglip.py:45-51,92-95,154-155; modeling_gemma.py:129-131,220-223,
// 391,433) with the reference's rounding points fused into the epilogue.
//
// Tile: BM x BN x 64, 256 threads = 4 waves in a 2x2 grid, each wave (BM/2)x(BN/2) of
// 16x16 MFMA tiles; A/B tiles staged global -> registers -> LDS (double buffered, one
// barrier per k-tile, next tile's global loads in flight during the MFMAs).  LDS rows
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
template <int BM, int BN, int EPI, bool SPLIT>
__global__ void __launch_bounds__(256) k_gemm(const uint16_t* __restrict__ A, int lda, const uint16_t* __restrict__ W,
                                              int ldw, int M, int N, int K, int kt_per_split, EpiArgs ea,
                                              float* __restrict__ ws, long up_off) {
    constexpr bool DUAL = (EPI == EPI_GEGLU);
    constexpr int WM = BM / 2, WN = BN / 2;
    constexpr int TM = WM / 16, TN = WN / 16;
    constexpr int ACH = BM * 8 / 256;  // 16-B chunks of the A tile per thread
    constexpr int BCH = BN * 8 / 256;
    constexpr int NB = DUAL ? 2 : 1;
    extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
    uint16_t* As = smem;                         // [2][BM][LDSK]
    uint16_t* Bs = smem + 2 * BM * LDSK;         // [2][NB][BN][LDSK]

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    // XCD-aware-free simple mapping: blocks walk N fastest so neighbours share the A panel
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

    uint4 ra[ACH], rb[NB][BCH];
    auto gload = [&](int kt) {
        const int kbase = kt * BK;
#pragma unroll
        for (int i = 0; i < ACH; ++i) {
            const int c = tid + 256 * i, r = c >> 3, kc = (c & 7) * 8;
            const int gm = m0 + r, gk = kbase + kc;
            ra[i] = (gm < M && gk < K) ? ldg16(A + (long)gm * lda + gk) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
            for (int i = 0; i < BCH; ++i) {
                const int c = tid + 256 * i, r = c >> 3, kc = (c & 7) * 8;
                const int gn = n0 + r, gk = kbase + kc;
                rb[b][i] = (gn < N && gk < K) ? ldg16(W + b * up_off + (long)gn * ldw + gk) : make_uint4(0, 0, 0, 0);
            }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < ACH; ++i) {
            const int c = tid + 256 * i, r = c >> 3, kc = (c & 7) * 8;
            *reinterpret_cast<uint4*>(As + (buf * BM + r) * LDSK + kc) = ra[i];
        }
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
            for (int i = 0; i < BCH; ++i) {
                const int c = tid + 256 * i, r = c >> 3, kc = (c & 7) * 8;
                *reinterpret_cast<uint4*>(Bs + ((buf * NB + b) * BN + r) * LDSK + kc) = rb[b][i];
            }
    };

    if (nkt > 0) {
        gload(kt0);
        lstore(0);
    }
    __syncthreads();
    int cur = 0;
    for (int t = 0; t < nkt; ++t) {
        if (t + 1 < nkt) gload(kt0 + t + 1);
#pragma unroll
        for (int kk = 0; kk < BK / 32; ++kk) {
            const int kof = kk * 32 + 8 * (lane >> 4);
            short8 af[TM], bfr[NB][TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
                af[i] = *reinterpret_cast<const short8*>(As + (cur * BM + wr * WM + i * 16 + (lane & 15)) * LDSK + kof);
#pragma unroll
            for (int b = 0; b < NB; ++b)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    bfr[b][j] = *reinterpret_cast<const short8*>(
                        Bs + ((cur * NB + b) * BN + wc * WN + j * 16 + (lane & 15)) * LDSK + kof);
#pragma unroll
            for (int b = 0; b < NB; ++b)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) acc[b][i][j] = mfma16(af[i], bfr[b][j], acc[b][i][j]);
        }
        if (t + 1 < nkt) lstore(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }

    // C/D map of 16x16x32: col = lane & 15, row = (lane >> 4) * 4 + r
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wc * WN + j * 16 + (lane & 15);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wr * WM + i * 16 + (lane >> 4) * 4 + r;
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

// split-K reduction in fixed z order + epilogue
template <int EPI>
__global__ void k_splitk_epi(const float* __restrict__ ws, int S, int M, int N, EpiArgs ea) {
    const long total = (long)M * N;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        float a = 0.f;
        for (int z = 0; z < S; ++z) a += ws[(long)z * total + i];
        epi_store<EPI>(ea, (int)(i / N), (int)(i % N), a, 0.f);
    }
}

struct Plan {
    int bm, bn, split;
};

static Plan choose(int M, int N, int K, bool dual) {
    // prefer BM that tiles M exactly (M = 256 vision rows, 288 = 256 + 32 text rows)
    int bm = 128;
    if (M % 128 != 0) {
        if (M % 96 == 0) bm = 96;
        else if (M <= 64) bm = 64;
        else bm = 128;
    }
    int bn = dual ? 64 : 128;
    const int tiles_m = (M + bm - 1) / bm;
    int tiles = tiles_m * ((N + bn - 1) / bn);
    if (!dual && tiles < 256) {
        bn = 64;
        tiles = tiles_m * ((N + bn - 1) / bn);
    }
    const int nkt = (K + BK - 1) / BK;
    int split = 1;
    if (!dual) {
        while (tiles * split < 256 && split * 2 <= 16 && nkt / (split * 2) >= 4) split *= 2;
    }
    return {bm, bn, split};
}

size_t gemm_ws_bytes(int M, int N, int K) {
    Plan p = choose(M, N, K, false);
    return p.split > 1 ? (size_t)p.split * M * N * sizeof(float) : 0;
}

template <int BM, int BN, int EPI>
static void launch_t(hipStream_t s, const uint16_t* A, int lda, const uint16_t* W, int ldw, int M, int N, int K,
                     const EpiArgs& ea, float* ws, int split, long up_off) {
    constexpr int NB = (EPI == EPI_GEGLU) ? 2 : 1;
    const size_t lds = (size_t)(2 * BM * LDSK + 2 * NB * BN * LDSK) * sizeof(uint16_t);
    const int nkt = (K + BK - 1) / BK;
    const int per = (nkt + split - 1) / split;
    dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM, split);
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm<BM, BN, EPI, false>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm<BM, BN, EPI_STORE, true>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr_set = true;
    }
    if (split == 1) {
        hipLaunchKernelGGL((k_gemm<BM, BN, EPI, false>), grid, dim3(256), lds, s, A, lda, W, ldw, M, N, K, per, ea,
                           ws, up_off);
    } else {
        hipLaunchKernelGGL((k_gemm<BM, BN, EPI_STORE, true>), grid, dim3(256), lds, s, A, lda, W, ldw, M, N, K, per,
                           ea, ws, up_off);
        long total = (long)M * N;
        long blocks = (total + 255) / 256;
        if (blocks > 8192) blocks = 8192;
        hipLaunchKernelGGL((k_splitk_epi<EPI>), dim3((unsigned)blocks), dim3(256), 0, s, ws, split, M, N, ea);
    }
}

template <int EPI>
static void launch_e(hipStream_t s, const uint16_t* A, int lda, const uint16_t* W, int ldw, int M, int N, int K,
                     const EpiArgs& ea, float* ws, const Plan& p, long up_off) {
#define PGMI_GEMM_CASE(BM_, BN_)                                                           \
    if (p.bm == BM_ && p.bn == BN_) {                                                      \
        launch_t<BM_, BN_, EPI>(s, A, lda, W, ldw, M, N, K, ea, ws, p.split, up_off);      \
        return;                                                                            \
    }
    PGMI_GEMM_CASE(128, 128)
    PGMI_GEMM_CASE(128, 64)
    PGMI_GEMM_CASE(96, 128)
    PGMI_GEMM_CASE(96, 64)
    PGMI_GEMM_CASE(64, 128)
    PGMI_GEMM_CASE(64, 64)
#undef PGMI_GEMM_CASE
}

void gemm(hipStream_t s, const uint16_t* A, int lda, const uint16_t* W, int ldw, int M, int N, int K, Epi epi,
          const EpiArgs& ea, float* ws, size_t ws_bytes, int up_offset_rows) {
    Plan p = choose(M, N, K, epi == EPI_GEGLU);
    if (p.split > 1 && (size_t)p.split * M * N * sizeof(float) > ws_bytes) p.split = 1;
    const long up_off = (long)up_offset_rows * ldw;
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
}

}  // namespace pgmi
