// kernels_sample.hip -- temperature softmax + top-p (nucleus) sampling on the device
// (inference.py:15-24 _sample_top_p, with the softmax(logits / T) of :65), SURVEY.md sec.8f rank 4.
//
// The reference sorts all 257,216 probabilities, takes the cumulative sum, zeroes every entry
// whose preceding mass already exceeds p, renormalises and draws with torch.multinomial.  The
// kept tokens are a prefix of the descending order, so both decisions are "the first sorted
// position whose inclusive cumulative mass exceeds a target": target p gives the nucleus
// cut-off k*, and target r = u * Z (Z = the kept mass, u ~ U[0,1) from the caller) gives the
// draw, which lands at or before k* because r < Z.  Each is a mass-weighted radix select over
// the fp32 bit patterns (probabilities are >= 0, so the bit order is the value order): four
// 8-bit digit levels of 256-bin (count, mass) histograms, walking bins from the top until the
// running mass crosses the target, then equal probabilities resolved in index order (our tie
// rule; torch.sort does not define one).  No sort and no materialised cumsum; masses in fp64.
//
// One 1024-thread workgroup per row; the row's probabilities live in a global scratch row
// (fp32, L2-resident across the passes).  The draw is a function of u, so it is checkable
// against the sort-based restatement in oracle/sampling_np.py.
#include "common.h"
#include "launch.h"

namespace pgmi {

constexpr int kSampleThreads = 1024;
// probability masses are summed as 2^-62 fixed point in u64: native integer LDS atomics (fp64
// atomics lower to CAS loops), order-independent and therefore deterministic sums; a row's total
// (<= 1 + rounding) stays below 2^63, and a single probability loses < 2^-62 to truncation
constexpr double kMassScale = 4611686018427387904.0;  // 2^62
constexpr double kMassUnit = 1.0 / kMassScale;
__device__ __forceinline__ unsigned long long mass_q(float v) { return (unsigned long long)((double)v * kMassScale); }
constexpr int kSampleWaves = kSampleThreads / 64;

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// block reductions; every thread gets the result (fixed combine order over waves)
__device__ __forceinline__ float block_max_f(float v, float* red) {
    v = wave_max(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    float m = red[0];
    for (int i = 1; i < kSampleWaves; ++i) m = fmaxf(m, red[i]);
    return m;
}

__device__ __forceinline__ double block_sum_d(double v, double* red) {
    v = wave_sum_d(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double s = 0.0;
    for (int i = 0; i < kSampleWaves; ++i) s += red[i];
    return s;
}

struct SelectOut {
    uint32_t key;  // bit pattern of the probability at the crossing position
    double above;  // mass of every probability > key
    int rank;      // the crossing is the rank-th (index order, 0-based) token equal to key
    bool crossed;  // false: target >= the total mass (no crossing)
};

struct SampleSmem {
    unsigned hcnt[256];
    unsigned long long hmq[256];
    double red_d[kSampleWaves];
    float red_f[kSampleWaves];
    int sel;
    double acc;
    int found;
    int scan[kSampleThreads];
    double suf[256 + 4];
};

// The first bin, walking from the top (bin 255) down, at which `above + (mass of that bin and
// every bin above it)` exceeds target: a suffix scan over the 256 bins (one per thread of the
// first 256), then the LARGEST bin whose suffix crosses (suffix sums are monotone up to
// rounding; taking the largest keeps the answer unique).  Returns the bin (-1: none) and sets
// *above_out to the mass above the bin.  Every thread of the block must call it.
__device__ int crossing_bin(const unsigned* cnt, const unsigned long long* mq, double above, double target,
                            double* suf, int* sh_int, double* sh_d, double* above_out) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    double v = 0.0;
    if (t < 256) {  // suffix within the wave's 64 bins (bin 64w + lane), by shuffles
        v = (double)mq[t] * kMassUnit;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const double x = __shfl_down(v, o, 64);
            if (lane + o < 64) v += x;
        }
        if (lane == 0) suf[256 + w] = v;  // the wave's total
    }
    if (t == 0) sh_int[0] = -1;
    __syncthreads();
    if (t < 256) {
        for (int q = w + 1; q < 4; ++q) v += suf[256 + q];  // higher waves' bins, fixed order
        suf[t] = v;
        if (cnt[t] != 0u && above + v > target) atomicMax(sh_int, t);
    }
    __syncthreads();
    const int d = sh_int[0];
    if (t == 0) sh_d[0] = d >= 0 ? above + (suf[d] - (double)mq[d] * kMassUnit) : above + suf[0];
    __syncthreads();
    *above_out = sh_d[0];
    return d;
}

__device__ __forceinline__ void hist_add(unsigned* hcnt, unsigned long long* hmq, bool valid, int d, float v) {
    if (valid) {
        atomicAdd(&hcnt[d], 1u);
        atomicAdd(&hmq[d], mass_q(v));
    }
}

// the first position of the descending order whose inclusive cumulative mass exceeds target
__device__ SelectOut radix_select(const float* __restrict__ p, int V, double target, double above0, SampleSmem& sm) {
    const int tid = threadIdx.x;
    uint32_t prefix = 0, pmask = 0;
    double above = above0;
    for (int level = 3; level >= 0; --level) {
        const int shift = level * 8;
        for (int i = tid; i < 256; i += kSampleThreads) {
            sm.hcnt[i] = 0u;
            sm.hmq[i] = 0ull;
        }
        __syncthreads();
        for (int i0 = 0; i0 < V; i0 += kSampleThreads) {  // wave-uniform trip count
            const int i = i0 + tid;
            const float v = i < V ? p[i] : 0.f;
            const uint32_t k = __float_as_uint(v);
            hist_add(sm.hcnt, sm.hmq, i < V && (k & pmask) == prefix, (int)((k >> shift) & 255), v);
        }
        __syncthreads();
        double a;
        const int sel = crossing_bin(sm.hcnt, sm.hmq, above, target, sm.suf, &sm.sel, &sm.acc, &a);
        above = a;
        if (sel < 0) return SelectOut{0u, above, 0, false};
        prefix |= (uint32_t)sel << shift;
        pmask |= 255u << shift;
    }
    // tokens equal to the key: the crossing is at the smallest tie rank j with
    // above + (j + 1) * value > target
    const double val = (double)__uint_as_float(prefix);
    int rank = 0;
    if (val > 0.0) {
        double need = floor((target - above) / val);
        rank = need < 0.0 ? 0 : (need > 2e9 ? 2000000000 : (int)need);
        while (rank > 0 && above + (double)rank * val > target) --rank;
        while (!(above + (double)(rank + 1) * val > target)) ++rank;
    }
    return SelectOut{prefix, above, rank, true};
}

// index of the rank-th token (index order) whose bit pattern equals key; -1 if fewer exist
__device__ int nth_equal(const float* __restrict__ p, int V, uint32_t key, int rank, SampleSmem& sm) {
    const int tid = threadIdx.x;
    const int per = (V + kSampleThreads - 1) / kSampleThreads;  // contiguous slice per thread
    const int i0 = tid * per, i1 = min(V, i0 + per);
    int c = 0;
    for (int i = i0; i < i1; ++i) c += (__float_as_uint(p[i]) == key);
    // exclusive prefix of the threads' counts: within the wave by shuffles, then wave totals
    const int lane = tid & 63, wave = tid >> 6;
    int incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
    }
    __syncthreads();
    if (lane == 63) sm.scan[wave] = incl;
    if (tid == 0) sm.found = -1;
    __syncthreads();
    int wbase = 0;
    for (int w = 0; w < wave; ++w) wbase += sm.scan[w];
    const int base = wbase + incl - c;
    if (rank >= base && rank < base + c) {
        int r = rank - base;
        for (int i = i0; i < i1; ++i)
            if (__float_as_uint(p[i]) == key) {
                if (r == 0) {
                    sm.found = i;
                    break;
                }
                --r;
            }
    }
    __syncthreads();
    return sm.found;
}

// ---------------------------------------------------------------- the multi-kernel pipeline
// Per row: (1) k_tp_stats, NB blocks: max and sum of exp of z = x / T per slice;
// (2) k_tp_hist, NB blocks: p = softmax, written once, and per-block histograms of the fp32
// exponent field (256 bins of count and fp64 mass, no global atomics: block order is the sum
// order); (3) k_tp_plan, one block: the cut-off bin c1 (where the running mass crosses p) and
// the highest bin c_hi the draw can reach (r = u Z >= u * mass above c1), so every position the
// two decisions can land on lies in bins [c1, c_hi], with A_out the mass above c_hi;
// (4) k_tp_compact, NB blocks: the tokens of bins [c1, c_hi] -> (value, index) in index order;
// (5) k_tp_select, one block: the two radix selects of the header over the candidates only.
constexpr int kTpThreads = 256;

struct TpLayout {
    size_t p, cv, ci, bm, bs, hc, rc, hm, pre, meta, stride;  // byte offsets within one row's scratch
};

__host__ __device__ inline size_t tp_align(size_t x) { return (x + 255) & ~(size_t)255; }

__host__ __device__ inline TpLayout tp_layout(int V, int NB) {
    TpLayout L;
    size_t o = 0;
    L.p = o; o = tp_align(o + (size_t)V * 4);
    L.cv = o; o = tp_align(o + (size_t)V * 4);
    L.ci = o; o = tp_align(o + (size_t)V * 4);
    L.bm = o; o = tp_align(o + (size_t)NB * 4);
    L.bs = o; o = tp_align(o + (size_t)NB * 8);
    L.hc = o; o = tp_align(o + (size_t)NB * 256 * 4);
    L.rc = o; o = tp_align(o + (size_t)256 * 4);
    L.hm = o; o = tp_align(o + (size_t)256 * 8);
    L.pre = o; o = tp_align(o + (size_t)NB * 4);
    L.meta = o; o = tp_align(o + 16 * 8);
    L.stride = o;
    return L;
}

struct TpMeta {  // one row's plan (k_tp_plan -> k_tp_compact, k_tp_select)
    double a_out;   // mass of the bins above c_hi
    double total;   // mass of the row
    int c1, c_hi;   // candidate bins [c1, c_hi]
    int n_cand;
    int crossed;    // the cut-off exists (p < total mass)
};

__device__ __forceinline__ int tp_bin(float v) { return (int)((__float_as_uint(v) >> 23) & 255u); }

__device__ __forceinline__ void tp_slice(int V, int NB, int b, int& i0, int& i1) {
    const int per = (V + NB - 1) / NB;
    i0 = b * per;
    i1 = min(V, i0 + per);
}

__global__ void __launch_bounds__(kTpThreads) k_tp_stats(const float* __restrict__ x, int V, float temperature,
                                                          int NB, uint8_t* __restrict__ scratch, TpLayout L) {
    __shared__ float red_f[kTpThreads / 64];
    __shared__ double red_d[kTpThreads / 64];
    const int b = blockIdx.x, row = blockIdx.y, tid = threadIdx.x;
    const float* xr = x + (long)row * V;
    uint8_t* base = scratch + (size_t)row * L.stride;
    int i0, i1;
    tp_slice(V, NB, b, i0, i1);
    float m = -INFINITY;
    for (int i = i0 + tid; i < i1; i += kTpThreads) m = fmaxf(m, xr[i] / temperature);
    m = wave_max(m);
    if ((tid & 63) == 0) red_f[tid >> 6] = m;
    __syncthreads();
    m = red_f[0];
    for (int w = 1; w < kTpThreads / 64; ++w) m = fmaxf(m, red_f[w]);
    double sum = 0.0;
    if (m != -INFINITY)
        for (int i = i0 + tid; i < i1; i += kTpThreads) sum += (double)expf(xr[i] / temperature - m);
    sum = wave_sum_d(sum);
    if ((tid & 63) == 0) red_d[tid >> 6] = sum;
    __syncthreads();
    if (tid == 0) {
        double t = 0.0;
        for (int w = 0; w < kTpThreads / 64; ++w) t += red_d[w];
        reinterpret_cast<float*>(base + L.bm)[b] = m;
        reinterpret_cast<double*>(base + L.bs)[b] = t;
    }
    if (b == 0) {  // the row histogram k_tp_hist accumulates into
        reinterpret_cast<unsigned*>(base + L.rc)[tid] = 0u;
        reinterpret_cast<unsigned long long*>(base + L.hm)[tid] = 0ull;
    }
}

__global__ void __launch_bounds__(kTpThreads) k_tp_zero(uint8_t* __restrict__ scratch, TpLayout L) {
    uint8_t* base = scratch + (size_t)blockIdx.x * L.stride;
    reinterpret_cast<unsigned*>(base + L.rc)[threadIdx.x] = 0u;
    reinterpret_cast<unsigned long long*>(base + L.hm)[threadIdx.x] = 0ull;
}

__global__ void __launch_bounds__(kTpThreads) k_tp_hist(const float* __restrict__ x, int V, float temperature, int NB,
                                                         uint8_t* __restrict__ scratch, TpLayout L) {
    __shared__ unsigned hcnt[256];
    __shared__ unsigned long long hmq[256];
    const int b = blockIdx.x, row = blockIdx.y, tid = threadIdx.x;
    const float* xr = x + (long)row * V;
    uint8_t* base = scratch + (size_t)row * L.stride;
    float* p = reinterpret_cast<float*>(base + L.p);
    hcnt[tid] = 0u;
    hmq[tid] = 0ull;
    __shared__ float red_f[kTpThreads / 64];
    __shared__ double red_d[kTpThreads / 64];
    float m = 0.f, sumf = 1.f;
    if (temperature > 0.f) {  // softmax(x / T): global max, then the slices' sums of exp rescaled to it
        const float* bm = reinterpret_cast<const float*>(base + L.bm);
        const double* bs = reinterpret_cast<const double*>(base + L.bs);
        float mq = -INFINITY;
        for (int q = tid; q < NB; q += kTpThreads) mq = fmaxf(mq, bm[q]);
        mq = wave_max(mq);
        if ((tid & 63) == 0) red_f[tid >> 6] = mq;
        __syncthreads();
        m = red_f[0];
        for (int w = 1; w < kTpThreads / 64; ++w) m = fmaxf(m, red_f[w]);
        double S = 0.0;
        for (int q = tid; q < NB; q += kTpThreads)
            if (bm[q] != -INFINITY) S += bs[q] * exp((double)bm[q] - (double)m);
        S = wave_sum_d(S);  // a fixed reduction tree: the same sum every run
        if ((tid & 63) == 0) red_d[tid >> 6] = S;
        __syncthreads();
        S = 0.0;
        for (int w = 0; w < kTpThreads / 64; ++w) S += red_d[w];
        sumf = (float)S;
    }
    __syncthreads();
    int i0, i1;
    tp_slice(V, NB, b, i0, i1);
    for (int c0 = i0; c0 < i1; c0 += kTpThreads) {  // block-uniform trip count
        const int i = c0 + tid;
        float v = 0.f;
        if (i < i1) {
            v = temperature > 0.f ? expf(xr[i] / temperature - m) / sumf : xr[i];
            if (!(v > 0.f)) v = 0.f;  // negative / NaN probabilities carry no mass
            p[i] = v;
        }
        hist_add(hcnt, hmq, i < i1, tp_bin(v), v);
    }
    __syncthreads();
    reinterpret_cast<unsigned*>(base + L.hc)[b * 256 + tid] = hcnt[tid];  // per-block counts (compaction offsets)
    if (hcnt[tid]) {  // the row histogram: integer atomics, so the sums do not depend on arrival order
        atomicAdd(reinterpret_cast<unsigned*>(base + L.rc) + tid, hcnt[tid]);
        atomicAdd(reinterpret_cast<unsigned long long*>(base + L.hm) + tid, hmq[tid]);
    }
}

__global__ void __launch_bounds__(256) k_tp_plan(int NB, float top_p, const float* __restrict__ u,
                                                 uint8_t* __restrict__ scratch, TpLayout L) {
    __shared__ unsigned cnt[256];
    __shared__ unsigned long long mq[256];
    __shared__ int range[2];
    const int row = blockIdx.x, t = threadIdx.x;
    uint8_t* base = scratch + (size_t)row * L.stride;
    const unsigned* hc = reinterpret_cast<const unsigned*>(base + L.hc);
    cnt[t] = reinterpret_cast<const unsigned*>(base + L.rc)[t];
    mq[t] = reinterpret_cast<const unsigned long long*>(base + L.hm)[t];
    __syncthreads();
    __shared__ double suf[256 + 4];
    __shared__ int sh_int[1];
    __shared__ double sh_d[1];
    double total = 0.0, a1 = 0.0;
    const double tp = (double)top_p;
    // lowest non-empty bin and the total mass
    if (t == 0) sh_int[0] = 256;
    __syncthreads();
    if (cnt[t]) atomicMin(sh_int, t);
    __syncthreads();
    const int lowest = sh_int[0] < 256 ? sh_int[0] : 0;
    __syncthreads();
    int c1 = crossing_bin(cnt, mq, 0.0, tp, suf, sh_int, sh_d, &a1);
    total = suf[0];
    __syncthreads();  // suf is rewritten by the next crossing_bin
    const bool crossed = c1 >= 0;
    if (!crossed) {  // everything is kept
        c1 = lowest;
        a1 = total - (double)mq[lowest] * kMassUnit;
    }
    double uu = (double)u[row];
    if (!(uu >= 0.0)) uu = 0.0;
    if (uu >= 1.0) uu = 1.0 - 1.0 / 16777216.0;
    double a_out = 0.0;
    int chi = crossing_bin(cnt, mq, 0.0, uu * a1, suf, sh_int, sh_d, &a_out);  // r = u Z >= u * a1
    if (chi < c1) {
        chi = c1;
        a_out = a1;
    }
    if (t == 0) {
        range[0] = c1;
        range[1] = chi;
        TpMeta M{};
        M.a_out = a_out;
        M.total = total;
        M.c1 = c1;
        M.c_hi = chi;
        M.crossed = crossed;
        *reinterpret_cast<TpMeta*>(base + L.meta) = M;
    }
    __syncthreads();
    // candidate prefix per block (block order = index order)
    __shared__ unsigned bc[256];
    for (int q = t; q < NB; q += 256) {
        unsigned k = 0u;
        for (int d = range[0]; d <= range[1]; ++d) k += hc[q * 256 + d];
        bc[q] = k;
    }
    __syncthreads();
    if (t == 0) {
        unsigned* pre = reinterpret_cast<unsigned*>(base + L.pre);
        unsigned run = 0u;
        for (int q = 0; q < NB; ++q) {
            pre[q] = run;
            run += bc[q];
        }
        reinterpret_cast<TpMeta*>(base + L.meta)->n_cand = (int)run;
    }
}

__global__ void __launch_bounds__(kTpThreads) k_tp_compact(int V, int NB, uint8_t* __restrict__ scratch, TpLayout L) {
    __shared__ unsigned wtot[kTpThreads / 64];
    const int b = blockIdx.x, row = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint8_t* base = scratch + (size_t)row * L.stride;
    const float* p = reinterpret_cast<const float*>(base + L.p);
    float* cv = reinterpret_cast<float*>(base + L.cv);
    int* ci = reinterpret_cast<int*>(base + L.ci);
    const TpMeta M = *reinterpret_cast<const TpMeta*>(base + L.meta);
    unsigned off = reinterpret_cast<const unsigned*>(base + L.pre)[b];
    int i0, i1;
    tp_slice(V, NB, b, i0, i1);
    for (int c0 = i0; c0 < i1; c0 += kTpThreads) {  // ordered compaction, 256 tokens per round
        const int i = c0 + tid;
        float v = 0.f;
        bool f = false;
        if (i < i1) {
            v = p[i];
            const int d = tp_bin(v);
            f = d >= M.c1 && d <= M.c_hi;
        }
        const unsigned long long bal = __ballot(f);
        const unsigned below = (unsigned)__popcll(bal & ((1ull << lane) - 1ull));
        __syncthreads();
        if (lane == 0) wtot[wave] = (unsigned)__popcll(bal);
        __syncthreads();
        unsigned wo = 0u, all = 0u;
        for (int w = 0; w < kTpThreads / 64; ++w) {
            if (w < wave) wo += wtot[w];
            all += wtot[w];
        }
        if (f) {
            cv[off + wo + below] = v;
            ci[off + wo + below] = i;
        }
        off += all;
    }
}

__global__ void __launch_bounds__(kSampleThreads) k_tp_select(float top_p, const float* __restrict__ u,
                                                               uint8_t* __restrict__ scratch, TpLayout L,
                                                               int64_t* __restrict__ out, float* __restrict__ kept_mass) {
    __shared__ SampleSmem sm;
    const int row = blockIdx.x, tid = threadIdx.x;
    uint8_t* base = scratch + (size_t)row * L.stride;
    const float* cv = reinterpret_cast<const float*>(base + L.cv);
    const int* ci = reinterpret_cast<const int*>(base + L.ci);
    const TpMeta M = *reinterpret_cast<const TpMeta*>(base + L.meta);
    const int n = M.n_cand;

    // nucleus cut-off.  In exact arithmetic the kept prefix ends at k, the first position whose
    // cumulative mass C exceeds p.  The reference decides in fp32 -- C is torch's CPU cumsum
    // (double accumulation, fp32 store) and position i is dropped iff fp32(fp32(C_i) - p_i) > p
    // (:18-19) -- which can drop k or keep positions after it when C lands within an fp32 ulp
    // of p; those boundary positions are re-decided by that formula.
    auto ref_dropped = [&](double C, float v) { return __fsub_rn((float)C, v) > top_p; };
    double Z = M.total;
    SelectOut cut{0u, 0.0, 0, false};
    if (M.crossed) {
        cut = radix_select(cv, n, (double)top_p, M.a_out, sm);
        if (cut.crossed) {
            const float vk = __uint_as_float(cut.key);
            const double Ck = cut.above + (double)(cut.rank + 1) * (double)vk;
            if (ref_dropped(Ck, vk)) {
                Z = Ck - (double)vk;
            } else {
                Z = Ck;
                for (int extra = 0; extra < 4; ++extra) {  // positions after k that fp32 still keeps
                    const SelectOut nx = radix_select(cv, n, Z, M.a_out, sm);
                    if (!nx.crossed) break;
                    const float vn = __uint_as_float(nx.key);
                    const double Cn = nx.above + (double)(nx.rank + 1) * (double)vn;
                    if (ref_dropped(Cn, vn)) break;
                    Z = Cn;
                }
            }
            if (!(Z > 0.0)) Z = Ck;  // a first token alone beyond p is always kept (:19, C_0 - p_0 = 0)
        }
    }
    // the draw: first position whose inclusive mass exceeds r = u * Z (r < Z, so it is <= k*)
    double uu = (double)u[row];
    if (!(uu >= 0.0)) uu = 0.0;
    if (uu >= 1.0) uu = 1.0 - 1.0 / 16777216.0;
    const SelectOut pick = radix_select(cv, n, uu * Z, M.a_out, sm);
    int pos = -1;
    if (pick.crossed) pos = nth_equal(cv, n, pick.key, pick.rank, sm);
    if (pos < 0 && cut.crossed) pos = nth_equal(cv, n, cut.key, cut.rank, sm);  // rounding at the very end
    if (tid == 0) {
        out[row] = pos >= 0 ? ci[pos] : 0;
        if (kept_mass) kept_mass[row] = (float)Z;
    }
}

static int tp_blocks(int V) {
    const int nb = (V + 2047) / 2048;
    return nb < 1 ? 1 : (nb > 128 ? 128 : nb);
}

size_t sample_scratch_bytes(int rows, int V) { return (size_t)rows * tp_layout(V, tp_blocks(V)).stride; }

void sample_top_p(hipStream_t s, const float* x, int rows, int V, float temperature, float top_p, const float* u,
                  void* scratch, int64_t* out, float* kept_mass) {
    const int NB = tp_blocks(V);
    const TpLayout L = tp_layout(V, NB);
    uint8_t* sc = reinterpret_cast<uint8_t*>(scratch);
    if (temperature > 0.f)
        hipLaunchKernelGGL(k_tp_stats, dim3(NB, rows), dim3(kTpThreads), 0, s, x, V, temperature, NB, sc, L);
    else
        hipLaunchKernelGGL(k_tp_zero, dim3(rows), dim3(kTpThreads), 0, s, sc, L);
    hipLaunchKernelGGL(k_tp_hist, dim3(NB, rows), dim3(kTpThreads), 0, s, x, V, temperature, NB, sc, L);
    hipLaunchKernelGGL(k_tp_plan, dim3(rows), dim3(256), 0, s, NB, top_p, u, sc, L);
    hipLaunchKernelGGL(k_tp_compact, dim3(NB, rows), dim3(kTpThreads), 0, s, V, NB, sc, L);
    hipLaunchKernelGGL(k_tp_select, dim3(rows), dim3(kSampleThreads), 0, s, top_p, u, sc, L, out, kept_mass);
}

}  // namespace pgmi
