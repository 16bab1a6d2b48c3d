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
    double hmass[256];
    double red_d[kSampleWaves];
    float red_f[kSampleWaves];
    int sel;
    double acc;
    int found;
    int scan[kSampleThreads];
};

// the first position of the descending order whose inclusive cumulative mass exceeds target
__device__ SelectOut radix_select(const float* __restrict__ p, int V, double target, SampleSmem& sm) {
    const int tid = threadIdx.x;
    uint32_t prefix = 0, pmask = 0;
    double above = 0.0;
    for (int level = 3; level >= 0; --level) {
        const int shift = level * 8;
        for (int i = tid; i < 256; i += kSampleThreads) {
            sm.hcnt[i] = 0u;
            sm.hmass[i] = 0.0;
        }
        __syncthreads();
        for (int i = tid; i < V; i += kSampleThreads) {
            const float v = p[i];
            const uint32_t k = __float_as_uint(v);
            if ((k & pmask) == prefix) {
                const int d = (k >> shift) & 255;
                atomicAdd(&sm.hcnt[d], 1u);
                atomicAdd(&sm.hmass[d], (double)v);
            }
        }
        __syncthreads();
        if (tid == 0) {
            int sel = -1;
            double a = above;
            for (int d = 255; d >= 0; --d) {
                if (sm.hcnt[d] == 0u) continue;
                if (a + sm.hmass[d] > target) {
                    sel = d;
                    break;
                }
                a += sm.hmass[d];
            }
            sm.sel = sel;
            sm.acc = a;
        }
        __syncthreads();
        const int sel = sm.sel;
        above = sm.acc;
        __syncthreads();
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
    __syncthreads();
    sm.scan[tid] = c;
    if (tid == 0) sm.found = -1;
    __syncthreads();
    if (tid == 0) {  // exclusive prefix over the threads' counts
        int s = 0;
        for (int t = 0; t < kSampleThreads; ++t) {
            const int x = sm.scan[t];
            sm.scan[t] = s;
            s += x;
        }
    }
    __syncthreads();
    const int base = sm.scan[tid];
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

// x: [rows][V] logits (temperature > 0: softmax(x / temperature), inference.py:65) or
// probabilities (temperature <= 0: used as given, _sample_top_p's input); u: [rows] uniforms.
__global__ void __launch_bounds__(kSampleThreads) k_sample_top_p(const float* __restrict__ x, int V,
                                                                float temperature, float top_p,
                                                                const float* __restrict__ u,
                                                                float* __restrict__ scratch,
                                                                int64_t* __restrict__ out,
                                                                float* __restrict__ kept_mass) {
    __shared__ SampleSmem sm;
    const int row = blockIdx.x, tid = threadIdx.x;
    const float* xr = x + (long)row * V;
    float* p = scratch + (long)row * V;

    if (temperature > 0.f) {
        // torch.softmax(logits / T, -1): max, exp(z - max), sum, divide (fp32 values; the sum
        // in fp64, rounded once to fp32 for the division)
        float m = -INFINITY;
        for (int i = tid; i < V; i += kSampleThreads) m = fmaxf(m, xr[i] / temperature);
        m = block_max_f(m, sm.red_f);
        double s = 0.0;
        for (int i = tid; i < V; i += kSampleThreads) {
            const float e = expf(xr[i] / temperature - m);
            p[i] = e;
            s += (double)e;
        }
        const float sum = (float)block_sum_d(s, sm.red_d);
        for (int i = tid; i < V; i += kSampleThreads) p[i] = p[i] / sum;
    } else {
        for (int i = tid; i < V; i += kSampleThreads) p[i] = xr[i];
    }
    __syncthreads();

    // nucleus cut-off.  In exact arithmetic the kept prefix ends at k, the first position whose
    // cumulative mass C exceeds p.  The reference decides in fp32 -- C is torch's CPU cumsum
    // (double accumulation, fp32 store) and position i is dropped iff fp32(fp32(C_i) - p_i) > p
    // (:18-19) -- which can drop k or keep positions after it when C lands within an fp32 ulp
    // of p; those boundary positions are re-decided by that formula.
    const SelectOut cut = radix_select(p, V, (double)top_p, sm);
    auto ref_dropped = [&](double C, float v) { return __fsub_rn((float)C, v) > top_p; };
    double Z;
    if (cut.crossed) {
        const float vk = __uint_as_float(cut.key);
        const double Ck = cut.above + (double)(cut.rank + 1) * (double)vk;
        if (ref_dropped(Ck, vk)) {
            Z = Ck - (double)vk;
        } else {
            Z = Ck;
            for (int extra = 0; extra < 4; ++extra) {  // positions after k that fp32 still keeps
                const SelectOut nx = radix_select(p, V, Z, sm);
                if (!nx.crossed) break;
                const float vn = __uint_as_float(nx.key);
                const double Cn = nx.above + (double)(nx.rank + 1) * (double)vn;
                if (ref_dropped(Cn, vn)) break;
                Z = Cn;
            }
        }
        if (!(Z > 0.0)) Z = Ck;  // (a first token alone beyond p is always kept: :19 with C_0 - p_0 = 0)
    } else {
        double s = 0.0;
        for (int i = tid; i < V; i += kSampleThreads) s += (double)p[i];
        Z = block_sum_d(s, sm.red_d);
    }
    // the draw: first position whose inclusive mass exceeds r = u * Z (r < Z, so it is <= k*)
    double uu = (double)u[row];
    if (!(uu >= 0.0)) uu = 0.0;
    if (uu >= 1.0) uu = 1.0 - 1.0 / 16777216.0;
    const SelectOut pick = radix_select(p, V, uu * Z, sm);
    int idx = -1;
    if (pick.crossed) idx = nth_equal(p, V, pick.key, pick.rank, sm);
    if (idx < 0) {  // rounding pushed r to the very end: the last kept token
        idx = cut.crossed ? nth_equal(p, V, cut.key, cut.rank, sm) : -1;
        if (idx < 0) idx = 0;
    }
    if (tid == 0) {
        out[row] = idx;
        if (kept_mass) kept_mass[row] = (float)Z;
    }
}

void sample_top_p(hipStream_t s, const float* x, int rows, int V, float temperature, float top_p, const float* u,
                  float* scratch, int64_t* out, float* kept_mass) {
    hipLaunchKernelGGL(k_sample_top_p, dim3(rows), dim3(kSampleThreads), 0, s, x, V, temperature, top_p, u, scratch,
                       out, kept_mass);
}

}  // namespace pgmi
