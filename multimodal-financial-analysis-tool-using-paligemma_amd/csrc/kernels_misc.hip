// kernels_misc.hip -- memory-bound helpers of the PaliGemma path (gfx950).
//
// Each kernel restates one reference op with its bf16 rounding points:
//   rmsnorm        GemmaRMSNorm            modeling_gemma.py:107-120
//   layernorm      nn.LayerNorm (SigLIP)   modeling_siglip.py:175,177,234
//   embed/merge    Embedding + merge + x sqrt(hidden)   modeling_gemma.py:565,468-537,367-368
//   rope_kv_append rotary + KVCache.update modeling_gemma.py:143-199,259, :10-36
//   patchify       Conv2d(k=s=14) as im2col (+ pixel cast to bf16)  modeling_siglip.py:45-51,67; modeling_gemma.py:570
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "common.h"
#include "launch.h"

namespace pgmi {

// ---------------------------------------------------------------- block reductions
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) red[w] = v;
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) t += red[i];
    return t;
}

// ---------------------------------------------------------------- RMSNorm (rows x D), 256 threads/row
__global__ void __launch_bounds__(256) k_rmsnorm(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                 float eps, uint16_t* __restrict__ out, int D) {
    __shared__ float red[4];
    const long row = blockIdx.x;
    const uint16_t* xr = x + row * D;
    float ss = 0.f;
    for (int c = threadIdx.x * 8; c < D; c += 256 * 8) {
        uint4 v = ldg16(xr + c);
        const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
        for (int j = 0; j < 8; ++j) { float f = bf2f(e[j]); ss += f * f; }
    }
    ss = block_sum<256>(ss, red);
    const float r = 1.0f / sqrtf(ss / (float)D + eps);
    for (int c = threadIdx.x * 8; c < D; c += 256 * 8) {
        uint4 v = ldg16(xr + c), wv = ldg16(w + c);
        const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
        const uint16_t* we = reinterpret_cast<const uint16_t*>(&wv);
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o.v[j] = f2bf((bf2f(e[j]) * r) * (1.0f + bf2f(we[j])));
        *reinterpret_cast<u16x8*>(out + row * D + c) = o;
    }
}

void rmsnorm(hipStream_t s, const uint16_t* x, const uint16_t* w, float eps, uint16_t* out, int rows, int D) {
    hipLaunchKernelGGL(k_rmsnorm, dim3(rows), dim3(256), 0, s, x, w, eps, out, D);
}

// ---------------------------------------------------------------- LayerNorm (rows x D), fp32 stats
__global__ void __launch_bounds__(256) k_layernorm(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                   const uint16_t* __restrict__ b, float eps,
                                                   uint16_t* __restrict__ out, int D) {
    __shared__ float red[4];
    const long row = blockIdx.x;
    const uint16_t* xr = x + row * D;
    float vals[16];
    float sum = 0.f;
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const int c = (threadIdx.x + it * 256) * 8;
        if (c < D) {
            uint4 v = ldg16(xr + c);
            const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
            for (int j = 0; j < 8; ++j) { float f = bf2f(e[j]); vals[it * 8 + j] = f; sum += f; }
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) vals[it * 8 + j] = 0.f;
        }
    }
    const float mu = block_sum<256>(sum, red) / (float)D;
    float sq = 0.f;
#pragma unroll
    for (int it = 0; it < 2; ++it)
        if ((threadIdx.x + it * 256) * 8 < D)
#pragma unroll
            for (int j = 0; j < 8; ++j) { float d = vals[it * 8 + j] - mu; sq += d * d; }
    const float var = block_sum<256>(sq, red) / (float)D;
    const float rstd = 1.0f / sqrtf(var + eps);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const int c = (threadIdx.x + it * 256) * 8;
        if (c >= D) continue;
        uint4 wv = ldg16(w + c), bv = ldg16(b + c);
        const uint16_t* we = reinterpret_cast<const uint16_t*>(&wv);
        const uint16_t* be = reinterpret_cast<const uint16_t*>(&bv);
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o.v[j] = f2bf((vals[it * 8 + j] - mu) * rstd * bf2f(we[j]) + bf2f(be[j]));
        *reinterpret_cast<u16x8*>(out + row * D + c) = o;
    }
}

void layernorm(hipStream_t s, const uint16_t* x, const uint16_t* w, const uint16_t* b, float eps, uint16_t* out,
               int rows, int D) {
    // D <= 2 * 256 * 8 (vals[] holds two 8-wide chunks per thread)
    hipLaunchKernelGGL(k_layernorm, dim3(rows), dim3(256), 0, s, x, w, b, eps, out, D);
}

// ---------------------------------------------------------------- embedding (decode path)
// final_embedding for a text/pad token (modeling_gemma.py:486-500) times the bf16
// normalizer (modeling_gemma.py:367-368): bf16(E[id] * 45.25), pad rows -> 0.
__global__ void k_embed_rows(const int64_t* __restrict__ ids, const uint16_t* __restrict__ E, int D,
                             float normalizer, int64_t pad_id, uint16_t* __restrict__ out) {
    const long r = blockIdx.x;
    const int64_t id = ids[r];
    for (int c = threadIdx.x * 8; c < D; c += blockDim.x * 8) {
        u16x8 o;
        if (id == pad_id) {
#pragma unroll
            for (int j = 0; j < 8; ++j) o.v[j] = 0;
        } else {
            uint4 v = ldg16(E + id * (long)D + c);
            const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
            for (int j = 0; j < 8; ++j) o.v[j] = f2bf(bf2f(e[j]) * normalizer);
        }
        *reinterpret_cast<u16x8*>(out + r * D + c) = o;
    }
}

void embed_rows(hipStream_t s, const int64_t* ids, int rows, const uint16_t* E, int D, float normalizer,
                int64_t pad_id, uint16_t* out) {
    hipLaunchKernelGGL(k_embed_rows, dim3(rows), dim3(256), 0, s, ids, E, D, normalizer, pad_id, out);
}

// ---------------------------------------------------------------- merge (prefill)
// masked_scatter order: the k-th <image> token (row-major over B x L) takes image row k.
__global__ void __launch_bounds__(1024) k_image_scan(const int64_t* __restrict__ ids, int n, int64_t image_token,
                                                     int* __restrict__ idx) {
    __shared__ int warp_tot[16];
    __shared__ int carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int base = 0; base < n; base += 1024) {
        const int i = base + threadIdx.x;
        const int f = (i < n && ids[i] == image_token) ? 1 : 0;
        // inclusive scan within the wave
        int v = f;
        const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            int t = __shfl_up(v, o, 64);
            if (l >= o) v += t;
        }
        if (l == 63) warp_tot[w] = v;
        __syncthreads();
        int pre = carry;
        for (int k = 0; k < w; ++k) pre += warp_tot[k];
        if (i < n) idx[i] = f ? (pre + v - 1) : -1;
        __syncthreads();
        if (threadIdx.x == 1023) carry = pre + v;
        __syncthreads();
    }
}

__global__ void k_merge(const int64_t* __restrict__ ids, const int* __restrict__ img_idx,
                        const uint16_t* __restrict__ E, int D, const uint16_t* __restrict__ img, int n_img_rows,
                        int64_t pad_id, float sqrt_h, float normalizer,
                        const uint16_t* __restrict__ embeds_in, uint16_t* __restrict__ out) {
    const long r = blockIdx.x;
    const int64_t id = ids[r];
    const int k = img_idx[r];
    for (int c = threadIdx.x * 8; c < D; c += blockDim.x * 8) {
        u16x8 o;
        if (k >= 0) {
            if (k < n_img_rows) {
                uint4 v = ldg16(img + (long)k * D + c);
                const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
                // image_features / sqrt(hidden) (true division, :481), then x 45.25 (:368)
#pragma unroll
                for (int j = 0; j < 8; ++j) o.v[j] = f2bf(rbf(bf2f(e[j]) / sqrt_h) * normalizer);
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) o.v[j] = 0;
            }
        } else if (id == pad_id) {
#pragma unroll
            for (int j = 0; j < 8; ++j) o.v[j] = 0;
        } else {
            uint4 v = embeds_in ? ldg16(embeds_in + r * D + c) : ldg16(E + id * (long)D + c);
            const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
            for (int j = 0; j < 8; ++j) o.v[j] = f2bf(bf2f(e[j]) * normalizer);
        }
        *reinterpret_cast<u16x8*>(out + r * D + c) = o;
    }
}

void merge_embed(hipStream_t s, const int64_t* ids, int B, int L, const uint16_t* E, int D, const uint16_t* img,
                 int n_img_rows, int64_t image_token, int64_t pad_id, float sqrt_h, float normalizer,
                 const uint16_t* embeds_in, int* scan_buf, uint16_t* out) {
    const int n = B * L;
    hipLaunchKernelGGL(k_image_scan, dim3(1), dim3(1024), 0, s, ids, n, image_token, scan_buf);
    hipLaunchKernelGGL(k_merge, dim3(n), dim3(256), 0, s, ids, scan_buf, E, D, img, n_img_rows, pad_id, sqrt_h,
                       normalizer, embeds_in, out);
}

__global__ void k_scale(const uint16_t* __restrict__ x, long n, float a, uint16_t* __restrict__ out) {
    for (long i = (blockIdx.x * (long)blockDim.x + threadIdx.x) * 8; i < n; i += (long)gridDim.x * blockDim.x * 8) {
        uint4 v = ldg16(x + i);
        const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o.v[j] = f2bf(bf2f(e[j]) * a);
        *reinterpret_cast<u16x8*>(out + i) = o;
    }
}

__global__ void k_add(const uint16_t* __restrict__ x, const uint16_t* __restrict__ y, long n, uint16_t* __restrict__ out) {
    for (long i = (blockIdx.x * (long)blockDim.x + threadIdx.x) * 8; i < n; i += (long)gridDim.x * blockDim.x * 8) {
        const uint4 u = ldg16(x + i), v = ldg16(y + i);
        const uint16_t* e = reinterpret_cast<const uint16_t*>(&u);
        const uint16_t* f = reinterpret_cast<const uint16_t*>(&v);
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o.v[j] = f2bf(bf2f(e[j]) + bf2f(f[j]));
        *reinterpret_cast<u16x8*>(out + i) = o;
    }
}

void add_rows(hipStream_t s, const uint16_t* x, const uint16_t* y, long n, uint16_t* out) {
    long blocks = (n / 8 + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_add, dim3((unsigned)blocks), dim3(256), 0, s, x, y, n, out);
}

void scale_rows(hipStream_t s, const uint16_t* x, long n, float a, uint16_t* out) {
    long blocks = (n / 8 + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_scale, dim3((unsigned)blocks), dim3(256), 0, s, x, n, a, out);
}

// ---------------------------------------------------------------- RoPE + KV append (prefill)
// qkv rows: [q (nh*256) | k (nkv*256) | v (nkv*256)].  apply_rotary_pos_emb rounds three
// times (q*cos, rotate_half(q)*sin, sum), modeling_gemma.py:197-198.
template <bool PART>
__global__ void k_rope_kv(const uint16_t* __restrict__ qkv, const float* __restrict__ ws, int split, long slab,
                          int L, int nh, int nkv, const int64_t* __restrict__ pos,
                          const uint16_t* __restrict__ cosT, const uint16_t* __restrict__ sinT, int max_pos,
                          uint16_t* __restrict__ q_out, uint16_t* __restrict__ kc, uint16_t* __restrict__ vc,
                          long kv_b_stride, int kv_start) {
    const long r = blockIdx.x;  // b*L + l
    const int b = (int)(r / L), l = (int)(r % L);
    long p = pos[r];
    if (p < 0) p = 0;
    if (p > max_pos - 1) p = max_pos - 1;
    const int ncol = (nh + 2 * nkv) * 256;
    auto val = [&](int c) -> float {  // projection output, rounded to bf16 as the reference's q/k/v_proj
        if constexpr (PART) {
            float a = 0.f;
            for (int z = 0; z < split; ++z) a += ws[z * slab + r * ncol + c];
            return rbf(a);
        } else {
            return bf2f(qkv[r * ncol + c]);
        }
    };
    // pairs (d, d+128) of every rotated head: nh + nkv heads x 128 pairs.  A thread's pairs (at most
    // kRopeIt; rows past the end re-read the last pair and are not stored), their cos/sin and its V
    // column are all loaded before the first is used: one memory round trip per row
    constexpr int kRopeIt = 5;  // ceil((8 + 1) * 128 / 256) at PaliGemma's 8 q heads + 1 kv head
    const int npair = (nh + nkv) * 128;
    float av[kRopeIt], bv[kRopeIt], cv[kRopeIt], sv[kRopeIt];
#pragma unroll
    for (int i = 0; i < kRopeIt; ++i) {
        int u = threadIdx.x + i * blockDim.x;
        u = u < npair ? u : npair - 1;
        const int hh = u >> 7, d = u & 127;
        av[i] = val(hh * 256 + d);
        bv[i] = val(hh * 256 + d + 128);
        cv[i] = bf2f(cosT[p * 128 + d]);
        sv[i] = bf2f(sinT[p * 128 + d]);
    }
    const int vcols = nkv * 256;
    const int vu = (int)threadIdx.x < vcols ? (int)threadIdx.x : vcols - 1;
    const float vval = val((nh + nkv) * 256 + vu);
#pragma unroll
    for (int i = 0; i < kRopeIt; ++i) {
        const int u = threadIdx.x + i * blockDim.x;
        if (u >= npair) break;
        const int hh = u >> 7, d = u & 127;
        const float a = av[i], bb = bv[i], c = cv[i], sn = sv[i];
        const uint16_t oa = f2bf(rbf(a * c) + rbf(-bb * sn));
        const uint16_t ob = f2bf(rbf(bb * c) + rbf(a * sn));
        if (hh < nh) {
            q_out[r * (nh * 256) + hh * 256 + d] = oa;
            q_out[r * (nh * 256) + hh * 256 + d + 128] = ob;
        } else {
            const int kh = hh - nh;
            uint16_t* dst = kc + b * kv_b_stride + (long)(kv_start + l) * (nkv * 256) + kh * 256;
            dst[d] = oa;
            dst[d + 128] = ob;
        }
    }
    if ((int)threadIdx.x < vcols) vc[b * kv_b_stride + (long)(kv_start + l) * (nkv * 256) + threadIdx.x] = f2bf(vval);
    // (shapes beyond the unrolled coverage: the remaining pairs and V columns, plain loop)
    for (int u = threadIdx.x + kRopeIt * blockDim.x; u < npair; u += blockDim.x) {
        const int hh = u >> 7, d = u & 127;
        const float a = val(hh * 256 + d), bb = val(hh * 256 + d + 128);
        const float c = bf2f(cosT[p * 128 + d]), sn = bf2f(sinT[p * 128 + d]);
        const uint16_t oa = f2bf(rbf(a * c) + rbf(-bb * sn));
        const uint16_t ob = f2bf(rbf(bb * c) + rbf(a * sn));
        if (hh < nh) {
            q_out[r * (nh * 256) + hh * 256 + d] = oa;
            q_out[r * (nh * 256) + hh * 256 + d + 128] = ob;
        } else {
            uint16_t* dst = kc + b * kv_b_stride + (long)(kv_start + l) * (nkv * 256) + (hh - nh) * 256;
            dst[d] = oa;
            dst[d + 128] = ob;
        }
    }
    for (int u = threadIdx.x + blockDim.x; u < vcols; u += blockDim.x)
        vc[b * kv_b_stride + (long)(kv_start + l) * (nkv * 256) + u] = f2bf(val((nh + nkv) * 256 + u));
}

void rope_kv_append(hipStream_t s, const uint16_t* qkv, const float* ws, int split, int B, int L, int nh, int nkv,
                    const int64_t* pos, const uint16_t* cosT, const uint16_t* sinT, int max_pos, uint16_t* q_out,
                    uint16_t* kcache, uint16_t* vcache, long kv_b_stride, int kv_start) {
    const long slab = (long)B * L * (nh + 2 * nkv) * 256;
    if (split > 1)
        hipLaunchKernelGGL(k_rope_kv<true>, dim3(B * L), dim3(256), 0, s, qkv, ws, split, slab, L, nh, nkv, pos, cosT,
                           sinT, max_pos, q_out, kcache, vcache, kv_b_stride, kv_start);
    else
        hipLaunchKernelGGL(k_rope_kv<false>, dim3(B * L), dim3(256), 0, s, qkv, ws, split, slab, L, nh, nkv, pos, cosT,
                           sinT, max_pos, q_out, kcache, vcache, kv_b_stride, kv_start);
}

// ---------------------------------------------------------------- split-K reduce + residual + norm
// Row per workgroup, 256 threads x 8 columns x 2 chunks (D <= 4096).  Every global read of the
// row -- residual h, the split-K partial slabs (up to kMaxSplit, clamped to the live ones and
// weighted 0 past `split`), bias, and the norm's weight / bias -- is issued before the first is
// consumed: one memory round trip per row instead of one per slab plus one after the reductions.
constexpr int kMaxSplit = 16;
template <bool LN, int MS>
__global__ void __launch_bounds__(256) k_splitk_res_norm(const float* __restrict__ ws, int split, long slab,
                                                         const uint16_t* __restrict__ bias, uint16_t* __restrict__ h,
                                                         const uint16_t* __restrict__ w, const uint16_t* __restrict__ b,
                                                         float eps, uint16_t* __restrict__ out, int D) {
    __shared__ float red[4];
    const long row = blockIdx.x;
    float v[16];
    uint4 wv[2], bnv[2];
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const int c = (threadIdx.x + it * 256) * 8;
        if (c >= D) {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[it * 8 + j] = 0.f;
            continue;
        }
        const uint4 hv = ldg16(h + row * D + c);
        wv[it] = ldg16(w + c);
        if constexpr (LN) bnv[it] = ldg16(b + c);
        const uint16_t* he = reinterpret_cast<const uint16_t*>(&hv);
        if (split > 1) {
            const uint4 bv = ldg16(bias ? bias + c : h + row * D + c);  // (h: any valid address, unused)
            f32x4 p0[MS], p1[MS];
#pragma unroll
            for (int z = 0; z < MS; ++z) {
                const long zo = (long)(z < split ? z : 0) * slab + row * D + c;
                p0[z] = *reinterpret_cast<const f32x4*>(ws + zo);
                p1[z] = *reinterpret_cast<const f32x4*>(ws + zo + 4);
            }
            float a[8];
#pragma unroll
            for (int j = 0; j < 4; ++j) { a[j] = p0[0][j]; a[4 + j] = p1[0][j]; }
#pragma unroll
            for (int z = 1; z < MS; ++z) {
                // slabs in a fixed order; past `split` the sum is kept as is (a select after the
                // loads, not a multiply by 0: Inf * 0 would turn the sum into NaN, -0 + 0 into +0)
                const bool live = z < split;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    a[j] = live ? a[j] + p0[z][j] : a[j];
                    a[4 + j] = live ? a[4 + j] + p1[z][j] : a[4 + j];
                }
            }
            const uint16_t* be = reinterpret_cast<const uint16_t*>(&bv);
            u16x8 o;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float t = bias ? rbf(a[j] + bf2f(be[j])) : rbf(a[j]);
                o.v[j] = f2bf(t + bf2f(he[j]));
                v[it * 8 + j] = bf2f(o.v[j]);
            }
            *reinterpret_cast<u16x8*>(h + row * D + c) = o;
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[it * 8 + j] = bf2f(he[j]);
        }
    }
    float r, mu = 0.f;
    if constexpr (LN) {
        float sum = 0.f;
#pragma unroll
        for (int j = 0; j < 16; ++j) sum += v[j];
        mu = block_sum<256>(sum, red) / (float)D;
        float sq = 0.f;
#pragma unroll
        for (int it = 0; it < 2; ++it)
            if ((threadIdx.x + it * 256) * 8 < D)
#pragma unroll
                for (int j = 0; j < 8; ++j) { const float d = v[it * 8 + j] - mu; sq += d * d; }
        r = 1.0f / sqrtf(block_sum<256>(sq, red) / (float)D + eps);
    } else {
        float ss = 0.f;
#pragma unroll
        for (int j = 0; j < 16; ++j) ss += v[j] * v[j];
        r = 1.0f / sqrtf(block_sum<256>(ss, red) / (float)D + eps);
    }
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const int c = (threadIdx.x + it * 256) * 8;
        if (c >= D) continue;
        const uint16_t* we = reinterpret_cast<const uint16_t*>(&wv[it]);
        u16x8 o;
        if constexpr (LN) {
            const uint16_t* be = reinterpret_cast<const uint16_t*>(&bnv[it]);
#pragma unroll
            for (int j = 0; j < 8; ++j) o.v[j] = f2bf((v[it * 8 + j] - mu) * r * bf2f(we[j]) + bf2f(be[j]));
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) o.v[j] = f2bf((v[it * 8 + j] * r) * (1.0f + bf2f(we[j])));
        }
        *reinterpret_cast<u16x8*>(out + row * D + c) = o;
    }
}

void splitk_res_norm(hipStream_t s, const float* ws, int split, const uint16_t* bias, uint16_t* h, const uint16_t* w,
                     const uint16_t* b, float eps, uint16_t* out, int rows, int D) {
    const long slab = (long)rows * D;
    if (split > kMaxSplit) {
        fprintf(stderr, "pgmi: splitk_res_norm: split %d > %d\n", split, kMaxSplit);
        std::abort();
    }
    // slab loads issued up front: as many register slots as the split needs (4, 8 or 16)
#define SRN_(ln, ms) hipLaunchKernelGGL((k_splitk_res_norm<ln, ms>), dim3(rows), dim3(256), 0, s, ws, split, slab, bias, h, \
                                        w, b, eps, out, D)
    if (b) {
        if (split <= 4) SRN_(true, 4);
        else if (split <= 8) SRN_(true, 8);
        else SRN_(true, 16);
    } else {
        if (split <= 4) SRN_(false, 4);
        else if (split <= 8) SRN_(false, 8);
        else SRN_(false, 16);
    }
#undef SRN_
}

// ---------------------------------------------------------------- patch im2col
// out[(b*gh + i)*gw + j][c*P*P + kh*P + kw] = bf16(px[b][c][i*P+kh][j*P+kw]); zero pad to Kpad
__global__ void k_patchify(const void* __restrict__ px, int is_f32, int C, int H, int W, int P, int Kpad,
                           uint16_t* __restrict__ out) {
    const int gw = W / P, gh = H / P;
    const long row = blockIdx.x;  // (b, i, j)
    const int b = (int)(row / (gh * gw)), ij = (int)(row % (gh * gw));
    const int i = ij / gw, j = ij % gw;
    for (int col = threadIdx.x; col < Kpad; col += blockDim.x) {
        uint16_t v = 0;
        if (col < C * P * P) {
            const int c = col / (P * P), kh = (col / P) % P, kw = col % P;
            const long off = (((long)b * C + c) * H + (i * P + kh)) * W + (j * P + kw);
            v = is_f32 ? f2bf(reinterpret_cast<const float*>(px)[off]) : reinterpret_cast<const uint16_t*>(px)[off];
        }
        out[row * Kpad + col] = v;
    }
}

void patchify(hipStream_t s, const void* px, int px_is_f32, int B, int C, int H, int W, int P, int Kpad,
              uint16_t* out) {
    const int rows = B * (H / P) * (W / P);
    hipLaunchKernelGGL(k_patchify, dim3(rows), dim3(256), 0, s, px, px_is_f32, C, H, W, P, Kpad, out);
}

__global__ void k_pad_rows(const uint16_t* __restrict__ src, int K, int Kpad, uint16_t* __restrict__ dst) {
    const long r = blockIdx.x;
    for (int c = threadIdx.x; c < Kpad; c += blockDim.x) dst[r * Kpad + c] = c < K ? src[r * K + c] : 0;
}

void pad_rows(hipStream_t s, const uint16_t* src, int rows, int K, int Kpad, uint16_t* dst) {
    hipLaunchKernelGGL(k_pad_rows, dim3(rows), dim3(256), 0, s, src, K, Kpad, dst);
}

// ---------------------------------------------------------------- argmax (first max, torch semantics)
__global__ void k_argmax_finish(const float* __restrict__ pmax, const int* __restrict__ pidx, int nparts,
                                int64_t* __restrict__ out, StepState* adv, int64_t* __restrict__ hist) {
    const int b = blockIdx.x;
    // the decode step's last kernel: every reader of the step state is done, so advance it to
    // the next step's (kv_len + 1, position + 1); pgmi_decode then skips its host-side set
    if (adv && b == 0 && threadIdx.x == 0) {
        adv->kv_len += 1;
        adv->position += 1;
    }
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for (int i = threadIdx.x; i < nparts; i += blockDim.x) {
        const float v = pmax[(long)b * nparts + i];
        const int ix = pidx[(long)b * nparts + i];
        if (v > best || (v == best && ix < bi)) { best = v; bi = ix; }
    }
    __shared__ float sv[256];
    __shared__ int si[256];
    sv[threadIdx.x] = best;
    si[threadIdx.x] = bi;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) {
            const float v = sv[threadIdx.x + o];
            const int ix = si[threadIdx.x + o];
            if (v > sv[threadIdx.x] || (v == sv[threadIdx.x] && ix < si[threadIdx.x])) {
                sv[threadIdx.x] = v;
                si[threadIdx.x] = ix;
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out[b] = si[0];
        if (hist) hist[b] = si[0];
    }
}

void argmax_finish(hipStream_t s, int B, const float* pmax, const int* pidx, int nparts, int64_t* out,
                   StepState* adv, int64_t* hist) {
    hipLaunchKernelGGL(k_argmax_finish, dim3(B), dim3(256), 0, s, pmax, pidx, nparts, out, adv, hist);
}

// ---------------------------------------------------------------- stop tokens of the batched loop
// inference.py:70-71 per row: the reference appends the stop token, then breaks.  A row that
// finished at an earlier step emits `pad` from then on; a row whose token is `eos` is marked
// finished (its eos is kept).  One workgroup; n_alive = rows still running after this step.
__global__ void k_eos_update(int64_t* __restrict__ next, int* __restrict__ finished, int B, int64_t eos,
                             int64_t pad, int* __restrict__ n_alive) {
    __shared__ int alive;
    if (threadIdx.x == 0) alive = 0;
    __syncthreads();
    int mine = 0;
    for (int b = threadIdx.x; b < B; b += blockDim.x) {
        if (finished[b]) {
            next[b] = pad;
        } else if (next[b] == eos) {
            finished[b] = 1;
        } else {
            ++mine;
        }
    }
    if (mine) atomicAdd(&alive, mine);
    __syncthreads();
    if (threadIdx.x == 0 && n_alive) *n_alive = alive;
}

void eos_update(hipStream_t s, int64_t* next, int* finished, int B, int64_t eos, int64_t pad, int* n_alive) {
    hipLaunchKernelGGL(k_eos_update, dim3(1), dim3(256), 0, s, next, finished, B, eos, pad, n_alive);
}

// torch.argmax over each row of x [rows][V] (first max wins).  Stage 1: a (nb x rows) grid, each
// block scans a contiguous slice of a row with 16-B loads and leaves (max, first index); stage 2
// (k_argmax_finish) reduces the nb partials of each row.  nb == 1 writes the answer directly.
__device__ __forceinline__ void amax_take(float v, int i, float& best, int& bi) {
    if (v > best || (v == best && i < bi)) { best = v; bi = i; }
}

__global__ void k_argmax_part(const float* __restrict__ x, int V, int slice, float* __restrict__ pmax,
                              int* __restrict__ pidx, int64_t* __restrict__ out) {
    const int row = blockIdx.y, nb = gridDim.x;
    const float* xr = x + (long)row * V;
    const int lo = blockIdx.x * slice, hi = min(V, lo + slice);
    float best = -INFINITY;
    int bi = 0x7fffffff;
    const bool vec = ((V & 3) == 0) && ((reinterpret_cast<uintptr_t>(x) & 15) == 0);
    if (vec) {
        for (int i = lo + 4 * threadIdx.x; i < hi; i += 4 * blockDim.x) {
            const float4 v = *reinterpret_cast<const float4*>(xr + i);
            amax_take(v.x, i, best, bi);
            amax_take(v.y, i + 1, best, bi);
            amax_take(v.z, i + 2, best, bi);
            amax_take(v.w, i + 3, best, bi);
        }
    } else {
        for (int i = lo + threadIdx.x; i < hi; i += blockDim.x) amax_take(xr[i], i, best, bi);
    }
    for (int o = 32; o > 0; o >>= 1) {
        const float v = __shfl_xor(best, o, 64);
        const int ix = __shfl_xor(bi, o, 64);
        amax_take(v, ix, best, bi);
    }
    __shared__ float sv[4];
    __shared__ int si[4];
    if ((threadIdx.x & 63) == 0) {
        sv[threadIdx.x >> 6] = best;
        si[threadIdx.x >> 6] = bi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) amax_take(sv[w], si[w], best, bi);
        if (nb == 1) {
            out[row] = bi;
        } else {
            pmax[(long)row * nb + blockIdx.x] = best;
            pidx[(long)row * nb + blockIdx.x] = bi;
        }
    }
}

int argmax_scratch_parts() { return 1024; }

void argmax_rows(hipStream_t s, const float* x, int rows, int V, float* pmax, int* pidx, int64_t* out) {
    int nb = rows >= argmax_scratch_parts() ? 1 : argmax_scratch_parts() / rows;
    nb = std::max(1, std::min(nb, std::min(128, (V + 2047) / 2048)));
    const int slice = ((V + nb - 1) / nb + 3) & ~3;
    nb = (V + slice - 1) / slice;
    hipLaunchKernelGGL(k_argmax_part, dim3(nb, rows), dim3(256), 0, s, x, V, slice, pmax, pidx, out);
    if (nb > 1) hipLaunchKernelGGL(k_argmax_finish, dim3(rows), dim3(256), 0, s, pmax, pidx, nb, out, nullptr, nullptr);
}

// ---------------------------------------------------------------- synthetic weights (bench / tests)
// Same recipe as oracle/wgen.c: u = splitmix64(key + i), v = ((u>>40) - 2^23) * 2^-23,
// w = bf16(offset + v*scale) with the two f32 roundings kept separate.
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

__global__ void k_fill_synth(uint16_t* __restrict__ dst, long n, uint64_t key, float scale, float offset) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const uint64_t u = splitmix64(key + (uint64_t)i);
        const float v = (float)((int32_t)(u >> 40) - (1 << 23)) * (1.0f / 8388608.0f);
        const float t = __fmul_rn(v, scale);
        dst[i] = f2bf(__fadd_rn(offset, t));
    }
}

void fill_synthetic(hipStream_t s, uint16_t* dst, long n, uint64_t key, float scale, float offset) {
    long blocks = (n + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(k_fill_synth, dim3((unsigned)blocks), dim3(256), 0, s, dst, n, key, scale, offset);
}

__global__ void k_set_step(StepState* st, int kv_len, int position) {
    st->kv_len = kv_len;
    st->position = position;
}

void set_step(hipStream_t s, StepState* st, int kv_len, int position) {
    hipLaunchKernelGGL(k_set_step, dim3(1), dim3(1), 0, s, st, kv_len, position);
}

// position = round(pos[0]) (modeling_gemma.py:526's cumsum, float when the mask grew by a float column)
__global__ void k_set_step_dev(StepState* st, int kv_len, const void* pos, int dtype) {
    double v;
    if (dtype == 2) v = (double)*reinterpret_cast<const float*>(pos);
    else if (dtype == 12) v = *reinterpret_cast<const double*>(pos);
    else if (dtype == 11) v = (double)*reinterpret_cast<const int32_t*>(pos);
    else if (dtype == 0) v = (double)bf2f(*reinterpret_cast<const uint16_t*>(pos));
    else v = (double)*reinterpret_cast<const int64_t*>(pos);
    st->kv_len = kv_len;
    st->position = (int)rint(v);
}

void set_step_dev(hipStream_t s, StepState* st, int kv_len, const void* pos, int dtype) {
    hipLaunchKernelGGL(k_set_step_dev, dim3(1), dim3(1), 0, s, st, kv_len, pos, dtype);
}

__global__ void k_stage_mask(const void* src, int dtype, long b_stride, int n, float* dst, int ld) {
    const int b = blockIdx.y;
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
        const long o = (long)b * b_stride + j;
        dst[(long)b * ld + j] = dtype == 2 ? reinterpret_cast<const float*>(src)[o]
                                           : bf2f(reinterpret_cast<const uint16_t*>(src)[o]);
    }
}

void stage_mask(hipStream_t s, const void* src, int dtype, int B, long b_stride, int n, float* dst, int ld) {
    int bx = (n + 255) / 256;
    if (bx > 64) bx = 64;
    if (bx < 1) bx = 1;
    hipLaunchKernelGGL(k_stage_mask, dim3(bx, B), dim3(256), 0, s, src, dtype, b_stride, n, dst, ld);
}

}  // namespace pgmi
