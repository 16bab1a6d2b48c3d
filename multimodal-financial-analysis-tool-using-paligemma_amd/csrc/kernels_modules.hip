// kernels_modules.hip -- the per-module entry points of the drop-in API (pgmi/modules.py) that the
// fused forwards never need: a rotary application on given cos/sin rows, and an attention that
// materialises the probability matrix and takes an additive mask.  They restate the reference
// module bodies op by op with its bf16 rounding points; they are not on the hot path (a module
// called on its own, or a layer with forward hooks), so they favour exactness over speed.
#include "common.h"
#include "launch.h"

namespace pgmi {

// apply_rotary_pos_emb for one tensor (modeling_gemma.py:187-199): x rows (rows, heads * hd),
// cos/sin rows (rows, hd) -- GemmaRotaryEmbedding.forward's output (:155-185), already in x's dtype.
//   out = bf16(bf16(x * cos) + bf16(rotate_half(x) * sin)),  rotate_half(x)[d] = -x[d + hd/2] | x[d - hd/2]
__global__ void k_rope_rows(const uint16_t* __restrict__ x, const uint16_t* __restrict__ cs,
                            const uint16_t* __restrict__ sn, long rows, int heads, int hd,
                            uint16_t* __restrict__ out) {
    const long per_row = (long)heads * hd;
    const long n = rows * per_row;
    const int half = hd / 2;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const long r = i / per_row;
        const int d = (int)(i % per_row) % hd;
        const long base = i - d;  // the head's first element
        const float a = bf2f(x[i]);
        const float rot = d < half ? -bf2f(x[base + d + half]) : bf2f(x[base + d - half]);
        const float c = bf2f(cs[r * hd + d]), s = bf2f(sn[r * hd + d]);
        out[i] = f2bf(rbf(a * c) + rbf(rot * s));
    }
}

void rope_rows(hipStream_t s, const uint16_t* x, const uint16_t* cs, const uint16_t* sn, long rows, int heads,
               int hd, uint16_t* out) {
    const long n = rows * heads * hd;
    long blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_rope_rows, dim3((unsigned)blocks), dim3(256), 0, s, x, cs, sn, rows, heads, hd, out);
}

// Reference-order attention for one (query row, head, batch) per workgroup
// (modeling_siglip.py:116-131, modeling_gemma.py:262-277):
//   s = bf16(q . k)                     torch.matmul in bf16 (fp32 accumulation, one rounding)
//   s = bf16(s * scale) | bf16(s / scale)     "* self.scale" (SigLIP) or "/ math.sqrt(head_dim)" (Gemma)
//   s = bf16(s + mask)   (bf16 mask)  |  s + mask in fp32 (fp32 mask: torch promotes)
//   p = bf16(softmax_fp32(s))           softmax(dim=-1, dtype=float32).to(bf16)   -> probs (optional)
//   o = bf16(p . v)                     torch.matmul in bf16
// LDS: the row's scores (Lk floats) + q (hd floats) + the P.V reduction (256 floats).
__global__ void __launch_bounds__(256) k_attn_exact(ModAttnArgs a) {
    extern __shared__ float smf[];
    float* sc = smf;                  // [Lk]
    float* qs = smf + a.Lk;           // [hd]
    float* red = qs + a.hd;           // [256]
    const int i = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
    const int tid = threadIdx.x;
    const int hk = h / (a.H / a.Hkv);  // repeat_kv: query head h reads KV head h / n_rep
    const uint16_t* q = a.q + (long)b * a.Lq * a.H * a.hd + ((long)i * a.H + h) * a.hd;
    for (int d = tid; d < a.hd; d += 256) qs[d] = bf2f(q[d]);
    __syncthreads();
    const uint16_t* kb = a.k + (long)b * a.kv_b_stride + (long)hk * a.kv_h_stride;
    const uint16_t* vb = a.v + (long)b * a.kv_b_stride + (long)hk * a.kv_h_stride;
    float lmax = -INFINITY;
    for (int j = tid; j < a.Lk; j += 256) {
        const uint16_t* kr = kb + (long)j * a.kv_row_stride;
        float acc = 0.f;
        for (int d = 0; d < a.hd; ++d) acc += qs[d] * bf2f(kr[d]);
        float s = rbf(acc);
        s = a.scale_div ? rbf(s / a.scale) : rbf(s * a.scale);
        if (a.mask) {
            const long mo = (long)b * a.m_b_stride + (long)h * a.m_h_stride + (long)i * a.m_q_stride + j;
            s = a.mask_f32 ? s + reinterpret_cast<const float*>(a.mask)[mo]
                           : rbf(s + bf2f(reinterpret_cast<const uint16_t*>(a.mask)[mo]));
        }
        sc[j] = s;
        lmax = fmaxf(lmax, s);
    }
    // row max
    red[tid] = lmax;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (tid < o) red[tid] = fmaxf(red[tid], red[tid + o]);
        __syncthreads();
    }
    const float m = red[0];
    __syncthreads();
    float lsum = 0.f;
    for (int j = tid; j < a.Lk; j += 256) {
        const float e = m == -INFINITY ? 0.f : expf(sc[j] - m);
        sc[j] = e;
        lsum += e;
    }
    red[tid] = lsum;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (tid < o) red[tid] += red[tid + o];
        __syncthreads();
    }
    const float l = red[0];
    __syncthreads();
    uint16_t* pr = a.probs ? a.probs + (((long)b * a.H + h) * a.Lq + i) * a.Lk : nullptr;
    for (int j = tid; j < a.Lk; j += 256) {
        const uint16_t pb = f2bf(sc[j] / l);
        sc[j] = bf2f(pb);
        if (pr) pr[j] = pb;
    }
    __syncthreads();
    // P.V (hd <= 256): thread (g, d) sums keys j = g, g + G, ... for column d, G = 256 / hd groups;
    // the G partial sums meet in LDS in a fixed order
    const int G = 256 / a.hd;
    const int g = tid / a.hd, d = tid % a.hd;
    float acc = 0.f;
    if (g < G)
        for (int j = g; j < a.Lk; j += G) acc += sc[j] * bf2f(vb[(long)j * a.kv_row_stride + d]);
    red[tid] = acc;
    __syncthreads();
    if (tid < a.hd) {
        float t = 0.f;
        for (int gg = 0; gg < G; ++gg) t += red[gg * a.hd + tid];
        a.o[(long)b * a.Lq * a.H * a.hd + ((long)i * a.H + h) * a.hd + tid] = f2bf(t);
    }
}

size_t attention_exact_lds(int Lk, int hd) { return (size_t)(Lk + hd + 256) * sizeof(float); }

void attention_exact(hipStream_t s, const ModAttnArgs& a) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_attn_exact),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
    }
    dim3 grid(a.Lq, a.H, a.B);
    hipLaunchKernelGGL(k_attn_exact, grid, dim3(256), attention_exact_lds(a.Lk, a.hd), s, a);
}

}  // namespace pgmi
