// kernels_step.hip -- one KV-cached decode step (batch 1) as ONE dataflow launch.
//
// The step of decode_body (engine.hip) -- embed, 18 x [RMSNorm+qkv+RoPE+KV append, attention,
// combine+o_proj+residual, RMSNorm+gate/up+GeGLU, down+residual], final norm + lm_head, argmax
// (modeling_gemma.py:357-427 for one token, inference.py:63-68) -- is laid out as consecutive
// workgroup ranges of a single grid, one range per phase, in dependency order:
//
//   [embed:1] { [qkv:n_qkv] [attn:max_chunks] [o:n_o] [gate/up:n_gu] [down:n_dn] } x layers
//   [lm_head:n_lm] [argmax:1]
//
// Each workgroup runs exactly the body of the standalone kernel of its phase (gemv_body.h,
// attn_decode_body.h), but it first issues the loads of the bytes that do not depend on the
// step (its weight rows; for attention, the cache rows written before this step), THEN waits
// for the counter of the phase it consumes, then reads its inputs coherently (coh.h).  The
// in-order dispatcher places workgroups of later phases while earlier phases still compute,
// so the weight stream of e.g. gate/up runs under the latency-bound attention phases instead
// of after them, and no launch boundary separates the ~94 phases of the step.
#include "attn_decode_body.h"
#include "gemv_body.h"

namespace pgmi {

constexpr int kStepMaxLayers = 28;

struct StepLayerW {
    const uint16_t *ln1, *wqkv, *wo, *ln2, *wgu, *wdn;
    uint16_t *kc, *vc;
};

struct StepArgs {
    StepLayerW L[kStepMaxLayers];
    int layers;
    const int64_t* ids;
    const uint16_t* E;
    const uint16_t* fnorm;
    float normalizer, eps, scale;
    long long pad_id;
    const uint16_t *cosT, *sinT;
    int max_pos;
    const StepState* st;
    uint16_t *h, *q, *act;
    float* part;
    int max_chunks;
    long kvb;
    int nh, nkv, H, I, V;
    float* logits;
    float* pmax;
    int* pidx;
    int64_t* next;
    unsigned* sync;  // [0] embed, [1 + 5l + phase] per layer, [1 + 5 layers] lm_head; zero between launches
    unsigned* err;
    int n_qkv, n_attn, n_o, n_gu, n_dn, n_lm;
};

__global__ void __launch_bounds__(256) k_decode_step(StepArgs a) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[kAttnDecodeLds];
    const int tid = threadIdx.x;
    const int per = a.n_qkv + a.n_attn + a.n_o + a.n_gu + a.n_dn;
    int bid = blockIdx.x;
    if (bid == 0) {  // embedding row x bf16(sqrt(H)) (modeling_gemma.py:367-369), pad id -> zeros
        const int64_t id = a.ids[0];
        for (int c = tid * 8; c < a.H; c += 256 * 8) {
            u16x8 o;
            if (id == a.pad_id) {
#pragma unroll
                for (int j = 0; j < 8; ++j) o.v[j] = 0;
            } else {
                const uint4 v = ldg16(a.E + id * (long)a.H + c);
                const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
                for (int j = 0; j < 8; ++j) o.v[j] = f2bf(bf2f(e[j]) * a.normalizer);
            }
            st16_coh(a.h + c, *reinterpret_cast<const uint4*>(&o));
        }
        Dep d;
        d.arrive = a.sync;
        dep_arrive(d);
        return;
    }
    bid -= 1;
    if (bid < a.layers * per) {
        const int l = bid / per;
        int r = bid - l * per;
        const StepLayerW& w = a.L[l];
        unsigned* cnt = a.sync + 1 + 5 * l;
        Dep d;
        d.err = a.err;
        if (r < a.n_qkv) {
            d.wait = l == 0 ? a.sync : cnt - 1;  // embed, or the previous layer's down phase
            d.target = l == 0 ? 1u : (unsigned)a.n_dn;
            d.arrive = cnt + 0;
            GemvArgs g{};
            g.x = a.h; g.norm_w = w.ln1; g.eps = a.eps; g.W = w.wqkv; g.n_units = (a.nh + 2 * a.nkv) * 128;
            g.K = a.H; g.nb = 1; g.I = a.nh; g.out = a.q; g.cosT = a.cosT; g.sinT = a.sinT; g.max_pos = a.max_pos;
            g.st = a.st; g.kc = w.kc; g.vc = w.vc; g.kv_b_stride = a.kvb; g.nkv = a.nkv;
            gemv_block<1, 4, 1, GV_QKV, 1, true, true>(g, r, a.n_qkv, nullptr, d);
            return;
        }
        r -= a.n_qkv;
        if (r < a.n_attn) {
            d.wait = cnt + 0;
            d.target = (unsigned)a.n_qkv;
            d.arrive = cnt + 1;
            const int kvd = a.nkv * 256;
            AttnArgs at{};
            at.q = a.q; at.q_b_stride = (long)a.nh * 256; at.q_row_stride = a.nh * 256; at.q_head_stride = 256;
            at.k = w.kc; at.k_b_stride = a.kvb; at.k_row_stride = kvd; at.k_head_stride = 256;
            at.v = w.vc; at.v_b_stride = a.kvb; at.v_row_stride = kvd; at.v_head_stride = 256;
            at.Lq = 1; at.G = a.nh / a.nkv; at.n_kv = a.nkv; at.B = 1; at.scale = a.scale;
            attn_decode_block<true>(at, a.st, a.part, a.max_chunks, r, 0, 0, lds, d);
            return;
        }
        r -= a.n_attn;
        if (r < a.n_o) {
            d.wait = cnt + 1;
            d.target = (unsigned)((a.st->kv_len + 1 + kAttnChunk - 1) / kAttnChunk);
            d.arrive = cnt + 2;
            GemvArgs g{};
            g.W = w.wo; g.n_units = a.H; g.K = a.nh * 256; g.nb = 1; g.out = a.h; g.part = a.part;
            g.max_chunks = a.max_chunks; g.G = a.nh / a.nkv; g.st = a.st;
            gemv_block<1, 4, 2, GV_ORES, 1, false, true>(g, r, a.n_o, reinterpret_cast<uint16_t*>(lds), d);
            return;
        }
        r -= a.n_o;
        if (r < a.n_gu) {
            d.wait = cnt + 2;
            d.target = (unsigned)a.n_o;
            d.arrive = cnt + 3;
            GemvArgs g{};
            g.x = a.h; g.norm_w = w.ln2; g.eps = a.eps; g.W = w.wgu; g.n_units = a.I; g.K = a.H; g.nb = 1;
            g.I = a.I; g.out = a.act;
            gemv_block<1, 4, 2, GV_GEGLU, 1, true, true>(g, r, a.n_gu, nullptr, d);
            return;
        }
        r -= a.n_gu;
        d.wait = cnt + 3;
        d.target = (unsigned)a.n_gu;
        d.arrive = cnt + 4;
        GemvArgs g{};
        g.x = a.act; g.W = w.wdn; g.n_units = a.H; g.K = a.I; g.nb = 1; g.out = a.h;
        gemv_block<1, 32, 2, GV_RES, 4, true, true>(g, r, a.n_dn, nullptr, d);
        return;
    }
    bid -= a.layers * per;
    unsigned* lm_cnt = a.sync + 1 + 5 * a.layers;
    if (bid < a.n_lm) {  // final RMSNorm + tied lm_head, fp32 logits + per-workgroup first max
        Dep d;
        d.err = a.err;
        d.wait = lm_cnt - 1;
        d.target = (unsigned)a.n_dn;
        d.arrive = lm_cnt;
        GemvArgs g{};
        g.x = a.h; g.norm_w = a.fnorm; g.eps = a.eps; g.W = a.E; g.n_units = a.V; g.K = a.H; g.nb = 1;
        g.logits = a.logits; g.pmax = a.pmax; g.pidx = a.pidx;
        gemv_block<1, 4, 4, GV_LOGITS, 1, true, true>(g, bid, a.n_lm, nullptr, d);
        return;
    }
    // argmax over the lm_head partials (torch.argmax: first maximum wins, inference.py:68)
    Dep d;
    d.err = a.err;
    d.wait = lm_cnt;
    d.target = (unsigned)a.n_lm;
    dep_wait(d);
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for (int i = tid; i < a.n_lm; i += 256) {
        const float v = ldf_coh(a.pmax + i);
        const int ix = ldi_coh(a.pidx + i);
        if (v > best || (v == best && ix < bi)) { best = v; bi = ix; }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const float v = __shfl_xor(best, o, 64);
        const int ix = __shfl_xor(bi, o, 64);
        if (v > best || (v == best && ix < bi)) { best = v; bi = ix; }
    }
    float* sv = reinterpret_cast<float*>(lds);
    int* si = reinterpret_cast<int*>(lds + 16);
    if ((tid & 63) == 0) { sv[tid >> 6] = best; si[tid >> 6] = bi; }
    __syncthreads();
    if (tid == 0) {
        for (int q = 1; q < 4; ++q)
            if (sv[q] > best || (sv[q] == best && si[q] < bi)) { best = sv[q]; bi = si[q]; }
        a.next[0] = bi;
    }
    // Every other workgroup has passed its last wait (each arrived after waiting, and all
    // arrivals precede the lm_head count this workgroup waited for; attention workgroups past
    // the last chunk never wait): re-arm the counters for the next launch.
    const int nw = 2 + 5 * a.layers;
    for (int i = tid; i < nw; i += 256) __hip_atomic_store(a.sync + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------- host side
int decode_step_sync_words(int layers) { return (2 + 5 * layers + 3) & ~3; }  // 16-B multiple

int decode_step_launch(hipStream_t s, const DecodeStepDesc& d) {
    if (d.layers > kStepMaxLayers) return -1;
    StepArgs a{};
    for (int l = 0; l < d.layers; ++l) {
        a.L[l].ln1 = d.ln1[l]; a.L[l].wqkv = d.wqkv[l]; a.L[l].wo = d.wo[l]; a.L[l].ln2 = d.ln2[l];
        a.L[l].wgu = d.wgu[l]; a.L[l].wdn = d.wdn[l]; a.L[l].kc = d.kc[l]; a.L[l].vc = d.vc[l];
    }
    a.layers = d.layers; a.ids = d.ids; a.E = d.E; a.fnorm = d.fnorm; a.normalizer = d.normalizer; a.eps = d.eps;
    a.scale = d.scale; a.pad_id = d.pad_id; a.cosT = d.cosT; a.sinT = d.sinT; a.max_pos = d.max_pos; a.st = d.st;
    a.h = d.h; a.q = d.q; a.act = d.act; a.part = d.part; a.max_chunks = d.max_chunks; a.kvb = d.kvb; a.nh = d.nh;
    a.nkv = d.nkv; a.H = d.H; a.I = d.I; a.V = d.V; a.logits = d.logits; a.pmax = d.pmax; a.pidx = d.pidx;
    a.next = d.next; a.sync = d.sync; a.err = d.err;
    a.n_qkv = (d.nh + 2 * d.nkv) * 128 / 4;  // 4 row pairs per workgroup
    a.n_attn = d.max_chunks;
    a.n_o = d.H / 8;                         // 8 rows per workgroup (4 waves x 2)
    a.n_gu = d.I / 8;                        // 8 (gate, up) pairs per workgroup
    a.n_dn = d.H / 2;                        // 2 rows per workgroup (K split over 4 waves)
    a.n_lm = gemv_logits_blocks();
    const long grid = 1 + (long)d.layers * (a.n_qkv + a.n_attn + a.n_o + a.n_gu + a.n_dn) + a.n_lm + 1;
    // counters start at zero (hipMemset at allocation) and the final workgroup re-arms them
    hipLaunchKernelGGL(k_decode_step, dim3((unsigned)grid), dim3(256), 0, s, a);
    return 0;
}

}  // namespace pgmi
