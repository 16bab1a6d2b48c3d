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
constexpr int kCntStride = 32;  // words between counter words: each on its own 128-B line
constexpr int kShards = 32;     // arrival shards per phase (+1 top word the consumers poll)
// Streaming phases: one contiguous slice of units per workgroup, ~one workgroup per CU, rounds
// of (4 waves x RPW) units with the next round's rows in flight; few consumers per hand-off
// (each reads its whole input coherently).  RPW keeps the kernel at <= 128 VGPRs (4 per CU).
constexpr int kGuRpw = 1, kDnRpw = 1, kLmRpw = 2;
constexpr int kGuUpb = 64;   // gate/up pairs per workgroup  (16384 / 64 = 256 workgroups)
constexpr int kDnUpb = 8;    // down rows per workgroup      (2048 / 8 = 256)
constexpr int kOUpb = 32;    // o_proj rows per workgroup    (2048 / 32 = 64)
constexpr int kLmUpb = 1008; // lm_head rows per workgroup   (257216 / 1008 -> 256)
constexpr int kPhaseWords = (kShards + 1) * kCntStride;

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
    unsigned* sync;  // counter i at sync[i * kCntStride]: 0 embed, 1 + 5l + phase, 1 + 5 layers lm_head
    long long* trace;  // optional per-workgroup timestamps [grid][4]
    unsigned* err;
    int n_qkv, n_attn, n_o, n_gu, n_dn, n_lm;
};

// phase i: top word (polled by consumers) then kShards shard words
__device__ __forceinline__ unsigned* cnt_at(const StepArgs& a, int i) { return a.sync + (long)i * kPhaseWords; }

// producer r of n in phase i: shard r % kShards (holding ceil((n - s) / kShards) producers)
__device__ __forceinline__ void set_arrive(Dep& d, const StepArgs& a, int i, int r, int n) {
    const int sh = r % kShards;
    d.arrive = cnt_at(a, i);
    d.arrive_shard = cnt_at(a, i) + (1 + sh) * kCntStride;
    d.shard_n = (unsigned)((n - sh + kShards - 1) / kShards);
}
// consumers of a phase with n producers wait for this many completed shards
__host__ __device__ __forceinline__ unsigned shards_of(int n) { return (unsigned)(n < kShards ? n : kShards); }

__global__ void __launch_bounds__(256, 4) k_decode_step(StepArgs a) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[kAttnDecodeLds];
    const int tid = threadIdx.x;
    if (a.trace && tid == 0) a.trace[(long)blockIdx.x * 4] = __builtin_amdgcn_s_memrealtime();
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
        d.trace = a.trace ? a.trace + (long)blockIdx.x * 4 : nullptr;
        set_arrive(d, a, 0, 0, 1);
        dep_arrive(d);
        return;
    }
    bid -= 1;
    if (bid < a.layers * per) {
        const int l = bid / per;
        int r = bid - l * per;
        const StepLayerW& w = a.L[l];
        const int c0 = 1 + 5 * l;  // this layer's phase counters c0 .. c0 + 4
        Dep d;
        d.err = a.err;
        d.trace = a.trace ? a.trace + (long)blockIdx.x * 4 : nullptr;
        if (r < a.n_qkv) {
            d.wait = cnt_at(a, c0 - 1);  // embed, or the previous layer's down phase
            d.target = shards_of(l == 0 ? 1 : a.n_dn);
            set_arrive(d, a, c0, r, a.n_qkv);
            GemvArgs g{};
            g.x = a.h; g.norm_w = w.ln1; g.eps = a.eps; g.W = w.wqkv; g.n_units = (a.nh + 2 * a.nkv) * 128;
            g.K = a.H; g.nb = 1; g.I = a.nh; g.out = a.q; g.cosT = a.cosT; g.sinT = a.sinT; g.max_pos = a.max_pos;
            g.st = a.st; g.kc = w.kc; g.vc = w.vc; g.kv_b_stride = a.kvb; g.nkv = a.nkv;
            gemv_block<1, 4, 1, GV_QKV, 1, true, true>(g, r, a.n_qkv, nullptr, d);
            return;
        }
        r -= a.n_qkv;
        if (r < a.n_attn) {
            d.wait = cnt_at(a, c0);
            d.target = shards_of(a.n_qkv);
            set_arrive(d, a, c0 + 1, r, (a.st->kv_len + 1 + kAttnChunk - 1) / kAttnChunk);
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
            d.wait = cnt_at(a, c0 + 1);
            d.target = shards_of((a.st->kv_len + 1 + kAttnChunk - 1) / kAttnChunk);
            set_arrive(d, a, c0 + 2, r, a.n_o);
            GemvArgs g{};
            g.W = w.wo; g.n_units = a.H; g.K = a.nh * 256; g.nb = 1; g.out = a.h; g.part = a.part;
            g.max_chunks = a.max_chunks; g.G = a.nh / a.nkv; g.st = a.st; g.upb = kOUpb;
            gemv_block<1, 4, 2, GV_ORES, 1, false, true>(g, r, a.n_o, reinterpret_cast<uint16_t*>(lds), d);
            return;
        }
        r -= a.n_o;
        if (r < a.n_gu) {
            d.wait = cnt_at(a, c0 + 2);
            d.target = shards_of(a.n_o);
            set_arrive(d, a, c0 + 3, r, a.n_gu);
            GemvArgs g{};
            g.x = a.h; g.norm_w = w.ln2; g.eps = a.eps; g.W = w.wgu; g.n_units = a.I; g.K = a.H; g.nb = 1;
            g.I = a.I; g.out = a.act; g.upb = kGuUpb;
            gemv_block<1, 4, kGuRpw, GV_GEGLU, 1, true, true>(g, r, a.n_gu, nullptr, d);
            return;
        }
        r -= a.n_gu;
        d.wait = cnt_at(a, c0 + 3);
        d.target = shards_of(a.n_gu);
        set_arrive(d, a, c0 + 4, r, a.n_dn);
        GemvArgs g{};
        g.x = a.act; g.W = w.wdn; g.n_units = a.H; g.K = a.I; g.nb = 1; g.out = a.h; g.upb = kDnUpb;
        gemv_block<1, 32, kDnRpw, GV_RES, 4, true, true>(g, r, a.n_dn, nullptr, d);
        return;
    }
    bid -= a.layers * per;
    const int lm_c = 1 + 5 * a.layers;
    if (bid < a.n_lm) {  // final RMSNorm + tied lm_head, fp32 logits + per-workgroup first max
        Dep d;
        d.err = a.err;
        d.trace = a.trace ? a.trace + (long)blockIdx.x * 4 : nullptr;
        d.wait = cnt_at(a, lm_c - 1);
        d.target = shards_of(a.n_dn);
        set_arrive(d, a, lm_c, bid, a.n_lm);
        GemvArgs g{};
        g.x = a.h; g.norm_w = a.fnorm; g.eps = a.eps; g.W = a.E; g.n_units = a.V; g.K = a.H; g.nb = 1;
        g.logits = a.logits; g.pmax = a.pmax; g.pidx = a.pidx; g.upb = kLmUpb;
        gemv_block<1, 4, kLmRpw, GV_LOGITS, 1, true, true>(g, bid, a.n_lm, nullptr, d);
        return;
    }
    // argmax over the lm_head partials (torch.argmax: first maximum wins, inference.py:68)
    Dep d;
    d.err = a.err;
    d.trace = a.trace ? a.trace + (long)blockIdx.x * 4 : nullptr;
    d.wait = cnt_at(a, lm_c);
    d.target = shards_of(a.n_lm);
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
    for (int i = tid; i < (lm_c + 1) * (kShards + 1); i += 256)
        __hip_atomic_store(a.sync + (long)i * kCntStride, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------- attention chain (batch 1)
// One launch per layer for GemmaAttention's latency-bound chain at q_len = 1 (modeling_gemma.py:
// 231-293): workgroup ranges [qkv:n_qkv][attn:n_attn][o:n_o] in dependency order with the
// hand-offs of the fused step above (same bodies, same arithmetic), so the qkv -> attention ->
// o_proj boundaries cost a counter wait instead of two kernel launches each.  The HBM-streaming
// gate/up and down projections stay standalone launches.  Counters: 3 phases per layer, re-armed
// by lm_head's last workgroup at the end of the step (gemv_body.h fold; every chain workgroup of
// the step has passed its waits by then).
struct ChainArgs {
    StepLayerW w;
    const StepState* st;
    const uint16_t *cosT, *sinT;
    int max_pos;
    uint16_t *h, *q;
    float* part;
    int max_chunks;
    long kvb;
    int nh, nkv, H;
    float eps, scale;
    unsigned* sync;  // this layer's 3 phase counters
    unsigned* err;
    int n_qkv, n_attn, n_o, o_upb;
};

__global__ void __launch_bounds__(256, 4) k_attn_chain(ChainArgs a) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[kAttnDecodeLds];
    auto cnt = [&](int i) { return a.sync + (long)i * kPhaseWords; };
    Dep d;
    d.err = a.err;
    auto arrive_on = [&](int i, int r, int n) {
        const int sh = r % kShards;
        d.arrive = cnt(i);
        d.arrive_shard = cnt(i) + (1 + sh) * kCntStride;
        d.shard_n = (unsigned)((n - sh + kShards - 1) / kShards);
    };
    int r = blockIdx.x;
    if (r < a.n_qkv) {  // inputs come from the previous launch: no wait
        arrive_on(0, r, a.n_qkv);
        GemvArgs g{};
        g.x = a.h; g.norm_w = a.w.ln1; g.eps = a.eps; g.W = a.w.wqkv; g.n_units = (a.nh + 2 * a.nkv) * 128;
        g.K = a.H; g.nb = 1; g.I = a.nh; g.out = a.q; g.cosT = a.cosT; g.sinT = a.sinT; g.max_pos = a.max_pos;
        g.st = a.st; g.kc = a.w.kc; g.vc = a.w.vc; g.kv_b_stride = a.kvb; g.nkv = a.nkv;
        gemv_block<1, 4, 1, GV_QKV, 1, true, true>(g, r, a.n_qkv, nullptr, d);
        return;
    }
    r -= a.n_qkv;
    const int n_chunks = (a.st->kv_len + 1 + kAttnChunk - 1) / kAttnChunk;
    if (r < a.n_attn) {
        d.wait = cnt(0);
        d.target = shards_of(a.n_qkv);
        arrive_on(1, r, n_chunks);
        const int kvd = a.nkv * 256;
        AttnArgs at{};
        at.q = a.q; at.q_b_stride = (long)a.nh * 256; at.q_row_stride = a.nh * 256; at.q_head_stride = 256;
        at.k = a.w.kc; at.k_b_stride = a.kvb; at.k_row_stride = kvd; at.k_head_stride = 256;
        at.v = a.w.vc; at.v_b_stride = a.kvb; at.v_row_stride = kvd; at.v_head_stride = 256;
        at.Lq = 1; at.G = a.nh / a.nkv; at.n_kv = a.nkv; at.B = 1; at.scale = a.scale;
        attn_decode_block<true>(at, a.st, a.part, a.max_chunks, r, 0, 0, lds, d);
        return;
    }
    r -= a.n_attn;
    d.wait = cnt(1);
    d.target = shards_of(n_chunks);
    arrive_on(2, r, a.n_o);
    GemvArgs g{};
    g.W = a.w.wo; g.n_units = a.H; g.K = a.nh * 256; g.nb = 1; g.out = a.h; g.part = a.part;
    g.max_chunks = a.max_chunks; g.G = a.nh / a.nkv; g.st = a.st; g.upb = a.o_upb;
    gemv_block<1, 4, 2, GV_ORES, 1, false, true>(g, r, a.n_o, reinterpret_cast<uint16_t*>(lds), d);
}

int attn_chain_sync_words(int layers) { return 3 * layers * kPhaseWords; }
int attn_chain_counter_stride() { return kCntStride; }

void attn_chain_launch(hipStream_t s, const DecodeStepDesc& d, int layer, int launch_keys, unsigned* sync) {
    ChainArgs a{};
    a.w.ln1 = d.ln1[layer]; a.w.wqkv = d.wqkv[layer]; a.w.wo = d.wo[layer]; a.w.kc = d.kc[layer]; a.w.vc = d.vc[layer];
    a.st = d.st; a.cosT = d.cosT; a.sinT = d.sinT; a.max_pos = d.max_pos; a.h = d.h; a.q = d.q; a.part = d.part;
    a.max_chunks = d.max_chunks; a.kvb = d.kvb; a.nh = d.nh; a.nkv = d.nkv; a.H = d.H; a.eps = d.eps;
    a.scale = d.scale; a.sync = sync + (long)layer * 3 * kPhaseWords; a.err = d.err;
    a.n_qkv = (d.nh + 2 * d.nkv) * 128 / 4;
    const int nch = (launch_keys + kAttnChunk - 1) / kAttnChunk;
    a.n_attn = nch < d.max_chunks ? nch : d.max_chunks;
    a.o_upb = 8;  // 256 workgroups of 8 rows, as the standalone o_proj launch
    a.n_o = (d.H + a.o_upb - 1) / a.o_upb;
    hipLaunchKernelGGL(k_attn_chain, dim3(a.n_qkv + a.n_attn + a.n_o), dim3(256), 0, s, a);
}

// ---------------------------------------------------------------- host side
int decode_step_sync_words(int layers) { return (2 + 5 * layers) * kPhaseWords; }

long decode_step_grid(const DecodeStepDesc& d) {
    return 1 + (long)d.layers * ((d.nh + 2 * d.nkv) * 128 / 4 + d.max_chunks + (d.H + kOUpb - 1) / kOUpb +
                                 (d.I + kGuUpb - 1) / kGuUpb + (d.H + kDnUpb - 1) / kDnUpb) +
           (d.V + kLmUpb - 1) / kLmUpb + 1;
}

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
    a.next = d.next; a.sync = d.sync; a.err = d.err; a.trace = d.trace;
    a.n_qkv = (d.nh + 2 * d.nkv) * 128 / 4;  // 4 row pairs per workgroup
    a.n_attn = d.max_chunks;
    a.n_o = (d.H + kOUpb - 1) / kOUpb;
    a.n_gu = (d.I + kGuUpb - 1) / kGuUpb;
    a.n_dn = (d.H + kDnUpb - 1) / kDnUpb;
    a.n_lm = (d.V + kLmUpb - 1) / kLmUpb;
    const long grid = 1 + (long)d.layers * (a.n_qkv + a.n_attn + a.n_o + a.n_gu + a.n_dn) + a.n_lm + 1;
    // counters start at zero (hipMemset at allocation) and the final workgroup re-arms them
    hipLaunchKernelGGL(k_decode_step, dim3((unsigned)grid), dim3(256), 0, s, a);
    return 0;
}

}  // namespace pgmi
