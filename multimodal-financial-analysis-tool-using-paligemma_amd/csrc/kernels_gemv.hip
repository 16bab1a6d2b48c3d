// kernels_gemv.hip -- launchers of the decode GEMV kernels (bodies: gemv_body.h).
#include <cstdlib>

#include "gemv_body.h"

namespace pgmi {

// MFMA path for 3..16 lock-step sequences (kernels_gemv_mfma.hip)
int gemv_mf_min_batch();
void gemv_mf_qkv(hipStream_t s, const GemvArgs& a, float* ws);
void gemv_mf_geglu(hipStream_t s, const GemvArgs& a);
void gemv_mf_ores(hipStream_t s, const GemvArgs& a, uint16_t* o);
int gemv_mf_logits(hipStream_t s, const GemvArgs& a, int max_blocks);
void gemv_mf_res(hipStream_t s, const GemvArgs& a, float* ws);
void gemv_mf_res_norm(hipStream_t s, const GemvArgs& a, float* ws, const uint16_t* norm_w, float eps, uint16_t* hn);

template <int B, int KCH, int RPW, int MODE, int WK = 1, int DEPTH = 1, bool EMB = false>
static void launch_gemv(hipStream_t s, const GemvArgs& a, int max_blocks = 0) {
    constexpr bool XREG = (MODE != GV_ORES) && B * (KCH / WK) <= 8;
    size_t lds = XREG ? 0 : (size_t)B * KCH * 512 * sizeof(uint16_t);
    static size_t attr = 0;  // largest dynamic LDS size granted so far
    if (lds > attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemv<B, KCH, RPW, MODE, WK, XREG, DEPTH, EMB>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr = lds;
    }
    constexpr int per_block = (4 / WK) * RPW;
    int blocks = (a.n_units + per_block - 1) / per_block;
    if (max_blocks > 0 && blocks > max_blocks) blocks = max_blocks;
    hipLaunchKernelGGL((k_gemv<B, KCH, RPW, MODE, WK, XREG, DEPTH, EMB>), dim3(blocks), dim3(256), lds, s, a);
}

// K = 2048 (hidden); nh q heads, nkv kv heads of 256
bool gemv_qkv_folds_embed(int B) { return B <= 2 && B < gemv_mf_min_batch(); }

void gemv_qkv(hipStream_t s, int B, int nh, int nkv, const uint16_t* h, const uint16_t* norm_w, float eps,
              const uint16_t* Wqkv, const uint16_t* cosT, const uint16_t* sinT, int max_pos, const StepState* st,
              uint16_t* q_out, uint16_t* kc, uint16_t* vc, long kv_b_stride, float* ws, const EmbedFold* emb,
              const uint16_t* Wf) {
    GemvArgs a{};
    a.x = h; a.norm_w = norm_w; a.eps = eps; a.W = Wqkv; a.n_units = (nh + 2 * nkv) * 128; a.K = 2048; a.nb = B;
    a.I = nh; a.out = q_out; a.cosT = cosT; a.sinT = sinT; a.max_pos = max_pos; a.st = st; a.kc = kc; a.vc = vc;
    a.kv_b_stride = kv_b_stride; a.nkv = nkv;
    if (emb) {  // layer 0: the token's embedding row is the input (and is written to h)
        a.ids = emb->ids; a.E = emb->E; a.normalizer = emb->normalizer; a.pad_id = emb->pad_id; a.emb_out = emb->h_out;
        if (B <= 1) launch_gemv<1, 4, 1, GV_QKV, 1, 1, true>(s, a);
        else launch_gemv<2, 4, 1, GV_QKV, 1, 1, true>(s, a);
        return;
    }
#define L_(b_, kch, rpw, mode) launch_gemv<b_, kch, rpw, mode>(s, a)
    if (B >= gemv_mf_min_batch()) {
        a.Wf = Wf;
        gemv_mf_qkv(s, a, ws);
        return;
    }
    if (B <= 1) L_(1, 4, 1, GV_QKV);
    else L_(2, 4, 1, GV_QKV);  // B >= 3 runs on MFMA (above)
}

void gemv_res(hipStream_t s, int B, int K, const uint16_t* x, const uint16_t* W, int N, uint16_t* h_inout,
              float* ws) {
    GemvArgs a{};
    a.x = x; a.norm_w = nullptr; a.W = W; a.n_units = N; a.K = K; a.nb = B; a.out = h_inout;
    if (B >= gemv_mf_min_batch() && K % 128 == 0 && ws) {
        gemv_mf_res(s, a, ws);
        return;
    }
    if (K == 2048) {
        if (B <= 1) L_(1, 4, 1, GV_RES);
        else if (B <= 2) L_(2, 4, 1, GV_RES);
        else if (B <= 4) L_(4, 4, 1, GV_RES);
        else L_(8, 4, 1, GV_RES);
    } else {  // K = 16384: x staged per <= 4 rows (LDS 32 KiB per row)
        for (int b0 = 0; b0 < B; b0 += 4) {
            const int nb = (B - b0) < 4 ? (B - b0) : 4;
            GemvArgs c = a;
            c.x = x + (long)b0 * K; c.out = h_inout + (long)b0 * N; c.nb = nb;
            // K split in 4 inside the workgroup: 512 workgroups of one row each
            if (nb <= 1) launch_gemv<1, 32, 1, GV_RES, 4>(s, c, 512);
            else if (nb <= 2) launch_gemv<2, 32, 2, GV_RES, 4>(s, c);
            else launch_gemv<4, 32, 2, GV_RES, 4>(s, c);
        }
    }
}

// batched (MFMA) residual projection whose combine also writes the next RMSNorm of h (hn); other
// batches / shapes: gemv_res, then rows_norm
void gemv_res_norm(hipStream_t s, int B, int K, const uint16_t* x, const uint16_t* W, int N, uint16_t* h_inout,
                   float* ws, const uint16_t* norm_w, float eps, uint16_t* hn, const uint16_t* Wf) {
    if (B >= gemv_mf_min_batch() && K % 2048 == 0 && K / 2048 <= 8 && K > 2048 && ws) {
        GemvArgs a{};
        a.x = x; a.norm_w = nullptr; a.W = W; a.n_units = N; a.K = K; a.nb = B; a.out = h_inout;
        a.Wf = N % 16 == 0 ? Wf : nullptr;
        gemv_mf_res_norm(s, a, ws, norm_w, eps, hn);
        return;
    }
    gemv_res(s, B, K, x, W, N, h_inout, ws);
    if (norm_w) rows_norm(s, h_inout, norm_w, eps, B, N, hn);
}

void gemv_o_attn(hipStream_t s, int B, int G, const float* part, int max_chunks, const StepState* st,
                 const uint16_t* Wo, int N, uint16_t* h_inout, uint16_t* o_out, float* ssq, const uint16_t* Wf) {
    GemvArgs a{};
    a.x = nullptr; a.norm_w = nullptr; a.W = Wo; a.n_units = N; a.K = G * 256; a.nb = B; a.out = h_inout;
    a.part = part; a.max_chunks = max_chunks; a.G = G; a.st = st; a.o_out = o_out;
    if (B >= gemv_mf_min_batch() && o_out) {
        a.ssq = ssq;
        a.Wf = N % 16 == 0 ? Wf : nullptr;
        gemv_mf_ores(s, a, o_out);
        return;
    }
    // grid capped so each workgroup's combine prologue is amortised over 8 output rows (256 / 128 / 64
    // measured in round 4: 952 / 928-939 / 894-899 tok/s, profiles/r04_b1_probes_ab.txt)
    if (B <= 1) launch_gemv<1, 4, 2, GV_ORES>(s, a, 256);
    else if (B <= 2) launch_gemv<2, 4, 2, GV_ORES>(s, a, 256);
    else if (B <= 4) launch_gemv<4, 4, 1, GV_ORES>(s, a, 256);
    else launch_gemv<8, 4, 1, GV_ORES>(s, a, 256);
}

void gemv_geglu(hipStream_t s, int B, const uint16_t* h, const uint16_t* norm_w, float eps, const uint16_t* Wgu,
                int I, uint16_t* act, float* ssq, const uint16_t* Wf) {
    GemvArgs a{};
    a.x = h; a.norm_w = norm_w; a.eps = eps; a.W = Wgu; a.n_units = I; a.K = 2048; a.nb = B; a.I = I; a.out = act;
    if (B >= gemv_mf_min_batch()) {
        a.ssq = norm_w ? ssq : nullptr;
        a.Wf = I % 16 == 0 ? Wf : nullptr;
        gemv_mf_geglu(s, a);
        return;
    }
    if (B <= 1) launch_gemv<1, 4, 1, GV_GEGLU>(s, a, 1024);
    else L_(2, 4, 2, GV_GEGLU);  // B >= 3 runs on MFMA (above)
}

int gemv_logits_blocks() { return 2048; }

// the streaming lm_head (B < the MFMA batch) folds the argmax into its last workgroup
bool gemv_logits_folds(int B) { return B < gemv_mf_min_batch(); }

bool gemv_logits(hipStream_t s, int B, const uint16_t* h, const uint16_t* norm_w, float eps, const uint16_t* E,
                 int V, float* logits, float* pmax, int* pidx, int* nparts, unsigned* done, int64_t* next,
                 StepState* adv, int64_t* hist) {
    GemvArgs a{};
    a.x = h; a.norm_w = norm_w; a.eps = eps; a.W = E; a.n_units = V; a.K = 2048; a.nb = B; a.logits = logits;
    a.pmax = pmax; a.pidx = pidx;
    const int mb = gemv_logits_blocks();  // pmax/pidx capacity
    int blocks;
    if (B >= gemv_mf_min_batch()) {
        *nparts = gemv_mf_logits(s, a, mb);
        return false;
    }
    const bool fold = done && next && gemv_logits_folds(B);
    if (fold) {
        a.done = done;
        a.next = next;
        a.adv = adv;
        a.hist = hist;
    }
#define LG_(b_, rpw)                                                    \
    do {                                                                \
        blocks = (V + 4 * rpw - 1) / (4 * rpw);                         \
        if (blocks > mb) blocks = mb;                                   \
        launch_gemv<b_, 4, rpw, GV_LOGITS>(s, a, mb);                   \
    } while (0)
    if (B <= 1) LG_(1, 4);
    else LG_(2, 4);  // B >= 3 runs on MFMA (above)
    *nparts = blocks;
    return fold;
#undef LG_
#undef L_
}

}  // namespace pgmi
