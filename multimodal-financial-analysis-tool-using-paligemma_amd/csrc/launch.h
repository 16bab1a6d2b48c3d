// launch.h -- host-side launchers for the libpgmi kernels (internal, not the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pgmi {

// ---------------------------------------------------------------- GEMM (prefill)
enum Epi : int {
    EPI_STORE = 0,      // out = bf16(acc)
    EPI_BIAS = 1,       // out = bf16(acc + bias)
    EPI_BIAS_GELU = 2,  // out = bf16(gelu(bf16(acc + bias)))
    EPI_BIAS_RES = 3,   // out = bf16(bf16(acc + bias) + res)
    EPI_RES = 4,        // out = bf16(bf16(acc) + res)
    EPI_BIAS_POS = 5,   // out = bf16(bf16(acc + bias) + pos[m % npos])
    EPI_F32 = 6,        // out_f32 = float(bf16(acc))
    EPI_GEGLU = 7,      // out = bf16(bf16(gelu(bf16(acc_gate))) * bf16(acc_up))  (dual B)
    EPI_ROPE = 8,       // Gemma q|k|v rows: RoPE on q and k, q -> q_out, k / v appended to the KV cache
                        // (modeling_gemma.py:197-198,259); gemm_qkv_rope only
};

struct EpiArgs {
    const uint16_t* bias = nullptr;
    const uint16_t* res = nullptr;  // [M][ldr]
    int ldr = 0;
    const uint16_t* pos = nullptr;  // [npos][N]
    int npos = 0;
    uint16_t* out = nullptr;        // [M][ldo]
    int ldo = 0;
    float* out_f32 = nullptr;       // [M][ldo]
    // EPI_ROPE: rows m = b * L + l at rotary position rpos[m]; heads [0, nh) are q (-> q_out
    // [M][nh*256]), nh .. nh+nkv-1 are k, the rest v (-> kc / vc at token kv_start + l)
    const int64_t* rpos = nullptr;
    const uint16_t* cosT = nullptr;
    const uint16_t* sinT = nullptr;
    int max_pos = 0;
    uint16_t* q_out = nullptr;
    uint16_t* kc = nullptr;
    uint16_t* vc = nullptr;
    long kv_b_stride = 0;
    int kv_start = 0;
    int L = 1;
    int nh = 0;
    int nkv = 0;
};

// C[M,N] = A[M,K] (row-major, lda) x W[N,K]^T (row-major, ldw).  For EPI_GEGLU the
// "up" weight rows are W + up_offset_rows*ldw.  `ws` is fp32 scratch for split-K.
// Returns the split-K factor used.  With defer = true and a split > 1 only the fp32 partial
// slabs ws[split][M][N] are written and the epilogue is left to the consumer kernel
// (splitk_res_norm / rope_kv_append); otherwise the epilogue is applied and 1 is returned.
// q|k|v projection with the RoPE / KV-append epilogue (EPI_ROPE) when the measured plan for the
// shape allows it (two 16-column tiles per wave, no split-K); false: nothing launched, the caller
// runs gemm(EPI_STORE) + rope_kv_append
bool gemm_qkv_rope(hipStream_t s, const uint16_t* A, int lda, const uint16_t* W, int ldw, int M, int N, int K,
                   const EpiArgs& ea);
int gemm(hipStream_t s, const uint16_t* A, int lda, const uint16_t* W, int ldw, int M, int N, int K,
         Epi epi, const EpiArgs& ea, float* ws, size_t ws_bytes, int up_offset_rows = 0, bool defer = false);
size_t gemm_ws_bytes(int M, int N, int K);
void gemm_force_plan(int cfg, int split);  // cfg < 0: automatic
int gemm_force_shape(int M, int N, int K, int dual, int cfg, int split);  // cfg < 0: remove the override
// probe: the next GEMM kernel launched takes these events as its own start / stop (hipExtLaunchKernelGGL)
void gemm_probe_events(hipEvent_t start, hipEvent_t stop);
// host replica of the panel / 8-phase GEMMs' workgroup -> tile order (CPU test); returns the XCD block code
int gemm_tile_order(int n_mt, int n_nt, int S, int BM, int BN, int K, int* mt, int* nt, int* z);
constexpr int kGemmCfgs = 39;              // tile configurations (kernels_gemm.hip Cfg)

// ---------------------------------------------------------------- decode GEMV
struct StepState {  // device-resident decode step (read by kernels -> graph-replayable)
    int kv_len;     // index the new token's K/V is written at (= KVCache.num_items())
    int position;   // rotary position (= attention_mask.cumsum(-1)[:, -1], modeling_gemma.py:526)
};

// decode layer 0: the embedding lookup folded into the q|k|v GEMV (h_out receives the scaled row)
struct EmbedFold {
    const int64_t* ids;
    const uint16_t* E;
    float normalizer;
    int64_t pad_id;
    uint16_t* h_out;
};
bool gemv_qkv_folds_embed(int B);  // batches the fold covers (the register-input GEMV, B <= 2)
// fused input RMSNorm + q/k/v projection + RoPE + KV-cache append (K = 2048)
void gemv_qkv(hipStream_t s, int B, int nh, int nkv, const uint16_t* h, const uint16_t* norm_w, float eps,
              const uint16_t* Wqkv, const uint16_t* cosT, const uint16_t* sinT, int max_pos, const StepState* st,
              uint16_t* q_out, uint16_t* kc, uint16_t* vc, long kv_b_stride, float* ws = nullptr,
              const EmbedFold* emb = nullptr, const uint16_t* Wf = nullptr);  // Wf: as gemv_geglu's
// ws: fp32 scratch (>= 4 x B x N floats) for the MFMA path's K split of K = 16384 (B >= 3)
void gemv_res(hipStream_t s, int B, int K, const uint16_t* x, const uint16_t* W, int N, uint16_t* h_inout,
              float* ws);
// gemv_res, then hn = RMSNorm(h) with norm_w (nullptr: none); on the batched MFMA path the norm is
// fused into the K-split combine (one workgroup per row)
void gemv_res_norm(hipStream_t s, int B, int K, const uint16_t* x, const uint16_t* W, int N, uint16_t* h_inout,
                   float* ws, const uint16_t* norm_w, float eps, uint16_t* hn, const uint16_t* Wf = nullptr);
// the fragment-major image of a [rows][K] matrix for the batched decode GEMVs (rows % 16 == 0, K % 32 == 0)
// (qkv: in the batched q|k|v GEMV's row order)
void mf_swizzle(hipStream_t s, const uint16_t* W, int rows, int K, uint16_t* out, bool qkv = false);
// hn[b] = RMSNorm(x[b]) for nb rows of K (one workgroup per row)
void rows_norm(hipStream_t s, const uint16_t* x, const uint16_t* w, float eps, int nb, int K, uint16_t* out);
// o_proj + residual whose input is the combine of the decode-attention partials (MQA:
// n_kv = 1, G heads of 256); o_out (optional) receives the combined bf16 attention output.
// ssq (batched MFMA form only, else ignored): each row's 16-column partial sums of squares of the
// new h, [B][N / 16] -- the next RMSNorm's, read by gemv_geglu
void gemv_o_attn(hipStream_t s, int B, int G, const float* part, int max_chunks, const StepState* st,
                 const uint16_t* Wo, int N, uint16_t* h_inout, uint16_t* o_out, float* ssq = nullptr,
                 const uint16_t* Wf = nullptr);
// fused RMSNorm + gate|up + GeGLU; ssq (B >= gemv_mf_min_batch() only): h's RMSNorm from the
// partials gemv_o_attn wrote instead of the row pass; Wf (idem): the gate|up weights' fragment-major
// image (mf_swizzle: the gate rows', then the up rows'), read instead of Wgu
void gemv_geglu(hipStream_t s, int B, const uint16_t* h, const uint16_t* norm_w, float eps,
                const uint16_t* Wgu, int I, uint16_t* act, float* ssq = nullptr, const uint16_t* Wf = nullptr);
int gemv_logits_blocks();
int gemv_mf_min_batch();  // smallest batch on the MFMA decode projections
// done/next/adv (decode, may be null): fold the argmax into the launch's last workgroup and
// advance the step state there; returns true when it did (no argmax_finish needed)
bool gemv_logits(hipStream_t s, int B, const uint16_t* h, const uint16_t* norm_w, float eps,
                 const uint16_t* E, int V, float* logits, float* pmax, int* pidx, int* nparts,
                 unsigned* done = nullptr, int64_t* next = nullptr, StepState* adv = nullptr,
                 int64_t* hist = nullptr);
// adv (may be null): the decode step state, advanced by one step (the step's last kernel); hist (may be
// null): a second destination of the argmax (a multi-step graph's per-step token record)
void argmax_finish(hipStream_t s, int B, const float* pmax, const int* pidx, int nparts, int64_t* out,
                   StepState* adv = nullptr, int64_t* hist = nullptr);
int argmax_scratch_parts();
void argmax_rows(hipStream_t s, const float* x, int rows, int V, float* pmax, int* pidx, int64_t* out);
void eos_update(hipStream_t s, int64_t* next, int* finished, int B, int64_t eos, int64_t pad, int* n_alive);

// ---------------------------------------------------------------- attention
struct AttnArgs {
    const uint16_t* q; long q_b_stride; int q_row_stride; int q_head_stride;
    const uint16_t* k; long k_b_stride; int k_row_stride; int k_head_stride;
    const uint16_t* v; long v_b_stride; int v_row_stride; int v_head_stride;
    uint16_t* o; long o_b_stride; int o_row_stride; int o_head_stride;
    int Lq;        // query positions per batch element
    int Lk;        // keys
    int G;         // query heads per kv head
    int n_kv;      // kv heads
    int B;
    float scale;   // s = bf16(bf16(q.k) * scale)
    float* ws;     // prefill: fp32 scratch for key-split partials (nullptr: no key split)
    long ws_floats;
    // decode: additive attention mask (modeling_gemma.py:269), fp32, key j of batch row b at
    // mask[b * mask_b_stride + j * mask_k_stride]; mask_round: the sum is rounded to bf16 (a bf16
    // mask) or kept in fp32 (an fp32 mask, as torch promotes).  No mask: a zero word with stride 0
    const float* mask;
    long mask_b_stride;
    int mask_k_stride;
    int mask_round;
};
void attention_prefill(hipStream_t s, int head_dim, const AttnArgs& a);
// decode: Lq == 1, rows = the G heads; keys split over chunks; kv length from StepState (+1)
// flash-decoding over 64-key chunks (partials only; the combine is gemv_o_attn's prologue);
// launch_keys = upper bound on kv_len+1 this call
void attention_decode(hipStream_t s, const AttnArgs& a, const StepState* st, int launch_keys, float* part,
                      int max_chunks);
constexpr int kAttnChunk = 64;
constexpr int kAttnPartStride = 16 * 256 + 32;  // floats per (b, kv head, chunk) record
size_t attention_decode_part_floats(int B, int n_kv, int max_chunks);
int attention_prefill_max_keys(int head_dim);
void attention_force_variant(int v);  // tuning hook (kernels_attn.hip); -1 = measured choice

// ---------------------------------------------------------------- per-module entry points (kernels_modules.hip)
// reference-order attention with the probability matrix and an additive mask (module forwards)
struct ModAttnArgs {
    const uint16_t* q;           // (B, Lq, H, hd)
    const uint16_t* k;           // KV head hk of batch b, key j: k + b*kv_b_stride + hk*kv_h_stride + j*kv_row_stride
    const uint16_t* v;
    long kv_b_stride, kv_h_stride, kv_row_stride;
    uint16_t* o;                 // (B, Lq, H, hd)
    uint16_t* probs;             // (B, H, Lq, Lk) bf16 or nullptr
    const void* mask;            // additive, element (b, h, i, j) at b*m_b_stride + h*m_h_stride + i*m_q_stride + j
    long m_b_stride, m_h_stride, m_q_stride;
    int mask_f32;                // 1: fp32 mask (added in fp32), 0: bf16 mask (sum rounded to bf16)
    int B, Lq, Lk, H, Hkv, hd;
    float scale;
    int scale_div;               // 1: s / scale (Gemma's "/ math.sqrt(head_dim)"), 0: s * scale (SigLIP)
};
size_t attention_exact_lds(int Lk, int hd);
void attention_exact(hipStream_t s, const ModAttnArgs& a);
// apply_rotary_pos_emb on one projection: x (rows, heads*hd), cos/sin (rows, hd) bf16
void rope_rows(hipStream_t s, const uint16_t* x, const uint16_t* cs, const uint16_t* sn, long rows, int heads, int hd,
               uint16_t* out);

// ---------------------------------------------------------------- misc
// Fused consumer of a projection + residual: if split > 1, h = bf16(bf16(sum_z ws[z] (+bias)) + h)
// (fixed z order) is written back to h first; then out = norm(h): RMSNorm (b == nullptr,
// (1 + w) form) or LayerNorm (b != nullptr).  D <= 4096.
void splitk_res_norm(hipStream_t s, const float* ws, int split, const uint16_t* bias, uint16_t* h, const uint16_t* w,
                     const uint16_t* b, float eps, uint16_t* out, int rows, int D);
void rmsnorm(hipStream_t s, const uint16_t* x, const uint16_t* w, float eps, uint16_t* out, int rows, int D);
void layernorm(hipStream_t s, const uint16_t* x, const uint16_t* w, const uint16_t* b, float eps, uint16_t* out,
               int rows, int D);
void embed_rows(hipStream_t s, const int64_t* ids, int rows, const uint16_t* E, int D, float normalizer,
                int64_t pad_id, uint16_t* out);
// merge (modeling_gemma.py:468-537) + GemmaModel normalizer (:367-368)
void merge_embed(hipStream_t s, const int64_t* ids, int B, int L, const uint16_t* E, int D,
                 const uint16_t* img, int n_img_rows, int64_t image_token, int64_t pad_id, float sqrt_h,
                 float normalizer, const uint16_t* embeds_in, int* scan_buf, uint16_t* out);
void scale_rows(hipStream_t s, const uint16_t* x, long n, float normalizer, uint16_t* out);
void add_rows(hipStream_t s, const uint16_t* x, const uint16_t* y, long n, uint16_t* out);  // bf16(x + y), n % 8 == 0
// qkv: bf16 [B*L][(nh+2nkv)*256], or (split > 1) the fp32 partial slabs ws[split][B*L][...]
void rope_kv_append(hipStream_t s, const uint16_t* qkv, const float* ws, int split, int B, int L, int nh, int nkv,
                    const int64_t* pos, const uint16_t* cosT, const uint16_t* sinT, int max_pos, uint16_t* q_out,
                    uint16_t* kcache, uint16_t* vcache, long kv_b_stride, int kv_start);
void patchify(hipStream_t s, const void* px, int px_is_f32, int B, int C, int H, int W, int P, int Kpad,
              uint16_t* out);
void fill_synthetic(hipStream_t s, uint16_t* dst, long n, uint64_t key, float scale, float offset);
void set_step(hipStream_t s, StepState* st, int kv_len, int position);
// step state with the rotary position read on the device: round(pos[0]) of a (B, 1) position tensor
// of dtype PGMI_DTYPE_* (+ 10 = int64, 11 = int32, 12 = float64) -- no host read of a merge's positions
void set_step_dev(hipStream_t s, StepState* st, int kv_len, const void* pos, int dtype);
// an additive mask row set (B rows of n keys, element (b, j) at src[b * b_stride + j], dtype bf16 / fp32)
// -> fp32 [B][ld]
void stage_mask(hipStream_t s, const void* src, int dtype, int B, long b_stride, int n, float* dst, int ld);
// PIL-exact BICUBIC resize of a uint8 HWC RGB image + rescale/normalize -> float32 CHW
// (processing_paligemma.py:13-49); scratch of preprocess_scratch_bytes() on the device
size_t preprocess_scratch_bytes(int H, int W, int out_h, int out_w);
void preprocess(hipStream_t s, const uint8_t* src, int H, int W, int out_h, int out_w, float* out, void* scratch);
void pad_rows(hipStream_t s, const uint16_t* src, int rows, int K, int Kpad, uint16_t* dst);
// nucleus sampling (kernels_sample.hip; inference.py:15-24, :65); scratch of sample_scratch_bytes()
size_t sample_scratch_bytes(int rows, int V);
void sample_top_p(hipStream_t s, const float* x, int rows, int V, float temperature, float top_p, const float* u,
                  void* scratch, int64_t* out, float* kept_mass);


bool gemv_logits_folds(int B);

}  // namespace pgmi
