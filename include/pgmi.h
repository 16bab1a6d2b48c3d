/*
 * pgmi.h -- C ABI of libpgmi, the MI355X-native (gfx950) PaliGemma-3B inference path.
 *
 * This is the drop-in boundary below the reference's Python API
 * (PaliGemmaForConditionalGeneration / SiglipVisionModel / GemmaForCausalLM / KVCache in
 * /root/reference/modeling_gemma.py and modeling_siglip.py).  The reference itself has no
 * FFI -- it is pure PyTorch -- so each entry point names the reference function whose body it
 * replaces; INTEGRATION.md shows the ctypes binding a maintainer would add.
 *
 * Conventions
 *   - plain C, every call returns 0 on success or a negative PGMI_E* code; the message of the
 *     last failure on the calling thread is pgmi_last_error().
 *   - device pointers are HIP device memory of the context's device; streams are hipStream_t
 *     passed as void* (NULL = the default stream).  Calls are stream-ordered and do not
 *     synchronise unless stated.
 *   - bf16 tensors are raw uint16 bit patterns, row-major, contiguous.
 *   - one context per GPU; a context is not re-entrant (the reference is single-threaded).
 */
#ifndef PGMI_H
#define PGMI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PGMI_OK 0
#define PGMI_E_ARG -1     /* ValueError in the Python layer   */
#define PGMI_E_STATE -2   /* AssertionError / misuse          */
#define PGMI_E_HIP -3     /* HIP runtime error                */
#define PGMI_E_NOMEM -4   /* allocation failure               */

#define PGMI_DTYPE_BF16 0
#define PGMI_DTYPE_F16 1
#define PGMI_DTYPE_F32 2

typedef struct pgmi_ctx pgmi_ctx;

/* Mirrors SiglipVisionConfig (modeling_siglip.py:7-34), GemmaConfig (modeling_gemma.py:39-71)
 * and PaliGemmaConfig (modeling_gemma.py:74-105), plus workspace capacities. */
typedef struct pgmi_config {
    int v_hidden, v_intermediate, v_layers, v_heads, v_channels, v_image, v_patch;
    float v_ln_eps;
    int t_vocab, t_hidden, t_intermediate, t_layers, t_heads, t_kv_heads, t_head_dim, t_max_pos;
    float t_rms_eps, t_rope_theta;
    int projection_dim;
    int64_t image_token_index;
    int64_t pad_token_id; /* -1 when the config's pad_token_id is None (modeling_gemma.py:453) */
    int max_batch;        /* sequences / images per call                                    */
    int max_seq;          /* longest prefill (image + text tokens)                          */
    int max_kv;           /* KV-cache capacity in tokens (decode attention scratch)          */
} pgmi_config;

const char* pgmi_last_error(void);
const char* pgmi_version(void);

/* PaliGemmaForConditionalGeneration.__init__ (modeling_gemma.py:442-453): builds the weight
 * layout; device memory is touched only by the calls below. */
int pgmi_create(int device, const pgmi_config* cfg, pgmi_ctx** out);
int pgmi_destroy(pgmi_ctx* ctx);

/* ---- weights: one bf16 slab in caller-owned device memory, laid out by the library.
 * Tensor names and shapes are the reference state-dict keys; lm_head is
 * tied to embed_tokens (modeling_gemma.py:396-397) and has no slot of its own. */
int64_t pgmi_weights_bytes(const pgmi_ctx* ctx);
int pgmi_weight_count(const pgmi_ctx* ctx);
int pgmi_weight_info(const pgmi_ctx* ctx, int idx, const char** name, int64_t* offset_bytes, int64_t* shape4,
                     int* ndim);
int pgmi_bind_weights(pgmi_ctx* ctx, void* dev_slab);
/* load_state_dict for one tensor (utils.py:30-38 / ablation_study_fixed.py:315-320): copies
 * (and converts to bf16) from host or device memory into the slab. */
int pgmi_load_weight(pgmi_ctx* ctx, const char* name, const void* src, int src_dtype, int src_on_device,
                     void* stream);
/* Native safetensors reader (replaces the safe_open / accelerate
 * shard loop of utils.py:19-44 and ablation_study_fixed.py:304-332): one *.safetensors file is
 * memory-mapped and every tensor whose name is a slab weight is shape-checked, converted to bf16
 * (BF16 copied, F32/F16 rounded to nearest even on the device) and written into the slab.
 * Names that are not slab weights (e.g. a tied lm_head) are counted in *n_skipped.  Synchronises
 * `stream`; call pgmi_prepare again afterwards.  A malformed header or a shape / dtype mismatch
 * is PGMI_E_ARG (ValueError). */
int pgmi_load_safetensors(pgmi_ctx* ctx, const char* path, int* n_loaded, int* n_skipped, void* stream);
/* header inspection, no device needed: tensor count, and entry i's name (NUL-terminated, at most
 * name_cap bytes), dtype (PGMI_DTYPE_*, -1 for other dtypes), shape, data byte range */
int pgmi_safetensors_count(const char* path, int* n);
int pgmi_safetensors_entry(const char* path, int i, char* name, int name_cap, int* dtype, int64_t* shape4, int* ndim,
                           int64_t* begin, int64_t* end);
/* deterministic synthetic weights (benchmarks; oracle/wgen.c recipe) */
int pgmi_fill_synthetic(pgmi_ctx* ctx, const char* name, uint64_t key, float scale, float offset, void* stream);
uint64_t pgmi_synthetic_key(const char* name, uint64_t seed);
/* GemmaRotaryEmbedding.inv_freq (modeling_gemma.py:151), host fp32[head_dim/2]; default is
 * 1/theta^(2i/d) computed as the reference does. */
int pgmi_set_rope_inv_freq(pgmi_ctx* ctx, const float* inv_freq);
/* optional exact cos/sin table (bf16 [max_pos][head_dim/2]) as torch computes it (:178-185) */
int pgmi_set_rope_table(pgmi_ctx* ctx, const uint16_t* cos_tab, const uint16_t* sin_tab, int max_pos);
/* derived device tensors (padded patch-embedding matrix, RoPE table, workspace). Call after
 * the weights are in the slab and before the first forward; synchronises the device. */
int pgmi_prepare(pgmi_ctx* ctx);

/* ---- KV cache (KVCache, modeling_gemma.py:10-36): caller-owned slab
 * [layer][K|V][batch][max_tokens][kv_heads*head_dim] bf16 */
int64_t pgmi_kv_bytes(const pgmi_ctx* ctx, int batch, int max_tokens);

/* ---- forward pieces -------------------------------------------------------------------- */
/* SiglipVisionModel.forward (modeling_siglip.py:236-255) incl. the pixel cast of
 * modeling_gemma.py:570: pixels (B,C,H,W) fp32 or bf16 -> feats (B, N, v_hidden) bf16 */
int pgmi_vision(pgmi_ctx* ctx, const void* pixels, int pixel_dtype, int B, void* feats, void* stream);
/* PaliGemmaMultiModalProjector.forward (modeling_gemma.py:435-438): (rows, v_hidden) -> (rows, proj) */
int pgmi_project(pgmi_ctx* ctx, const void* feats, int rows, void* out, void* stream);
/* nn.Embedding lookup of GemmaModel.embed_tokens (modeling_gemma.py:565) */
int pgmi_embed(pgmi_ctx* ctx, const int64_t* ids, int rows, void* out, void* stream);
/* GemmaForCausalLM.forward (modeling_gemma.py:399-427) over the merged embeddings of
 * _merge_input_ids_with_image_features (modeling_gemma.py:468-537):
 *   ids (device int64 B x L) and image_feats (projected, n_img_rows x hidden, may be NULL) are
 *   merged on the device; if embeds != NULL they are used instead (already-merged embeddings,
 *   e.g. from a monkey-patched merge) and ids/image_feats are ignored.
 *   positions: HOST int64 B x L (rotary positions, modeling_gemma.py:516-535).
 *   KV: keys/values of the L tokens are written at rows kv_start.. of the caller's slab;
 *   attention covers rows [0, kv_start + L) (the reference's zero mask: non-causal).
 *   logits (device fp32): logits_rows == 0 -> (B, L, vocab); 1 -> (B, 1, vocab) last row only;
 *   2 -> (B, 1, vocab) as 1, and no row but the last needs its final hidden state (the generate
 *   loop, inference.py:55-63 takes logits[:, -1, :] only): the last layer writes every row's K/V,
 *   then runs attention, o_proj, the MLP and the final norm for the last row alone (row-wise ops,
 *   so the same values up to accumulation order); pgmi_lm_final_hidden then fails (PGMI_E_STATE). */
int pgmi_lm_forward(pgmi_ctx* ctx, const int64_t* ids, const void* image_feats, int n_img_rows, const void* embeds,
                    int B, int L, const int64_t* positions, void* kv, int kv_batch, int kv_max, int kv_start,
                    float* logits, int logits_rows, void* stream);
/* One KV-cached decode step for B sequences in lock-step (inference.py:56-78 loop body):
 *   ids (device int64 [B]), written at KV row kv_len, rotary position `position`
 *   (= attention_mask.cumsum(-1)[:, -1], modeling_gemma.py:526, i.e. kv_len + 1 after an
 *   inference.py prefill), attention over rows [0, kv_len]; logits (device fp32 [B][vocab]);
 *   next_ids (device int64 [B], may be NULL) = argmax (first max, torch.argmax semantics).
 *   use_graph != 0 replays a captured hipGraph of the whole step.  next_ids == ids feeds the
 *   argmax back in place (tokens are read first, the next ones written last): no staging copy. */
int pgmi_decode(pgmi_ctx* ctx, const int64_t* ids, int B, void* kv, int kv_batch, int kv_max, int kv_len,
                int position, float* logits, int64_t* next_ids, int use_graph, void* stream);
/* n_steps greedy decode steps back to back in one call (one hipGraph launch when use_graph != 0):
 * the generate loop of inference.py:56-78 without sampling, as Engine.generate runs it.  ids (device
 * int64 [B]) holds the input tokens and receives each step's argmax in place (step t + 1 reads step t's);
 * the steps write KV rows kv_len .. kv_len + n_steps - 1 at positions position .. position + n_steps - 1;
 * logits (device fp32 [B][vocab]) holds the last step's; tokens (device int64 [n_steps][B], may be
 * NULL) records every step's argmax.  Each step is pgmi_decode's step, kernel for kernel. */
int pgmi_decode_steps(pgmi_ctx* ctx, int64_t* ids, int B, void* kv, int kv_batch, int kv_max, int kv_len,
                      int position, int n_steps, float* logits, int64_t* tokens, int use_graph, void* stream);
/* The same decode step with already-merged input rows instead of token ids: embeds (device bf16
 * [B][hidden]) is the output of a caller's _merge_input_ids_with_image_features for a q_len == 1
 * step (the ablation harness monkey-patches the merge, ablation_study_fixed.py:99-142,335-337,
 * and then calls forward(input_ids=next_token, pixel_values=None, ...) per token, :215-221);
 * the rows are scaled by bf16(sqrt(hidden)) (GemmaModel, modeling_gemma.py:367-368) and run
 * through the same (graph-replayed) step.  The rows are staged into a context buffer first, so
 * the caller's buffer may change between calls. */
int pgmi_decode_embeds(pgmi_ctx* ctx, const void* embeds, int B, void* kv, int kv_batch, int kv_max, int kv_len,
                       int position, float* logits, int64_t* next_ids, int use_graph, void* stream);
/* pgmi_decode_embeds with the step's inputs left on the device (no host read of a merge's outputs):
 * position: the merge's (1, 1) position tensor (attention_mask.cumsum(-1)[:, -1:], modeling_gemma.py:526),
 * dtype PGMI_DTYPE_BF16 / _F32 or 10 = int64, 11 = int32, 12 = float64, rounded to the nearest integer;
 * mask (may be NULL): the merge's additive mask row over the kv_len + 1 keys (modeling_gemma.py:269),
 * bf16 (score + mask rounded to bf16) or fp32 (added in fp32, as torch promotes), row stride
 * mask_b_stride elements.  One sequence (B = 1). */
int pgmi_decode_embeds_dev(pgmi_ctx* ctx, const void* embeds, int B, void* kv, int kv_batch, int kv_max, int kv_len,
                           const void* position, int position_dtype, const void* mask, int mask_dtype,
                           int64_t mask_b_stride, float* logits, int64_t* next_ids, int use_graph, void* stream);
/* Prefill graphs (default on): pgmi_vision and pgmi_lm_forward replay a captured hipGraph when
 * called again with identical pointer and size arguments (the graph is captured on the second
 * such call; a replay reads the same addresses as the eager call would).  0 = always eager. */
int pgmi_set_prefill_graph(pgmi_ctx* ctx, int on);
/* Batched decode (B >= 3, MFMA projections) RMSNorm form: 0 = each input norm computed once per row
 * and read unstaged by the q|k|v / gate|up projections (default), 1 = staged inside each projection,
 * -1 = back to the default.  Same arithmetic either way (bf16 normalised rows);
 * drops captured decode graphs.  A tuning / test switch, no reference counterpart. */
int pgmi_set_decode_staged_norm(pgmi_ctx* ctx, int on);
/* lm_head + .float() of GemmaForCausalLM (modeling_gemma.py:417-418) over final-normed hidden
 * rows: logits (device fp32 [rows][vocab]) = fp32(bf16(normed . E^T)) with the tied embedding E.
 * Together with pgmi_lm_final_hidden this materialises the prefill's all-row logits on demand
 * after a last-row-only pgmi_lm_forward (SURVEY.md sec.7 hard part 3: lazy logits). */
int pgmi_lm_head(pgmi_ctx* ctx, const void* normed, int rows, float* logits, void* stream);
/* Copies the final RMSNorm output (GemmaModel.norm, modeling_gemma.py:379) of the B*L rows of the
 * last pgmi_lm_forward (bf16 [rows][hidden], row-major) into `out` (device memory). */
int pgmi_lm_final_hidden(pgmi_ctx* ctx, void* out, int rows, void* stream);

/* ---- replicas: the load-time weight broadcast over RCCL (xGMI).  The
 * reference has no multi-GPU path (accelerate placement only, utils.py:27-38).  One process per
 * GPU: the root calls pgmi_comm_unique_id, ships the PGMI_COMM_ID_BYTES bytes to every rank (any
 * channel), each rank calls pgmi_comm_init, then pgmi_broadcast_weights copies the root's whole
 * weight slab into every replica in one in-place ncclBroadcast; call pgmi_prepare afterwards.
 * A host that already owns an ncclComm_t passes it as `comm` directly. */
#define PGMI_COMM_ID_BYTES 128
int pgmi_comm_unique_id(void* id_out);
int pgmi_comm_init(int device, int nranks, int rank, const void* id, void** comm_out);
int pgmi_comm_destroy(void* comm);
int pgmi_broadcast_weights(pgmi_ctx* ctx, void* comm, int root, void* stream);

/* torch.argmax(logits, -1) over rows of a device fp32 [rows][V] matrix (inference.py:68) */
int pgmi_argmax(pgmi_ctx* ctx, const float* logits, int rows, int V, int64_t* out, void* stream);

/* Stop-token bookkeeping of the batched generate loop (inference.py:51,70-71, per row): rows with
 * finished[b] != 0 get next_ids[b] = pad_id; rows whose next_ids[b] == eos_id are marked finished
 * (their eos is kept, as the reference appends it before breaking).  n_alive (device int32, may be
 * NULL) receives the number of rows still running.  All pointers are device memory. */
int pgmi_eos_update(pgmi_ctx* ctx, int64_t* next_ids, int32_t* finished, int B, int64_t eos_id, int64_t pad_id,
                    int32_t* n_alive, void* stream);

/* Launch one decode kernel of `layer` on the context's decode workspace (benchmarking the
 * dominant kernel in isolation): 1 o_proj+residual, 2 RMSNorm+gate/up+GeGLU, 3 down+residual,
 * 4 final norm + lm_head (+argmax partials; layer ignored). */
int pgmi_decode_kernel(pgmi_ctx* ctx, int which, int layer, int B, void* stream);

/* Image preprocessing on the GPU (processing_paligemma.py:13-49, process_images): PIL-exact
 * BICUBIC resize of one decoded RGB image (uint8 HWC, device memory, H x W) to out_h x out_w,
 * then x/255 (float64 product cast to float32), (x - 0.5)/0.5 and HWC -> CHW, written to
 * `out_chw` (float32 [3][out_h][out_w], device) -- the reference's pixel_values for one image.
 * Uses the context's split-K scratch (stream-ordered with the prefill).  JPEG decode stays on
 * the host. */
int pgmi_preprocess(pgmi_ctx* ctx, const void* src_hwc, int H, int W, int out_h, int out_w, float* out_chw,
                    void* stream);

/* Launch one prefill GEMM of `layer` over `rows` rows of the context's prefill workspace
 * (benchmarking the MFMA path in isolation): 0 = gate|up GEMM + GeGLU epilogue
 * (modeling_gemma.py:134), 1 = down projection (split-K partials, as the prefill runs it). */
int pgmi_prefill_kernel(pgmi_ctx* ctx, int which, int layer, int rows, void* stream);

/* In-situ timing probe of the prefill MLP GEMMs (measurement only): on != 0 makes every following
 * pgmi_lm_forward eager (prefill graphs off) and times each layer's gate|up + GeGLU GEMM and down
 * GEMM kernel (modeling_gemma.py:133-134) with its own start / stop events (hipExtLaunchKernelGGL: the
 * kernel's execution alone); pgmi_prefill_probe_times writes the last probed
 * forward's durations in microseconds: us[i] = layer i's gate|up, us[layers + i] = its down.  on = 0
 * restores the graphs.  Probe with logits_rows 0 or 1: under logits_rows 2 the last layer's MLP runs on the
 * decode GEMVs (no GEMM to time) and pgmi_prefill_probe_times returns PGMI_E_HIP (the unset events). */
int pgmi_prefill_probe(pgmi_ctx* ctx, int on);
int pgmi_prefill_probe_times(pgmi_ctx* ctx, float* us, int n);
/* Tuning hook: force the prefill GEMM tile configuration and split-K factor for subsequent
 * calls (kernels_gemm.hip enum Cfg: 0-5 register-staged tiles, 6-29 LDS-DMA panel tiles, 30-35 warp-specialised panel tiles);
 * cfg < 0 restores the automatic (measured) plan. */
int pgmi_tune_gemm(int cfg, int split);
/* Tuning hook: the same for ONE GEMM shape (M x N x K, dual = the gate|up GeGLU form) while every
 * other shape keeps its plan (in-situ sweeps of a whole forward); cfg < 0 removes the override.
 * Split-K partials that a consumer reduces (out_proj, fc2, down: the residual + norm kernel) are
 * limited to 16 slabs. */
int pgmi_tune_gemm_shape(int M, int N, int K, int dual, int cfg, int split);

/* Test hook: the workgroup -> (row tile, column tile, K slice) order of a panel / 8-phase prefill GEMM
 * launch of n_mt x n_nt tiles x S K slices (tile BM x BN, K deep), as the kernels compute it (the XCD
 * block raster of kernels_gemm.hip xcd_tile); mt/nt/z receive n_mt*n_nt*S entries indexed by the linear
 * workgroup id.  Returns the XCD block code the launch uses (0 = run order); no device needed. */
int pgmi_debug_gemm_tiles(int n_mt, int n_nt, int S, int BM, int BN, int K, int* mt, int* nt, int* z);

/* Tuning hook: force the prefill attention kernel (kernels_attn.hip): 0 = 16-row kernel with
 * LDS-resident scores, 7 = one pass with K/V loaded once and scores in registers (head_dim 72, <= 256 keys),
 * 8 = the same 16-row kernel with every K/V load issued up front (head_dim 256, <= 320 keys), RK = K/V-tiled two-pass kernel with R row groups and K key-split groups
 * per workgroup (41, 42, 21, 22; 44, 24 for head_dim 72); 9 = one pass with the keys split over workgroups
 * (online softmax, fp32 partials merged by a combine kernel), 91 / 92 / 94 = the same with 1 / 2 / 4 key
 * ranges; -1 restores the measured choice. */
int pgmi_tune_attention(int variant);

/* Nucleus sampling, inference.py:15-24 (_sample_top_p) with inference.py:65's
 * softmax(logits / temperature) fused when temperature > 0 (temperature <= 0: x already holds
 * the probabilities, _sample_top_p's own input).  x: device fp32 [rows][V]; u: device fp32
 * [rows] uniforms in [0, 1) that replace torch.multinomial's internal draw (the token is the
 * first position of the descending order whose cumulative kept mass exceeds u * Z; equal
 * probabilities in index order); out: device int64 [rows]; kept_mass (device fp32 [rows], may
 * be NULL): Z, the renormalisation mass of :21.  Scratch: the context's split-K workspace. */
int pgmi_sample_top_p(pgmi_ctx* ctx, const float* x, int rows, int V, float temperature, float top_p,
                      const float* u, int64_t* out, float* kept_mass, void* stream);

/* ---- single-op entry points (kernel-level parity tests) ---------------------------------- */
/* out = epilogue(A[M,K] . W[N,K]^T): epi 0 store, 1 +bias, 2 +bias,gelu, 3 +bias,+res, 4 +res,
 * 6 fp32 out (out is float*), 7 GeGLU with up rows at W + N*K */
int pgmi_op_gemm(pgmi_ctx* ctx, const void* A, const void* W, int M, int N, int K, int epi, const void* bias,
                 const void* res, void* out, void* stream);
/* pgmi_op_gemm with explicit row strides (elements, multiples of 8, >= K) of A and W: the prefill GEMMs'
 * sensitivity to the operands' row pitch (tools/probes/stride_probe.py). */
int pgmi_op_gemm_strided(pgmi_ctx* ctx, const void* A, int lda, const void* W, int ldw, int M, int N, int K, int epi,
                         const void* bias, const void* res, void* out, void* stream);
int pgmi_op_rmsnorm(pgmi_ctx* ctx, const void* x, const void* w, int rows, int D, float eps, void* out,
                    void* stream);
int pgmi_op_layernorm(pgmi_ctx* ctx, const void* x, const void* w, const void* b, int rows, int D, float eps,
                      void* out, void* stream);
/* out = bf16(a + b) elementwise over n bf16 values (n a multiple of 8): the residual adds of the per-layer
 * module forwards (SiglipEncoderLayer.forward modeling_siglip.py:189,202; GemmaDecoderLayer :327,336) */
int pgmi_op_add(pgmi_ctx* ctx, const void* a, const void* b, int64_t n, void* out, void* stream);
/* SiglipVisionEmbeddings.forward (modeling_siglip.py:62-79) on given parameters: pixels (B, C, H, H)
 * bf16 or fp32 (pixel_dtype), conv weight [D][C][P][P] + bias [D], position embedding [(H/P)^2][D]
 * -> out (B, (H/P)^2, D) bf16 = bf16(bf16(conv + bias) + pos); uses the context's scratch */
int pgmi_op_patch_embed(pgmi_ctx* ctx, const void* pixels, int pixel_dtype, int B, int C, int H, int P,
                        const void* conv_w, const void* conv_b, const void* pos, int D, void* out, void* stream);
/* attention over q (B, Lq, H, hd), k/v (B, Lk, Hkv, hd) -> o (B, Lq, H, hd), all contiguous bf16;
 * s = bf16(bf16(q.k) * scale) */
int pgmi_op_attention(pgmi_ctx* ctx, const void* q, const void* k, const void* v, void* o, int B, int Lq, int Lk,
                      int H, int Hkv, int head_dim, float scale, void* stream);
/* Reference-order attention of the module forwards (SiglipAttention.forward modeling_siglip.py:116-131,
 * GemmaAttention.forward modeling_gemma.py:262-277), returning the probability matrix the reference
 * returns as its second output:
 *   s = bf16(q.k); s = bf16(s * scale) (scale_div 0) or bf16(s / scale) (scale_div 1, Gemma's
 *   "/ math.sqrt(head_dim)"); + mask (additive, optional: bf16 -> bf16(s + m), fp32 -> s + m in fp32,
 *   as torch promotes); p = bf16(softmax_fp32(s)); o = bf16(p.v).  q/o (B, Lq, H, hd); k/v
 *   (B, Lk, Hkv, hd) for kv_layout 0 or (B, Hkv, Lk, hd) for kv_layout 1 (the KVCache layout);
 *   query head h reads KV head h / (H / Hkv) (repeat_kv, :136-141).  mask element (b, h, i, j) at
 *   b*m_b_stride + h*m_h_stride + i*m_q_stride + j (a stride of 0 broadcasts).  probs (B, H, Lq, Lk)
 *   bf16, may be NULL.  hd <= 256. */
int pgmi_op_attention_ex(pgmi_ctx* ctx, const void* q, const void* k, const void* v, void* o, int B, int Lq, int Lk,
                         int H, int Hkv, int head_dim, int kv_layout, float scale, int scale_div, const void* mask,
                         int mask_dtype, int64_t m_b_stride, int64_t m_h_stride, int64_t m_q_stride, void* probs,
                         void* stream);
/* apply_rotary_pos_emb for one projection (modeling_gemma.py:187-199) with the caller's cos/sin rows
 * (GemmaRotaryEmbedding.forward's output, :155-185): x (rows, heads*hd) -> out = bf16(bf16(x*cos) +
 * bf16(rotate_half(x)*sin)), cos/sin bf16 (rows, hd). */
int pgmi_op_rope(pgmi_ctx* ctx, const void* x, const void* cos_rows, const void* sin_rows, int64_t rows, int heads,
                 int head_dim, void* out, void* stream);
/* out = bf16(x * a) over n bf16 values (n a multiple of 8): GemmaModel's normalizer (modeling_gemma.py:367-368) */
int pgmi_op_scale(pgmi_ctx* ctx, const void* x, float a, int64_t n, void* out, void* stream);
/* decode GEMV family on one layer's weights (tests): y[b][n] += W x (residual form) */
int pgmi_op_gemv_res(pgmi_ctx* ctx, const void* x, const void* W, int B, int N, int K, void* h_inout,
                     void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PGMI_H */
