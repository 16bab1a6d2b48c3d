// engine.hip -- libpgmi host side: weight layout, workspaces, forward orchestration, hipGraph
// decode, and the extern "C" ABI declared in include/pgmi.h.
//
// Orchestration restates the reference's call stacks:
//   vision   SiglipVisionTransformer.forward   modeling_siglip.py:236-244
//   lm       GemmaModel/GemmaForCausalLM        modeling_gemma.py:357-427
//   decode   one inference.py loop iteration    inference.py:56-78
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

#include <dlfcn.h>

#include <rccl/rccl.h>  // types only: librccl is dlopen'ed on first use

#include "../../include/pgmi.h"
#include "common.h"
#include "launch.h"
#include "safetensors_hdr.h"

using namespace pgmi;

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(expr)                                                                       \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess) return fail(PGMI_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

#define LAUNCHCHK()                                                                        \
    do {                                                                                   \
        hipError_t e_ = hipGetLastError();                                                 \
        if (e_ != hipSuccess) return fail(PGMI_E_HIP, std::string("kernel launch: ") + hipGetErrorString(e_)); \
    } while (0)

struct Slot {
    std::string name;
    int64_t off;
    int64_t shape[4];
    int ndim;
    int64_t numel;
};

struct GraphKey {
    int B;
    void* kv;
    int kv_batch, kv_max;
    float* logits;
    int64_t* next;
    const int64_t* ids;  // the ids buffer the graph reads (the context's staging copy, or in place)
    bool emb;            // the step's input is the staged embedding rows (pgmi_decode_embeds), not ids
    int masked;          // 0: no mask (a zero word), 1: staged bf16 mask (sum rounded), 2: staged fp32 mask
    int n_steps;         // decode steps captured back to back (pgmi_decode_steps; 1 otherwise)
    int64_t* tokens;     // their per-step token record ([n_steps][B], may be null)
    bool operator<(const GraphKey& o) const {
        return std::tie(B, kv, kv_batch, kv_max, logits, next, ids, emb, masked, n_steps, tokens) <
               std::tie(o.B, o.kv, o.kv_batch, o.kv_max, o.logits, o.next, o.ids, o.emb, o.masked, o.n_steps,
                        o.tokens);
    }
};

struct GraphEntry {
    int seen = 0;
    hipGraphExec_t exec = nullptr;
};

struct pgmi_ctx {
    pgmi_config c;
    int device;
    std::vector<Slot> slots;
    std::unordered_map<std::string, int> index;
    int64_t slab_bytes = 0;
    uint8_t* slab = nullptr;
    std::vector<float> inv_freq;
    std::vector<uint16_t> host_cos, host_sin;  // optional exact table
    bool prepared = false;
    std::vector<void*> allocs;
    // derived
    uint16_t* patch_w = nullptr;  // [v_hidden][kpad]
    int kpad = 0;
    uint16_t* cosT = nullptr;
    uint16_t* sinT = nullptr;
    // text prefill workspace (rows = max_batch*max_seq)
    uint16_t *Hs, *Tn, *QKV, *Qr, *AO, *ACT, *lastrows;
    long tn_rows = 0;  // rows of Tn holding the final RMSNorm of the last pgmi_lm_forward (pgmi_lm_final_hidden)
    int64_t* dpos;
    int64_t* dids_tmp;
    // vision workspace (rows = max_batch*N)
    uint16_t *vX, *vT, *vQKV, *vAO, *vH, *vP;
    float* ws;
    size_t ws_bytes;
    // decode workspace
    uint16_t *dH, *dQ, *dAO, *dACT;
    uint16_t* dHn;  // batched decode (B >= 3): the RMSNorm'd rows the unstaged MFMA projections read
    float* dSS;     // batched decode: o_proj's 16-column partial sums of squares of h, [B][H / 16]
    // batched decode (max_batch >= 3): fragment-major images of every layer's gate|up, q|k|v (in the GEMV's row
    // order), o_proj and down weights (mf_swizzle), [layer][gate|up 2 I x H | q|k|v QKVN x H | o_proj | down H x I]
    uint16_t* mfw = nullptr;
    size_t mfw_layer = 0;
    bool mfw_dirty = false;  // the fragment-major images are (re)built by the next batched decode step
    float *opart, *pmax, *dlogits, *amax_v;
    int *pidx, *amax_i;
    int max_chunks;
    StepState* step;
    StepState* pstep;  // the generate-loop prefill's last-row attention (flash-decoding over the prompt's keys)
    int64_t* d_ids;
    uint16_t* d_emb;             // staged input rows of pgmi_decode_embeds ([max_batch][hidden] bf16)
    float* d_mask;               // staged additive decode mask ([max_batch][max_kv] fp32, pgmi_decode_embeds_dev)
    float* d_zero;               // one zero word: the "no mask" mask of the decode attention
    int64_t* d_next;             // argmax target when the caller passes none
    unsigned* lm_done;           // lm_head arrival counter (argmax folded into its last workgroup)
    hipStream_t cap_stream = nullptr;
    std::map<GraphKey, GraphEntry> graphs;
    // prefill graphs (vision tower, language-model forward): replayed for repeated calls with
    // identical pointer/shape arguments (a replay is the eager call: kernels read the same
    // addresses at run time), captured on the second such call
    bool prefill_graph = true;
    int mf_staged = -1;  // batched decode RMSNorm form (mf_staged()); -1 = default (unstaged)
    // device step state as the last enqueued per-phase decode step leaves it (advanced in-graph)
    bool step_known = false;
    int step_kv = 0, step_pos = 0;
    std::map<std::vector<intptr_t>, GraphEntry> pgraphs;
    // in-situ timing probe of the prefill MLP GEMMs (pgmi_prefill_probe): events around layer i's gate|up
    // GEMM (ev[4i], ev[4i+1]) and down GEMM (ev[4i+2], ev[4i+3]) of eager forwards
    std::vector<hipEvent_t> probe_ev;
    bool probe_on = false;
    bool graph_before_probe = true;  // prefill_graph as the caller left it before the probe turned it off
};

namespace {

void clear_pgraphs(pgmi_ctx* x) {
    for (auto& kv : x->pgraphs)
        if (kv.second.exec) (void)hipGraphExecDestroy(kv.second.exec);
    x->pgraphs.clear();
}

// the captured decode steps
void clear_dgraphs(pgmi_ctx* x) {
    for (auto& kv : x->graphs)
        if (kv.second.exec) (void)hipGraphExecDestroy(kv.second.exec);
    x->graphs.clear();
}

int n_img(const pgmi_config& c) { return (c.v_image / c.v_patch) * (c.v_image / c.v_patch); }

void add_slot(pgmi_ctx* x, const std::string& name, std::initializer_list<int64_t> shape) {
    Slot s;
    s.name = name;
    s.ndim = (int)shape.size();
    s.numel = 1;
    int i = 0;
    for (int64_t d : shape) { s.shape[i++] = d; s.numel *= d; }
    for (; i < 4; ++i) s.shape[i] = 1;
    s.off = x->slab_bytes;
    x->slab_bytes += (s.numel * 2 + 255) / 256 * 256;
    x->index[name] = (int)x->slots.size();
    x->slots.push_back(s);
}

// Slab layout: the reference state-dict tensors, ordered so that the projections that are
// fused into one GEMM/GEMV are adjacent (q|k|v weights and biases, gate|up).
void build_layout(pgmi_ctx* x) {
    const pgmi_config& c = x->c;
    const int64_t D = c.v_hidden, I = c.v_intermediate, P = c.v_patch, C = c.v_channels, N = n_img(c);
    const std::string vp = "vision_tower.vision_model.";
    add_slot(x, vp + "embeddings.patch_embedding.weight", {D, C, P, P});
    add_slot(x, vp + "embeddings.patch_embedding.bias", {D});
    add_slot(x, vp + "embeddings.position_embedding.weight", {N, D});
    for (int i = 0; i < c.v_layers; ++i) {
        const std::string lp = vp + "encoder.layers." + std::to_string(i) + ".";
        for (const char* nm : {"q_proj", "k_proj", "v_proj"}) add_slot(x, lp + "self_attn." + nm + ".weight", {D, D});
        for (const char* nm : {"q_proj", "k_proj", "v_proj"}) add_slot(x, lp + "self_attn." + nm + ".bias", {D});
        add_slot(x, lp + "self_attn.out_proj.weight", {D, D});
        add_slot(x, lp + "self_attn.out_proj.bias", {D});
        add_slot(x, lp + "layer_norm1.weight", {D});
        add_slot(x, lp + "layer_norm1.bias", {D});
        add_slot(x, lp + "mlp.fc1.weight", {I, D});
        add_slot(x, lp + "mlp.fc1.bias", {I});
        add_slot(x, lp + "mlp.fc2.weight", {D, I});
        add_slot(x, lp + "mlp.fc2.bias", {D});
        add_slot(x, lp + "layer_norm2.weight", {D});
        add_slot(x, lp + "layer_norm2.bias", {D});
    }
    add_slot(x, vp + "post_layernorm.weight", {D});
    add_slot(x, vp + "post_layernorm.bias", {D});
    add_slot(x, "multi_modal_projector.linear.weight", {c.projection_dim, D});
    add_slot(x, "multi_modal_projector.linear.bias", {c.projection_dim});
    const int64_t H = c.t_hidden, TI = c.t_intermediate, V = c.t_vocab, HD = c.t_head_dim;
    add_slot(x, "language_model.model.embed_tokens.weight", {V, H});
    for (int i = 0; i < c.t_layers; ++i) {
        const std::string lp = "language_model.model.layers." + std::to_string(i) + ".";
        add_slot(x, lp + "self_attn.q_proj.weight", {c.t_heads * HD, H});
        add_slot(x, lp + "self_attn.k_proj.weight", {c.t_kv_heads * HD, H});
        add_slot(x, lp + "self_attn.v_proj.weight", {c.t_kv_heads * HD, H});
        add_slot(x, lp + "self_attn.o_proj.weight", {H, c.t_heads * HD});
        add_slot(x, lp + "mlp.gate_proj.weight", {TI, H});
        add_slot(x, lp + "mlp.up_proj.weight", {TI, H});
        add_slot(x, lp + "mlp.down_proj.weight", {H, TI});
        add_slot(x, lp + "input_layernorm.weight", {H});
        add_slot(x, lp + "post_attention_layernorm.weight", {H});
    }
    add_slot(x, "language_model.model.norm.weight", {H});
}

inline uint16_t* W(pgmi_ctx* x, const std::string& name) {
    auto it = x->index.find(name);
    if (it == x->index.end()) return nullptr;
    return reinterpret_cast<uint16_t*>(x->slab + x->slots[it->second].off);
}

inline uint16_t* VL(pgmi_ctx* x, int i, const char* suffix) {
    return W(x, "vision_tower.vision_model.encoder.layers." + std::to_string(i) + "." + suffix);
}
inline uint16_t* TL(pgmi_ctx* x, int i, const char* suffix) {
    return W(x, "language_model.model.layers." + std::to_string(i) + "." + suffix);
}

uint16_t host_f2bf(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

float bf16_round_host(float f) {
    uint32_t u = (uint32_t)host_f2bf(f) << 16;
    float r;
    std::memcpy(&r, &u, 4);
    return r;
}

uint64_t fnv1a(const char* s) {
    uint64_t h = 0xCBF29CE484222325ULL;
    for (const unsigned char* p = (const unsigned char*)s; *p; ++p) { h ^= *p; h *= 0x100000001B3ULL; }
    return h;
}

uint64_t splitmix64_h(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

__global__ void k_convert(const void* src, int dtype, long n, uint16_t* dst) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        if (dtype == PGMI_DTYPE_F32) dst[i] = f2bf(reinterpret_cast<const float*>(src)[i]);
        else dst[i] = f2bf((float)reinterpret_cast<const _Float16*>(src)[i]);
    }
}

int dalloc(pgmi_ctx* x, void** p, size_t bytes) {
    if (bytes == 0) bytes = 256;
    hipError_t e = hipMalloc(p, bytes);
    if (e != hipSuccess) return fail(PGMI_E_NOMEM, std::string("hipMalloc ") + std::to_string(bytes) + ": " + hipGetErrorString(e));
    x->allocs.push_back(*p);
    return 0;
}

template <typename T>
int dalloc_t(pgmi_ctx* x, T** p, size_t count) {
    return dalloc(x, reinterpret_cast<void**>(p), count * sizeof(T));
}

// RoPE tables: freqs = fp32(pos * inv_freq) (modeling_gemma.py:178), cos/sin in fp32 (:182-183),
// cast to bf16 (:185).  cos/sin of the fp32 angle are evaluated in double and rounded once.
void build_rope_host(pgmi_ctx* x, std::vector<uint16_t>& cs, std::vector<uint16_t>& sn) {
    const int half = x->c.t_head_dim / 2, mp = x->c.t_max_pos;
    cs.resize((size_t)mp * half);
    sn.resize((size_t)mp * half);
    for (int p = 0; p < mp; ++p)
        for (int i = 0; i < half; ++i) {
            const float ang = (float)p * x->inv_freq[i];
            cs[(size_t)p * half + i] = host_f2bf((float)std::cos((double)ang));
            sn[(size_t)p * half + i] = host_f2bf((float)std::sin((double)ang));
        }
}

int ensure_prepared(pgmi_ctx* x) {
    if (!x->prepared) return fail(PGMI_E_STATE, "pgmi_prepare() has not been called");
    if (!x->slab) return fail(PGMI_E_STATE, "weights are not bound (pgmi_bind_weights)");
    return 0;
}

}  // namespace

// ================================================================ C ABI
// RCCL is loaded on first use (dlopen), so a single-GPU process -- and the CPU tests that only load
// the library -- need no librccl; the four entry points it uses are resolved once.
namespace {
struct Rccl {
    void* h = nullptr;
    std::string why;  // dlerror() of the failed load
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
};

// thread-safe one-time load (a function-local static is initialised exactly once)
Rccl& rccl() {
    static Rccl r = [] {
        Rccl t;
        for (const char* n : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            if ((t.h = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
            const char* e = dlerror();
            if (e) t.why = e;
        }
        if (t.h) {
            t.get_unique_id = reinterpret_cast<decltype(t.get_unique_id)>(dlsym(t.h, "ncclGetUniqueId"));
            t.comm_init_rank = reinterpret_cast<decltype(t.comm_init_rank)>(dlsym(t.h, "ncclCommInitRank"));
            t.comm_destroy = reinterpret_cast<decltype(t.comm_destroy)>(dlsym(t.h, "ncclCommDestroy"));
            t.broadcast = reinterpret_cast<decltype(t.broadcast)>(dlsym(t.h, "ncclBroadcast"));
            t.error_string = reinterpret_cast<decltype(t.error_string)>(dlsym(t.h, "ncclGetErrorString"));
        }
        return t;
    }();
    return r;
}
}  // namespace

extern "C" {

const char* pgmi_last_error(void) { return g_err.c_str(); }
const char* pgmi_version(void) { return "pgmi 0.1.0 (gfx950)"; }

int pgmi_create(int device, const pgmi_config* cfg, pgmi_ctx** out) {
    if (!cfg || !out) return fail(PGMI_E_ARG, "null argument");
    const pgmi_config& c = *cfg;
    if (c.t_head_dim != 256) return fail(PGMI_E_ARG, "head_dim must be 256 (Gemma)");
    if (c.t_hidden != 2048) return fail(PGMI_E_ARG, "text hidden must be 2048 (decode kernels are specialised)");
    if (c.t_intermediate % 8 != 0 || c.v_intermediate % 8 != 0) return fail(PGMI_E_ARG, "intermediate sizes must be multiples of 8");
    if (c.v_hidden % c.v_heads != 0 || c.v_hidden / c.v_heads != 72) return fail(PGMI_E_ARG, "SigLIP head_dim must be 72");
    if (c.t_kv_heads != 1 || c.t_heads > 8)
        return fail(PGMI_E_ARG, "decode path is specialised for MQA with <= 8 query heads (num_key_value_heads = 1)");
    if (c.max_batch < 1 || c.max_batch > 8) return fail(PGMI_E_ARG, "max_batch must be in [1, 8]");
    if (c.v_hidden > 4096) return fail(PGMI_E_ARG, "v_hidden too large for the LayerNorm kernel");
    auto* x = new pgmi_ctx();
    x->c = c;
    if (x->c.max_kv <= 0) x->c.max_kv = c.t_max_pos;
    x->device = device;
    build_layout(x);
    x->inv_freq.resize(c.t_head_dim / 2);
    for (int i = 0; i < c.t_head_dim / 2; ++i) {
        // 1.0 / (base ** (arange(0, dim, 2).float() / dim)), fp32 (modeling_gemma.py:151)
        const float e = (float)(2 * i) / (float)c.t_head_dim;
        const float p = (float)std::pow((double)c.t_rope_theta, (double)e);
        x->inv_freq[i] = 1.0f / p;
    }
    *out = x;
    return 0;
}

int pgmi_destroy(pgmi_ctx* x) {
    if (x)
        for (auto& e : x->probe_ev) (void)hipEventDestroy(e);
    if (!x) return 0;
    clear_dgraphs(x);
    clear_pgraphs(x);
    for (void* p : x->allocs) (void)hipFree(p);
    if (x->cap_stream) (void)hipStreamDestroy(x->cap_stream);
    delete x;
    return 0;
}

int64_t pgmi_weights_bytes(const pgmi_ctx* x) { return x ? x->slab_bytes : -1; }
int pgmi_weight_count(const pgmi_ctx* x) { return x ? (int)x->slots.size() : -1; }

int pgmi_weight_info(const pgmi_ctx* x, int idx, const char** name, int64_t* off, int64_t* shape4, int* ndim) {
    if (!x || idx < 0 || idx >= (int)x->slots.size()) return fail(PGMI_E_ARG, "weight index out of range");
    const Slot& s = x->slots[idx];
    if (name) *name = s.name.c_str();
    if (off) *off = s.off;
    if (shape4) for (int i = 0; i < 4; ++i) shape4[i] = s.shape[i];
    if (ndim) *ndim = s.ndim;
    return 0;
}

int pgmi_bind_weights(pgmi_ctx* x, void* slab) {
    if (!x || !slab) return fail(PGMI_E_ARG, "null argument");
    if (reinterpret_cast<uintptr_t>(slab) % 256 != 0) return fail(PGMI_E_ARG, "weight slab must be 256-byte aligned");
    x->slab = reinterpret_cast<uint8_t*>(slab);
    clear_dgraphs(x);
    clear_pgraphs(x);
    return 0;
}

int pgmi_load_weight(pgmi_ctx* x, const char* name, const void* src, int dtype, int on_device, void* stream) {
    if (!x || !name || !src) return fail(PGMI_E_ARG, "null argument");
    if (!x->slab) return fail(PGMI_E_STATE, "weights are not bound");
    auto it = x->index.find(name);
    if (it == x->index.end()) return fail(PGMI_E_ARG, std::string("unknown weight ") + name);
    const Slot& s = x->slots[it->second];
    uint16_t* dst = reinterpret_cast<uint16_t*>(x->slab + s.off);
    hipStream_t st = (hipStream_t)stream;
    HIPCHK(hipSetDevice(x->device));
    if (dtype == PGMI_DTYPE_BF16) {
        HIPCHK(hipMemcpyAsync(dst, src, s.numel * 2, on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, st));
    } else if (dtype == PGMI_DTYPE_F32 || dtype == PGMI_DTYPE_F16) {
        if (on_device) {
            hipLaunchKernelGGL(k_convert, dim3(1024), dim3(256), 0, st, src, dtype, (long)s.numel, dst);
            LAUNCHCHK();
        } else {
            std::vector<uint16_t> tmp(s.numel);
            for (int64_t i = 0; i < s.numel; ++i) {
                float f = dtype == PGMI_DTYPE_F32 ? reinterpret_cast<const float*>(src)[i]
                                                 : (float)reinterpret_cast<const _Float16*>(src)[i];
                tmp[i] = host_f2bf(f);
            }
            HIPCHK(hipMemcpyAsync(dst, tmp.data(), s.numel * 2, hipMemcpyHostToDevice, st));
            HIPCHK(hipStreamSynchronize(st));
        }
    } else {
        return fail(PGMI_E_ARG, "unsupported dtype");
    }
    return 0;
}

int pgmi_safetensors_count(const char* path, int* n) {
    if (!path || !n) return fail(PGMI_E_ARG, "null argument");
    StFile f;
    if (!st_open(path, f)) return fail(PGMI_E_ARG, f.error);
    *n = (int)f.entries.size();
    return 0;
}

int pgmi_safetensors_entry(const char* path, int i, char* name, int name_cap, int* dtype, int64_t* shape4, int* ndim,
                           int64_t* begin, int64_t* end) {
    if (!path || !name || name_cap < 1 || !dtype || !shape4 || !ndim || !begin || !end)
        return fail(PGMI_E_ARG, "null argument");
    StFile f;
    if (!st_open(path, f)) return fail(PGMI_E_ARG, f.error);
    if (i < 0 || i >= (int)f.entries.size()) return fail(PGMI_E_ARG, "entry index out of range");
    const StEntry& e = f.entries[i];
    std::snprintf(name, (size_t)name_cap, "%s", e.name.c_str());
    *dtype = e.dtype == "BF16" ? PGMI_DTYPE_BF16 : e.dtype == "F16" ? PGMI_DTYPE_F16 : e.dtype == "F32" ? PGMI_DTYPE_F32 : -1;
    *ndim = (int)e.shape.size();
    for (int d = 0; d < 4; ++d) shape4[d] = d < *ndim ? e.shape[d] : 0;
    *begin = e.begin;
    *end = e.end;
    return 0;
}

// utils.py:19-44 (safe_open shard loop + load_state_dict(strict=False)) for one shard: tensors
// named like slab weights are shape-checked, converted to bf16 and written into the slab; BF16
// bytes go host -> slab directly from the mapped file, F32/F16 through the split-K scratch in
// chunks and a device-side RNE conversion.  Synchronises the stream before unmapping.
int pgmi_load_safetensors(pgmi_ctx* x, const char* path, int* n_loaded, int* n_skipped, void* stream) {
    if (!x || !path) return fail(PGMI_E_ARG, "null argument");
    if (!x->slab) return fail(PGMI_E_STATE, "weights are not bound");
    HIPCHK(hipSetDevice(x->device));
    StFile f;
    if (!st_open(path, f)) return fail(PGMI_E_ARG, f.error);
    hipStream_t st = (hipStream_t)stream;
    // scratch for conversions: the context's workspace if prepared, else a temporary buffer
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    uint8_t* scratch = reinterpret_cast<uint8_t*>(x->ws);
    size_t scratch_bytes = x->ws ? x->ws_bytes : 0;
    int loaded = 0, skipped = 0;
    int rc = 0;
    for (const StEntry& e : f.entries) {
        auto it = x->index.find(e.name);
        if (it == x->index.end()) {
            ++skipped;
            continue;
        }
        const Slot& sl = x->slots[it->second];
        bool same = (int)e.shape.size() == sl.ndim;
        for (int d = 0; same && d < sl.ndim; ++d) same = e.shape[d] == sl.shape[d];
        if (!same) {
            rc = fail(PGMI_E_ARG, "shape mismatch for " + e.name);
            break;
        }
        const int eb = st_elem_bytes(e.dtype);
        if (eb == 0) {
            rc = fail(PGMI_E_ARG, "unsupported dtype " + e.dtype + " for " + e.name);
            break;
        }
        if (e.end - e.begin != sl.numel * eb) {
            rc = fail(PGMI_E_ARG, "byte size mismatch for " + e.name);
            break;
        }
        const uint8_t* src = f.map + f.data0 + e.begin;
        uint16_t* dst = reinterpret_cast<uint16_t*>(x->slab + sl.off);
        if (e.dtype == "BF16") {
            if (hipMemcpyAsync(dst, src, (size_t)sl.numel * 2, hipMemcpyHostToDevice, st) != hipSuccess) {
                rc = fail(PGMI_E_HIP, "upload of " + e.name);
                break;
            }
        } else {
            const int dt = e.dtype == "F32" ? PGMI_DTYPE_F32 : PGMI_DTYPE_F16;
            if (scratch_bytes < ((size_t)8 << 20)) {
                if (!tmp) {
                    tmp_bytes = (size_t)64 << 20;
                    if (hipMalloc(&tmp, tmp_bytes) != hipSuccess) {
                        rc = fail(PGMI_E_NOMEM, "conversion scratch");
                        break;
                    }
                }
                scratch = reinterpret_cast<uint8_t*>(tmp);
                scratch_bytes = tmp_bytes;
            }
            const int64_t per = (int64_t)(scratch_bytes / (size_t)eb);
            for (int64_t i0 = 0; i0 < sl.numel && rc == 0; i0 += per) {
                const int64_t n = std::min<int64_t>(per, sl.numel - i0);
                if (hipMemcpyAsync(scratch, src + i0 * eb, (size_t)n * eb, hipMemcpyHostToDevice, st) != hipSuccess) {
                    rc = fail(PGMI_E_HIP, "upload of " + e.name);
                    break;
                }
                hipLaunchKernelGGL(k_convert, dim3(1024), dim3(256), 0, st, scratch, dt, (long)n, dst + i0);
            }
            if (rc) break;
        }
        ++loaded;
    }
    const hipError_t se = hipStreamSynchronize(st);  // the mapped bytes must outlive the copies
    if (tmp) (void)hipFree(tmp);
    if (rc) return rc;
    if (se != hipSuccess) return fail(PGMI_E_HIP, std::string("safetensors upload: ") + hipGetErrorString(se));
    x->prepared = false;  // derived tensors (padded patch matrix, ...) are rebuilt by pgmi_prepare
    if (n_loaded) *n_loaded = loaded;
    if (n_skipped) *n_skipped = skipped;
    return 0;
}

uint64_t pgmi_synthetic_key(const char* name, uint64_t seed) { return splitmix64_h(seed ^ fnv1a(name)); }

int pgmi_fill_synthetic(pgmi_ctx* x, const char* name, uint64_t key, float scale, float offset, void* stream) {
    if (!x || !name) return fail(PGMI_E_ARG, "null argument");
    if (!x->slab) return fail(PGMI_E_STATE, "weights are not bound");
    auto it = x->index.find(name);
    if (it == x->index.end()) return fail(PGMI_E_ARG, std::string("unknown weight ") + name);
    const Slot& s = x->slots[it->second];
    HIPCHK(hipSetDevice(x->device));
    fill_synthetic((hipStream_t)stream, reinterpret_cast<uint16_t*>(x->slab + s.off), (long)s.numel, key, scale, offset);
    LAUNCHCHK();
    return 0;
}

int pgmi_set_rope_inv_freq(pgmi_ctx* x, const float* inv) {
    if (!x || !inv) return fail(PGMI_E_ARG, "null argument");
    for (int i = 0; i < x->c.t_head_dim / 2; ++i) x->inv_freq[i] = inv[i];
    x->host_cos.clear();
    x->host_sin.clear();
    x->prepared = false;
    return 0;
}

int pgmi_set_rope_table(pgmi_ctx* x, const uint16_t* cs, const uint16_t* sn, int max_pos) {
    if (!x || !cs || !sn) return fail(PGMI_E_ARG, "null argument");
    if (max_pos != x->c.t_max_pos) return fail(PGMI_E_ARG, "rope table must cover max_position_embeddings");
    const size_t n = (size_t)max_pos * (x->c.t_head_dim / 2);
    x->host_cos.assign(cs, cs + n);
    x->host_sin.assign(sn, sn + n);
    x->prepared = false;
    return 0;
}

int pgmi_prepare(pgmi_ctx* x) {
    if (!x) return fail(PGMI_E_ARG, "null argument");
    if (!x->slab) return fail(PGMI_E_STATE, "weights are not bound");
    HIPCHK(hipSetDevice(x->device));
    const pgmi_config& c = x->c;
    int rc;
    if (!x->cosT) {
        const int N = n_img(c);
        const size_t R = (size_t)c.max_batch * c.max_seq, RV = (size_t)c.max_batch * N;
        const int H = c.t_hidden, QKVN = (c.t_heads + 2 * c.t_kv_heads) * c.t_head_dim;
        x->kpad = (c.v_channels * c.v_patch * c.v_patch + 63) / 64 * 64;
        if ((rc = dalloc_t(x, &x->patch_w, (size_t)c.v_hidden * x->kpad))) return rc;
        if ((rc = dalloc_t(x, &x->cosT, (size_t)c.t_max_pos * c.t_head_dim / 2))) return rc;
        if ((rc = dalloc_t(x, &x->sinT, (size_t)c.t_max_pos * c.t_head_dim / 2))) return rc;
        if ((rc = dalloc_t(x, &x->Hs, R * H))) return rc;
        if ((rc = dalloc_t(x, &x->Tn, R * H))) return rc;
        if ((rc = dalloc_t(x, &x->QKV, R * QKVN))) return rc;
        if ((rc = dalloc_t(x, &x->Qr, R * c.t_heads * c.t_head_dim))) return rc;
        if ((rc = dalloc_t(x, &x->AO, R * H))) return rc;
        if ((rc = dalloc_t(x, &x->ACT, R * c.t_intermediate))) return rc;
        if ((rc = dalloc_t(x, &x->lastrows, (size_t)c.max_batch * H))) return rc;
        if ((rc = dalloc_t(x, &x->dpos, R))) return rc;
        if ((rc = dalloc_t(x, &x->dids_tmp, R))) return rc;
        if ((rc = dalloc_t(x, &x->vX, RV * c.v_hidden))) return rc;
        if ((rc = dalloc_t(x, &x->vT, RV * c.v_hidden))) return rc;
        if ((rc = dalloc_t(x, &x->vQKV, RV * 3 * c.v_hidden))) return rc;
        if ((rc = dalloc_t(x, &x->vAO, RV * c.v_hidden))) return rc;
        if ((rc = dalloc_t(x, &x->vH, RV * c.v_intermediate))) return rc;
        if ((rc = dalloc_t(x, &x->vP, RV * x->kpad))) return rc;
        x->ws_bytes = (size_t)64 << 20;
        if ((rc = dalloc(x, reinterpret_cast<void**>(&x->ws), x->ws_bytes))) return rc;
        const int B = c.max_batch;
        if ((rc = dalloc_t(x, &x->dH, (size_t)B * H))) return rc;
        if ((rc = dalloc_t(x, &x->dQ, (size_t)B * c.t_heads * c.t_head_dim))) return rc;
        if ((rc = dalloc_t(x, &x->dAO, (size_t)B * H))) return rc;
        if ((rc = dalloc_t(x, &x->dACT, (size_t)B * c.t_intermediate))) return rc;
        if ((rc = dalloc_t(x, &x->dHn, (size_t)B * H))) return rc;
        if ((rc = dalloc_t(x, &x->dSS, (size_t)B * (H / 16)))) return rc;
        x->max_chunks = (c.max_kv + 63) / 64;
        if ((rc = dalloc_t(x, &x->opart, attention_decode_part_floats(B, c.t_kv_heads, x->max_chunks)))) return rc;
        if ((rc = dalloc_t(x, &x->pmax, (size_t)B * gemv_logits_blocks()))) return rc;
        if ((rc = dalloc_t(x, &x->dlogits, (size_t)B * c.t_vocab))) return rc;
        if ((rc = dalloc_t(x, &x->pidx, (size_t)B * gemv_logits_blocks()))) return rc;
        if ((rc = dalloc_t(x, &x->step, 1))) return rc;
        if ((rc = dalloc_t(x, &x->pstep, 1))) return rc;
        if ((rc = dalloc_t(x, &x->amax_v, (size_t)argmax_scratch_parts()))) return rc;
        if ((rc = dalloc_t(x, &x->amax_i, (size_t)argmax_scratch_parts()))) return rc;
        if ((rc = dalloc_t(x, &x->d_ids, (size_t)B))) return rc;
        if ((rc = dalloc_t(x, &x->d_emb, (size_t)B * H))) return rc;
        if ((rc = dalloc_t(x, &x->d_mask, (size_t)B * c.max_kv))) return rc;
        if ((rc = dalloc_t(x, &x->d_zero, 64))) return rc;
        HIPCHK(hipMemset(x->d_zero, 0, 64 * sizeof(float)));
        if ((rc = dalloc_t(x, &x->d_next, (size_t)B))) return rc;
        if ((rc = dalloc_t(x, &x->lm_done, 33 * 32))) return rc;  // top word + 32 shards, a 128-B line each
        HIPCHK(hipMemset(x->lm_done, 0, 33 * 32 * sizeof(unsigned)));
        HIPCHK(hipStreamCreateWithFlags(&x->cap_stream, hipStreamNonBlocking));
    }
    // derived tensors
    pad_rows(nullptr, W(x, "vision_tower.vision_model.embeddings.patch_embedding.weight"), c.v_hidden,
             c.v_channels * c.v_patch * c.v_patch, x->kpad, x->patch_w);
    LAUNCHCHK();
    // the batched decode's fragment-major weight images: built by the first decode step with B >= 3 after this
    // call (ensure_mf_image), not here -- a context that never decodes a batch (the drop-in's single-sequence
    // loop on its max_batch-8 context) neither allocates their 3.96 GB nor pays for the swizzle
    x->mfw_dirty = c.max_batch >= gemv_mf_min_batch() && c.t_intermediate % 32 == 0 && c.t_hidden % 32 == 0;
    std::vector<uint16_t> cs, sn;
    if (!x->host_cos.empty()) {
        cs = x->host_cos;
        sn = x->host_sin;
    } else {
        build_rope_host(x, cs, sn);
    }
    HIPCHK(hipMemcpy(x->cosT, cs.data(), cs.size() * 2, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(x->sinT, sn.data(), sn.size() * 2, hipMemcpyHostToDevice));
    HIPCHK(hipDeviceSynchronize());
    clear_dgraphs(x);
    clear_pgraphs(x);
    x->prepared = true;
    return 0;
}

int64_t pgmi_kv_bytes(const pgmi_ctx* x, int batch, int max_tokens) {
    if (!x) return -1;
    return (int64_t)x->c.t_layers * 2 * batch * max_tokens * x->c.t_kv_heads * x->c.t_head_dim * 2;
}

// Run body(stream) eagerly, or replay its captured hipGraph: the first call with a given key
// runs eagerly (kernel attributes are set on first launch), the second captures, later ones
// replay.  The key holds every pointer and size the body reads, so a replay is that call.
extern "C++" {
template <class F>
static int run_graphed(pgmi_ctx* x, hipStream_t s, const std::vector<intptr_t>& key, F body) {
    if (!x->prefill_graph) return body(s);
    GraphEntry& ge = x->pgraphs[key];
    if (!ge.exec) {
        if (ge.seen++ == 0) return body(s);
        if (x->pgraphs.size() > 64) {  // bound the cache (e.g. fresh buffers every call)
            clear_pgraphs(x);
            return body(s);
        }
        hipGraph_t g;
        HIPCHK(hipStreamBeginCapture(x->cap_stream, hipStreamCaptureModeThreadLocal));
        const int rc = body(x->cap_stream);
        HIPCHK(hipStreamEndCapture(x->cap_stream, &g));
        if (rc) {
            (void)hipGraphDestroy(g);
            return rc;
        }
        GraphEntry& ge2 = x->pgraphs[key];
        HIPCHK(hipGraphInstantiate(&ge2.exec, g, nullptr, nullptr, 0));
        (void)hipGraphDestroy(g);
        HIPCHK(hipGraphLaunch(ge2.exec, s));
        return 0;
    }
    HIPCHK(hipGraphLaunch(ge.exec, s));
    return 0;
}
}  // extern "C++"

static int vision_body(pgmi_ctx* x, hipStream_t s, const void* pixels, int dtype, int B, void* feats);

int pgmi_vision(pgmi_ctx* x, const void* pixels, int dtype, int B, void* feats, void* stream) {
    int rc;
    if ((rc = ensure_prepared(x))) return rc;
    const pgmi_config& c = x->c;
    if (B < 1 || B > c.max_batch) return fail(PGMI_E_ARG, "batch exceeds max_batch");
    if (!pixels || !feats) return fail(PGMI_E_ARG, "null argument");
    const std::vector<intptr_t> key{1, (intptr_t)pixels, dtype, B, (intptr_t)feats};
    rc = run_graphed(x, (hipStream_t)stream, key,
                     [&](hipStream_t st) { return vision_body(x, st, pixels, dtype, B, feats); });
    if (rc) return rc;
    LAUNCHCHK();
    return 0;
}

static int vision_body(pgmi_ctx* x, hipStream_t s, const void* pixels, int dtype, int B, void* feats) {
    const pgmi_config& c = x->c;
    const int N = n_img(c), D = c.v_hidden, Iv = c.v_intermediate, rows = B * N;
    const float eps = c.v_ln_eps;
    patchify(s, pixels, dtype == PGMI_DTYPE_F32, B, c.v_channels, c.v_image, c.v_image, c.v_patch, x->kpad, x->vP);
    // Conv2d + bias + position embedding (modeling_siglip.py:67,76)
    EpiArgs e{};
    e.bias = W(x, "vision_tower.vision_model.embeddings.patch_embedding.bias");
    e.pos = W(x, "vision_tower.vision_model.embeddings.position_embedding.weight");
    e.npos = N;
    e.out = x->vX;
    e.ldo = D;
    gemm(s, x->vP, x->kpad, x->patch_w, x->kpad, rows, D, x->kpad, EPI_BIAS_POS, e, x->ws, x->ws_bytes);
    const float scale = (float)std::pow((double)(D / c.v_heads), -0.5);  // head_dim**-0.5 (:89)
    // LayerNorm1 of layer 0; every later LayerNorm is fused with the preceding projection's
    // split-K reduction + bias + residual (splitk_res_norm)
    layernorm(s, x->vX, VL(x, 0, "layer_norm1.weight"), VL(x, 0, "layer_norm1.bias"), eps, x->vT, rows, D);
    for (int i = 0; i < c.v_layers; ++i) {
        const bool last = i + 1 == c.v_layers;
        EpiArgs q{};
        q.bias = VL(x, i, "self_attn.q_proj.bias");  // q|k|v biases adjacent
        q.out = x->vQKV;
        q.ldo = 3 * D;
        gemm(s, x->vT, D, VL(x, i, "self_attn.q_proj.weight"), D, rows, 3 * D, D, EPI_BIAS, q, x->ws, x->ws_bytes);
        AttnArgs a{};
        a.q = x->vQKV; a.q_b_stride = (long)N * 3 * D; a.q_row_stride = 3 * D; a.q_head_stride = 72;
        a.k = x->vQKV + D; a.k_b_stride = a.q_b_stride; a.k_row_stride = 3 * D; a.k_head_stride = 72;
        a.v = x->vQKV + 2 * D; a.v_b_stride = a.q_b_stride; a.v_row_stride = 3 * D; a.v_head_stride = 72;
        a.o = x->vAO; a.o_b_stride = (long)N * D; a.o_row_stride = D; a.o_head_stride = 72;
        a.Lq = N; a.Lk = N; a.G = 1; a.n_kv = c.v_heads; a.B = B; a.scale = scale;
        a.ws = x->ws; a.ws_floats = (long)(x->ws_bytes / sizeof(float));
        attention_prefill(s, 72, a);
        EpiArgs o{};
        o.bias = VL(x, i, "self_attn.out_proj.bias");
        o.res = x->vX; o.ldr = D; o.out = x->vX; o.ldo = D;
        const int spo = gemm(s, x->vAO, D, VL(x, i, "self_attn.out_proj.weight"), D, rows, D, D, EPI_BIAS_RES, o, x->ws,
                             x->ws_bytes, 0, true);
        splitk_res_norm(s, x->ws, spo, o.bias, x->vX, VL(x, i, "layer_norm2.weight"), VL(x, i, "layer_norm2.bias"),
                        eps, x->vT, rows, D);
        EpiArgs f1{};
        f1.bias = VL(x, i, "mlp.fc1.bias"); f1.out = x->vH; f1.ldo = Iv;
        gemm(s, x->vT, D, VL(x, i, "mlp.fc1.weight"), D, rows, Iv, D, EPI_BIAS_GELU, f1, x->ws, x->ws_bytes);
        EpiArgs f2{};
        f2.bias = VL(x, i, "mlp.fc2.bias"); f2.res = x->vX; f2.ldr = D; f2.out = x->vX; f2.ldo = D;
        const int sp = gemm(s, x->vH, Iv, VL(x, i, "mlp.fc2.weight"), Iv, rows, D, Iv, EPI_BIAS_RES, f2, x->ws,
                            x->ws_bytes, 0, true);
        splitk_res_norm(s, x->ws, sp, f2.bias, x->vX,
                        last ? W(x, "vision_tower.vision_model.post_layernorm.weight") : VL(x, i + 1, "layer_norm1.weight"),
                        last ? W(x, "vision_tower.vision_model.post_layernorm.bias") : VL(x, i + 1, "layer_norm1.bias"),
                        eps, last ? reinterpret_cast<uint16_t*>(feats) : x->vT, rows, D);
    }
    if (c.v_layers == 0)
        layernorm(s, x->vX, W(x, "vision_tower.vision_model.post_layernorm.weight"),
                  W(x, "vision_tower.vision_model.post_layernorm.bias"), eps, reinterpret_cast<uint16_t*>(feats), rows, D);
    LAUNCHCHK();
    return 0;
}

int pgmi_project(pgmi_ctx* x, const void* feats, int rows, void* out, void* stream) {
    int rc;
    if ((rc = ensure_prepared(x))) return rc;
    if (!feats || !out || rows < 1) return fail(PGMI_E_ARG, "bad argument");
    if (rows > x->c.max_batch * n_img(x->c)) return fail(PGMI_E_ARG, "rows exceed workspace capacity");
    EpiArgs e{};
    e.bias = W(x, "multi_modal_projector.linear.bias");
    e.out = reinterpret_cast<uint16_t*>(out);
    e.ldo = x->c.projection_dim;
    gemm((hipStream_t)stream, reinterpret_cast<const uint16_t*>(feats), x->c.v_hidden,
         W(x, "multi_modal_projector.linear.weight"), x->c.v_hidden, rows, x->c.projection_dim, x->c.v_hidden,
         EPI_BIAS, e, x->ws, x->ws_bytes);
    LAUNCHCHK();
    return 0;
}

int pgmi_embed(pgmi_ctx* x, const int64_t* ids, int rows, void* out, void* stream) {
    int rc;
    if ((rc = ensure_prepared(x))) return rc;
    if (!ids || !out) return fail(PGMI_E_ARG, "null argument");
    // plain lookup: normalizer 1, no pad zeroing (nn.Embedding, modeling_gemma.py:565)
    embed_rows((hipStream_t)stream, ids, rows, W(x, "language_model.model.embed_tokens.weight"), x->c.t_hidden,
               1.0f, INT64_MIN, reinterpret_cast<uint16_t*>(out));
    LAUNCHCHK();
    return 0;
}

static int lm_body(pgmi_ctx* x, hipStream_t s, const int64_t* ids, const void* image_feats, int n_img_rows,
                   const void* embeds, int B, int L, void* kv, int kv_batch, int kv_max, int kv_start, float* logits,
                   int logits_rows);

int pgmi_lm_forward(pgmi_ctx* x, const int64_t* ids, const void* image_feats, int n_img_rows, const void* embeds,
                    int B, int L, const int64_t* positions, void* kv, int kv_batch, int kv_max, int kv_start,
                    float* logits, int logits_rows, void* stream) {
    int rc;
    if ((rc = ensure_prepared(x))) return rc;
    const pgmi_config& c = x->c;
    if (B < 1 || B > c.max_batch || B > kv_batch) return fail(PGMI_E_ARG, "batch exceeds capacity");
    if (L < 1 || L > c.max_seq) return fail(PGMI_E_ARG, "sequence length exceeds max_seq");
    if (kv_start < 0 || kv_start + L > kv_max) return fail(PGMI_E_ARG, "KV cache capacity exceeded");
    if (!positions || !kv || !logits || (!embeds && !ids)) return fail(PGMI_E_ARG, "null argument");
    if (logits_rows < 0 || logits_rows > 2) return fail(PGMI_E_ARG, "logits_rows must be 0, 1 or 2");
    // host positions -> device (outside any graph: a pageable host copy is not captured)
    HIPCHK(hipMemcpyAsync(x->dpos, positions, (size_t)B * L * sizeof(int64_t), hipMemcpyHostToDevice,
                          (hipStream_t)stream));
    // Tn is overwritten from here on: no row of it is valid until this call has succeeded
    x->tn_rows = 0;
    const std::vector<intptr_t> key{2, (intptr_t)ids, (intptr_t)image_feats, n_img_rows, (intptr_t)embeds, B, L,
                                    (intptr_t)kv, kv_batch, kv_max, kv_start, (intptr_t)logits, logits_rows};
    rc = run_graphed(x, (hipStream_t)stream, key, [&](hipStream_t st) {
        return lm_body(x, st, ids, image_feats, n_img_rows, embeds, B, L, kv, kv_batch, kv_max, kv_start, logits,
                       logits_rows);
    });
    if (rc) return rc;
    x->tn_rows = logits_rows == 2 && L > 1 ? 0 : (long)B * L;
    LAUNCHCHK();
    return 0;
}

static int lm_body(pgmi_ctx* x, hipStream_t s, const int64_t* ids, const void* image_feats, int n_img_rows,
                   const void* embeds, int B, int L, void* kv, int kv_batch, int kv_max, int kv_start, float* logits,
                   int logits_rows) {
    const pgmi_config& c = x->c;
    const int H = c.t_hidden, R = B * L, NH = c.t_heads, NKV = c.t_kv_heads, HD = c.t_head_dim;
    const int QKVN = (NH + 2 * NKV) * HD;
    const float eps = c.t_rms_eps;
    const float normalizer = bf16_round_host(std::sqrt((float)H));  // torch.tensor(H**0.5, dtype=bf16) (:367)
    const uint16_t* E = W(x, "language_model.model.embed_tokens.weight");
    if (embeds) {
        scale_rows(s, reinterpret_cast<const uint16_t*>(embeds), (long)R * H, normalizer, x->Hs);
    } else {
        merge_embed(s, ids, B, L, E, H, reinterpret_cast<const uint16_t*>(image_feats), image_feats ? n_img_rows : 0,
                    c.image_token_index, c.pad_token_id, (float)std::sqrt((double)H), normalizer, nullptr,
                    reinterpret_cast<int*>(x->dids_tmp), x->Hs);
    }
    const long kvd = (long)NKV * HD, kvb = (long)kv_max * kvd;
    uint16_t* kvp = reinterpret_cast<uint16_t*>(kv);
    const uint16_t* fnorm = W(x, "language_model.model.norm.weight");
    const bool last_only = logits_rows == 2 && L > 1 && c.t_layers > 0;
    // input RMSNorm of layer 0; every later RMSNorm (and the final norm) is fused with the
    // preceding projection's split-K reduction + residual (splitk_res_norm)
    rmsnorm(s, x->Hs, c.t_layers ? TL(x, 0, "input_layernorm.weight") : fnorm, eps, x->Tn, R, H);
    for (int i = 0; i < c.t_layers; ++i) {
        uint16_t* Kc = kvp + ((long)(i * 2 + 0) * kv_batch) * kvb;
        uint16_t* Vc = kvp + ((long)(i * 2 + 1) * kv_batch) * kvb;
        EpiArgs q{};
        q.out = x->QKV; q.ldo = QKVN;
        // RoPE + KV append in the projection's epilogue where the shape's plan allows it
        q.rpos = x->dpos; q.cosT = x->cosT; q.sinT = x->sinT; q.max_pos = c.t_max_pos;
        q.q_out = x->Qr; q.kc = Kc; q.vc = Vc; q.kv_b_stride = kvb; q.kv_start = kv_start;
        q.L = L; q.nh = NH; q.nkv = NKV;
        const uint16_t* Wqkv = TL(x, i, "self_attn.q_proj.weight");
        if (HD != 256 || !gemm_qkv_rope(s, x->Tn, H, Wqkv, H, R, QKVN, H, q)) {
            int sp = gemm(s, x->Tn, H, Wqkv, H, R, QKVN, H, EPI_STORE, q, x->ws, x->ws_bytes, 0, true);
            rope_kv_append(s, x->QKV, x->ws, sp, B, L, NH, NKV, x->dpos, x->cosT, x->sinT, c.t_max_pos, x->Qr, Kc, Vc,
                           kvb, kv_start);
        }
        AttnArgs a{};
        a.q = x->Qr; a.q_b_stride = (long)L * NH * HD; a.q_row_stride = NH * HD; a.q_head_stride = HD;
        a.k = Kc; a.k_b_stride = kvb; a.k_row_stride = (int)kvd; a.k_head_stride = HD;
        a.v = Vc; a.v_b_stride = kvb; a.v_row_stride = (int)kvd; a.v_head_stride = HD;
        a.o = x->AO; a.o_b_stride = (long)L * H; a.o_row_stride = H; a.o_head_stride = HD;
        a.Lq = L; a.Lk = kv_start + L; a.G = NH / NKV; a.n_kv = NKV; a.B = B;
        a.scale = 1.0f / std::sqrt((float)HD);  // / math.sqrt(head_dim) (:266): exact power of two
        a.ws = x->ws; a.ws_floats = (long)(x->ws_bytes / sizeof(float));
        if (last_only && i + 1 == c.t_layers) {
            // logits_rows == 2, last layer: the K/V rows of every token are written above (the cache
            // the decode loop reads); the rest of the layer feeds only the final hidden state, and the
            // caller reads that for the last row alone, so attention, o_proj, the MLP and the final
            // norm run for the last row of each sequence (row-wise ops: the same values as the
            // all-row pass up to GEMV-vs-GEMM accumulation order), on the decode GEMVs
            a.q = x->Qr + (size_t)(L - 1) * NH * HD;
            a.o = x->dAO; a.o_b_stride = (long)H;
            a.Lq = 1;
            HIPCHK(hipMemcpy2DAsync(x->lastrows, (size_t)H * 2, x->Hs + (size_t)(L - 1) * H, (size_t)L * H * 2,
                                    (size_t)H * 2, B, hipMemcpyDeviceToDevice, s));
            if (kv_start + L <= c.max_kv) {
                // one query row over the prompt's keys: the decode step's flash-decoding (64-key chunks
                // in parallel, kv_len from a device step record set by a memset node) and its o_proj
                // GEMV with the chunk combine in the prologue; a single 16-row prefill workgroup
                // would walk every key alone
                a.Lk = 0;
                HIPCHK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(&x->pstep->kv_len), kv_start + L - 1, 1, s));
                a.mask = x->d_zero; a.mask_b_stride = 0; a.mask_k_stride = 0; a.mask_round = 1;
                attention_decode(s, a, x->pstep, kv_start + L, x->opart, x->max_chunks);
                gemv_o_attn(s, B, NH, x->opart, x->max_chunks, x->pstep, TL(x, i, "self_attn.o_proj.weight"), H,
                            x->lastrows, B >= gemv_mf_min_batch() ? x->dAO : nullptr);
            } else {
                attention_prefill(s, 256, a);
                gemv_res(s, B, NH * HD, x->dAO, TL(x, i, "self_attn.o_proj.weight"), H, x->lastrows, x->ws);
            }
            gemv_geglu(s, B, x->lastrows, TL(x, i, "post_attention_layernorm.weight"), eps,
                       TL(x, i, "mlp.gate_proj.weight"), c.t_intermediate, x->dACT);
            gemv_res(s, B, c.t_intermediate, x->dACT, TL(x, i, "mlp.down_proj.weight"), H, x->lastrows, x->ws);
            break;
        }
        attention_prefill(s, 256, a);
        EpiArgs o{};
        o.res = x->Hs; o.ldr = H; o.out = x->Hs; o.ldo = H;
        int sp = gemm(s, x->AO, H, TL(x, i, "self_attn.o_proj.weight"), H, R, H, NH * HD, EPI_RES, o, x->ws, x->ws_bytes,
                  0, true);
        splitk_res_norm(s, x->ws, sp, nullptr, x->Hs, TL(x, i, "post_attention_layernorm.weight"), nullptr, eps, x->Tn,
                        R, H);
        EpiArgs g{};
        g.out = x->ACT; g.ldo = c.t_intermediate;
        const bool probe = x->probe_on && (size_t)(4 * i + 3) < x->probe_ev.size();
        // probe: the GEMM kernel itself carries the events (its own start / end, gemm_probe_events)
        if (probe) gemm_probe_events(x->probe_ev[4 * i], x->probe_ev[4 * i + 1]);
        gemm(s, x->Tn, H, TL(x, i, "mlp.gate_proj.weight"), H, R, c.t_intermediate, H, EPI_GEGLU, g, x->ws,
             x->ws_bytes, c.t_intermediate);
        EpiArgs d{};
        d.res = x->Hs; d.ldr = H; d.out = x->Hs; d.ldo = H;
        if (probe) gemm_probe_events(x->probe_ev[4 * i + 2], x->probe_ev[4 * i + 3]);
        sp = gemm(s, x->ACT, c.t_intermediate, TL(x, i, "mlp.down_proj.weight"), c.t_intermediate, R, H,
                  c.t_intermediate, EPI_RES, d, x->ws, x->ws_bytes, 0, true);
        const bool last = i + 1 == c.t_layers;
        splitk_res_norm(s, x->ws, sp, nullptr, x->Hs, last ? fnorm : TL(x, i + 1, "input_layernorm.weight"), nullptr,
                        eps, x->Tn, R, H);
    }
    if (logits_rows == 0) {
        EpiArgs l{};  // Tn holds the final RMSNorm (modeling_gemma.py:379)
        l.out_f32 = logits; l.ldo = c.t_vocab;
        gemm(s, x->Tn, H, E, H, R, c.t_vocab, H, EPI_F32, l, x->ws, x->ws_bytes);
    } else {
        if (!last_only)
            HIPCHK(hipMemcpy2DAsync(x->lastrows, (size_t)H * 2, x->Hs + (size_t)(L - 1) * H, (size_t)L * H * 2,
                                    (size_t)H * 2, B, hipMemcpyDeviceToDevice, s));
        int nparts = 0;
        gemv_logits(s, B, x->lastrows, fnorm, eps, E, c.t_vocab, logits, x->pmax, x->pidx, &nparts);
    }
    LAUNCHCHK();
    return 0;
}

// The batched form's RMSNorms: computed once per row -- the input norm by the down projection's combine for
// the next layer (k_mf_combine_norm; q|k|v reads dHn unstaged), the post-attention norm from o_proj's 16-column
// partial sums of squares, applied by gate|up as it loads h (default) -- or each projection stages and
// normalises its rows itself (pgmi_set_decode_staged_norm,
// tested by test_batch_rows_teacher_forced_vs_own_reference[8-1]).  Round 4, the unstaged form reading rows
// normalised by separate passes against the staged form: equal
// while the weight streams were non-temporal (B = 8 step 1.5449 vs 1.5452 ms); with the default cache policy
// (kernels_gemv_mfma.hip PGMI_MF_NT) the unstaged form wins, same box: 1.4523 / 1.4550 -> 1.4330 / 1.4320 ms
static bool mf_staged(const pgmi_ctx* x) { return x->mf_staged > 0; }

static int decode_body(pgmi_ctx* x, hipStream_t s, const int64_t* ids, int B, void* kv, int kv_batch, int kv_max,
                       int launch_keys, float* logits, int64_t* next_ids, const uint16_t* embeds = nullptr,
                       int masked = 0, int64_t* hist = nullptr) {
    const pgmi_config& c = x->c;
    const int H = c.t_hidden, NH = c.t_heads, NKV = c.t_kv_heads, HD = c.t_head_dim;
    const float eps = c.t_rms_eps;
    const float normalizer = bf16_round_host(std::sqrt((float)H));
    const uint16_t* E = W(x, "language_model.model.embed_tokens.weight");
    const long kvd = (long)NKV * HD, kvb = (long)kv_max * kvd;
    uint16_t* kvp = reinterpret_cast<uint16_t*>(kv);
    // B <= 2: the embedding row is read by layer 0's q|k|v GEMV itself (one launch fewer per step)
    const bool fold = !embeds && gemv_qkv_folds_embed(B) && c.t_layers > 0;
    const EmbedFold emb{ids, E, normalizer, c.pad_token_id, x->dH};
    // given input rows (a caller's merge, pgmi_decode_embeds): h = rows x bf16(sqrt(hidden)) (modeling_gemma.py:367-368)
    if (embeds) scale_rows(s, embeds, (long)B * H, normalizer, x->dH);
    else if (!fold) embed_rows(s, ids, B, E, H, normalizer, c.pad_token_id, x->dH);
    // B >= 3 (MFMA projections): every RMSNorm is computed once per row -- the input norm fused into the
    // down projection's combine for the next layer (q|k|v reads dHn unstaged), the post-attention norm's
    // sums of squares written by o_proj's epilogue (dSS) and applied by gate|up as it loads h.  (Round 5,
    // the input norm the same way -- the down combine writing partials, q|k|v normalising on load: q|k|v
    // 5.97 -> 7.59 us for a combine no shorter, 4.63 -> 4.72 us; with the combine inside the down launch,
    // B = 8 step 1.437 -> 1.446-1.465 ms, same box.)
    const bool mf = B >= gemv_mf_min_batch() && !mf_staged(x);
    if (mf && c.t_layers > 0) rows_norm(s, x->dH, TL(x, 0, "input_layernorm.weight"), eps, B, H, x->dHn);
    for (int i = 0; i < c.t_layers; ++i) {
        uint16_t* Kc = kvp + ((long)(i * 2 + 0) * kv_batch) * kvb;
        uint16_t* Vc = kvp + ((long)(i * 2 + 1) * kv_batch) * kvb;
        // fragment-major weight images of this layer (prepare's mf_swizzle), when built: gate|up, q|k|v, o_proj
        const uint16_t* Lf = x->mfw ? x->mfw + x->mfw_layer * i : nullptr;
        const size_t gu_n = (size_t)2 * c.t_intermediate * H, qkv_n = (size_t)(NH + 2 * NKV) * HD * H;
        gemv_qkv(s, B, NH, NKV, mf ? x->dHn : x->dH, mf ? nullptr : TL(x, i, "input_layernorm.weight"), eps,
                 TL(x, i, "self_attn.q_proj.weight"), x->cosT, x->sinT, c.t_max_pos, x->step, x->dQ, Kc, Vc, kvb, x->ws,
                 (fold && i == 0) ? &emb : nullptr, Lf ? Lf + gu_n : nullptr);
        AttnArgs a{};
        a.q = x->dQ; a.q_b_stride = (long)NH * HD; a.q_row_stride = NH * HD; a.q_head_stride = HD;
        a.k = Kc; a.k_b_stride = kvb; a.k_row_stride = (int)kvd; a.k_head_stride = HD;
        a.v = Vc; a.v_b_stride = kvb; a.v_row_stride = (int)kvd; a.v_head_stride = HD;
        a.o = x->dAO; a.o_b_stride = (long)H; a.o_row_stride = H; a.o_head_stride = HD;
        a.Lq = 1; a.Lk = 0; a.G = NH / NKV; a.n_kv = NKV; a.B = B; a.scale = 1.0f / std::sqrt((float)HD);
        if (masked) {  // the staged additive mask (pgmi_decode_embeds_dev), row stride max_kv
            a.mask = x->d_mask; a.mask_b_stride = c.max_kv; a.mask_k_stride = 1; a.mask_round = masked == 1;
        } else {
            a.mask = x->d_zero; a.mask_b_stride = 0; a.mask_k_stride = 0; a.mask_round = 1;
        }
        attention_decode(s, a, x->step, launch_keys, x->opart, x->max_chunks);
        gemv_o_attn(s, B, NH, x->opart, x->max_chunks, x->step, TL(x, i, "self_attn.o_proj.weight"), H, x->dH,
                    B >= gemv_mf_min_batch() ? x->dAO : nullptr, mf ? x->dSS : nullptr, Lf ? Lf + gu_n + qkv_n : nullptr);
        if (mf) {
            // the post-attention RMSNorm: its sums of squares come from o_proj's epilogue (dSS), gate|up
            // normalises h on load (no k_rows_norm pass: B = 8 step -5 us per layer)
            gemv_geglu(s, B, x->dH, TL(x, i, "post_attention_layernorm.weight"), eps, TL(x, i, "mlp.gate_proj.weight"),
                       c.t_intermediate, x->dACT, x->dSS, Lf);
            gemv_res_norm(s, B, c.t_intermediate, x->dACT, TL(x, i, "mlp.down_proj.weight"), H, x->dH, x->ws,
                          i + 1 < c.t_layers ? TL(x, i + 1, "input_layernorm.weight") : nullptr, eps, x->dHn,
                          Lf ? Lf + gu_n + qkv_n + (size_t)H * NH * HD : nullptr);
            continue;
        }
        gemv_geglu(s, B, x->dH, TL(x, i, "post_attention_layernorm.weight"), eps, TL(x, i, "mlp.gate_proj.weight"),
                   c.t_intermediate, x->dACT);
        gemv_res(s, B, c.t_intermediate, x->dACT, TL(x, i, "mlp.down_proj.weight"), H, x->dH, x->ws);
    }
    int nparts = 0;
    int64_t* nx = next_ids ? next_ids : x->d_next;
    // the step's last work also advances the device step state (pgmi_decode skips its host-side
    // set when the next call continues the sequence): lm_head's last workgroup, or argmax_finish
    if (!gemv_logits(s, B, x->dH, W(x, "language_model.model.norm.weight"), eps, E, c.t_vocab, logits, x->pmax,
                     x->pidx, &nparts, x->lm_done, nx, x->step, hist))
        argmax_finish(s, B, x->pmax, x->pidx, nparts, nx, x->step, hist);
    return 0;
}

int pgmi_prefill_probe(pgmi_ctx* x, int on) {
    if (!x) return fail(PGMI_E_ARG, "null context");
    if (on && x->probe_ev.empty()) {
        x->probe_ev.resize((size_t)4 * x->c.t_layers);
        for (auto& e : x->probe_ev) HIPCHK(hipEventCreate(&e));
    }
    // the probe records its events in eager forwards: prefill graphs are off while it is on, and the
    // caller's own setting (pgmi_set_prefill_graph) is restored when it is turned off
    if (on && !x->probe_on) x->graph_before_probe = x->prefill_graph;
    if (!on && x->probe_on) x->prefill_graph = x->graph_before_probe;
    x->probe_on = on != 0;
    if (x->probe_on) x->prefill_graph = false;
    clear_pgraphs(x);
    return 0;
}

int pgmi_prefill_probe_times(pgmi_ctx* x, float* us, int n) {
    if (!x || !us) return fail(PGMI_E_ARG, "null argument");
    if (x->probe_ev.empty()) return fail(PGMI_E_STATE, "pgmi_prefill_probe(ctx, 1) has not been called");
    const int L = x->c.t_layers;
    if (n < 2 * L) return fail(PGMI_E_ARG, "us needs 2 x layers entries");
    HIPCHK(hipEventSynchronize(x->probe_ev.back()));
    for (int i = 0; i < L; ++i) {
        float a = 0.f, b = 0.f;
        HIPCHK(hipEventElapsedTime(&a, x->probe_ev[4 * i], x->probe_ev[4 * i + 1]));
        HIPCHK(hipEventElapsedTime(&b, x->probe_ev[4 * i + 2], x->probe_ev[4 * i + 3]));
        us[i] = a * 1e3f;
        us[L + i] = b * 1e3f;
    }
    return 0;
}

int pgmi_set_decode_staged_norm(pgmi_ctx* x, int on) {
    if (!x) return fail(PGMI_E_ARG, "null context");
    x->mf_staged = on < 0 ? -1 : on != 0;
    clear_dgraphs(x);  // captured steps hold the other form's launches
    return 0;
}

int pgmi_set_prefill_graph(pgmi_ctx* x, int on) {
    if (!x) return fail(PGMI_E_ARG, "null context");
    if (x->probe_on) x->graph_before_probe = on != 0;  // applied when the probe is turned off
    else x->prefill_graph = on != 0;
    clear_pgraphs(x);
    return 0;
}

// device-side inputs of a decode step over merged rows (pgmi_decode_embeds_dev): the rotary position
// and the additive mask come from the caller's merge outputs without a host read
struct DevStepIn {
    const void* pos = nullptr;  // (B, 1) position tensor on the device, dtype code (set_step_dev)
    int pos_dtype = 0;
    const void* mask = nullptr;  // additive mask rows (kv_len + 1 keys each)
    int mask_dtype = 0;
    long mask_b_stride = 0;
};

// The fragment-major images of every layer's gate|up, q|k|v, o_proj and down weights that the batched (B >= 3)
// decode projections read (kernels_gemv_mfma.hip; round 5), (re)built on stream s after a pgmi_prepare.  If the
// 3.96 GB (at the 3B shapes) cannot be allocated the batched decode reads the row-major weights instead (the
// same values in the same lanes: bit-identical results, slower), so the context stays usable.
static int ensure_mf_image(pgmi_ctx* x, hipStream_t s) {
    if (!x->mfw_dirty) return 0;
    const pgmi_config& c = x->c;
    const size_t I = c.t_intermediate, H = c.t_hidden, QKVN = (size_t)(c.t_heads + 2 * c.t_kv_heads) * c.t_head_dim,
                 OK = (size_t)c.t_heads * c.t_head_dim, per = 2 * I * H + QKVN * H + H * OK + H * I;
    x->mfw_dirty = false;
    if (!x->mfw) {
        void* p = nullptr;
        if (hipMalloc(&p, per * c.t_layers * sizeof(uint16_t)) != hipSuccess) {
            (void)hipGetLastError();  // out of memory: keep the row-major form
            return 0;
        }
        x->allocs.push_back(p);
        x->mfw = reinterpret_cast<uint16_t*>(p);
        clear_dgraphs(x);  // steps captured before held the row-major launches
    }
    x->mfw_layer = per;
    for (int i = 0; i < c.t_layers; ++i) {
        uint16_t* L = x->mfw + per * i;
        mf_swizzle(s, TL(x, i, "mlp.gate_proj.weight"), (int)(2 * I), (int)H, L);  // gate rows, then up rows
        mf_swizzle(s, TL(x, i, "self_attn.q_proj.weight"), (int)QKVN, (int)H, L + 2 * I * H, true);  // q|k|v
        mf_swizzle(s, TL(x, i, "self_attn.o_proj.weight"), (int)H, (int)OK, L + 2 * I * H + QKVN * H);
        mf_swizzle(s, TL(x, i, "mlp.down_proj.weight"), (int)H, (int)I, L + 2 * I * H + QKVN * H + H * OK);
    }
    LAUNCHCHK();
    return 0;
}

static int decode_step(pgmi_ctx* x, const int64_t* ids, const void* embeds, int B, void* kv, int kv_batch, int kv_max,
                       int kv_len, int position, float* logits, int64_t* next_ids, int use_graph, void* stream,
                       const DevStepIn* dev = nullptr, int n_steps = 1, int64_t* tokens = nullptr) {
    int rc;
    if ((rc = ensure_prepared(x))) return rc;
    const pgmi_config& c = x->c;
    if (B < 1 || B > c.max_batch || B > kv_batch) return fail(PGMI_E_ARG, "batch exceeds capacity");
    if (n_steps < 1) return fail(PGMI_E_ARG, "n_steps must be >= 1");
    if (n_steps > 1 && (!ids || embeds || dev)) return fail(PGMI_E_ARG, "multi-step decode: token ids only");
    if (kv_len < 0 || (long)kv_len + n_steps - 1 >= kv_max) return fail(PGMI_E_ARG, "KV cache capacity exceeded");
    if (kv_max > c.max_kv) return fail(PGMI_E_ARG, "kv_max exceeds config max_kv");
    if ((!ids && !embeds) || !kv || !logits) return fail(PGMI_E_ARG, "null argument");
    hipStream_t s = (hipStream_t)stream;
    if (B >= gemv_mf_min_batch() && (rc = ensure_mf_image(x, s))) return rc;
    int masked = 0;
    if (dev) {
        // position read on the device; the host no longer knows it, so the next call sets the state again
        set_step_dev(s, x->step, kv_len, dev->pos, dev->pos_dtype);
        if (dev->mask) {
            stage_mask(s, dev->mask, dev->mask_dtype, B, dev->mask_b_stride, kv_len + 1, x->d_mask, c.max_kv);
            masked = dev->mask_dtype == PGMI_DTYPE_F32 ? 2 : 1;
        }
    } else if (!x->step_known || x->step_kv != kv_len || x->step_pos != position) {
        set_step(s, x->step, kv_len, position);
    }
    // the step advances the device state itself (its last kernel); known only once this call has
    // enqueued its steps successfully
    x->step_known = false;
    auto advanced = [&]() {
        x->step_known = dev == nullptr;
        x->step_kv = kv_len + n_steps;
        x->step_pos = position + n_steps;
    };
    // input rows are always staged into the context's buffer (a stable address the graph reads)
    const uint16_t* erows = nullptr;
    if (embeds) {
        HIPCHK(hipMemcpyAsync(x->d_emb, embeds, (size_t)B * c.t_hidden * 2, hipMemcpyDeviceToDevice, s));
        erows = x->d_emb;
    }
    // n_steps greedy steps back to back: step t > 0 reads the argmax step t - 1 wrote (next_ids, or the
    // context's d_next when the caller passes none); step t's token also goes to tokens[t][B] when given
    int64_t* fb = next_ids ? next_ids : x->d_next;
    auto body = [&](hipStream_t st, const int64_t* first, int keys0, bool grow) -> int {
        for (int t = 0; t < n_steps; ++t) {
            const int r = decode_body(x, st, t == 0 ? first : fb, B, kv, kv_batch, kv_max, grow ? keys0 + t : keys0,
                                      logits, next_ids, erows, masked, tokens ? tokens + (long)t * B : nullptr);
            if (r) return r;
        }
        return 0;
    };
    if (!use_graph) {
        if ((rc = body(s, ids, kv_len + 1, true))) return rc;
        LAUNCHCHK();
        advanced();
        return 0;
    }
    // in-place feedback (next_ids == ids: the step reads its tokens first and writes the next
    // ones last) needs no staging copy; other callers' ids are staged into the context's buffer
    const int64_t* gids = ids;
    if (!embeds && ids != next_ids) {
        HIPCHK(hipMemcpyAsync(x->d_ids, ids, (size_t)B * sizeof(int64_t), hipMemcpyDeviceToDevice, s));
        gids = x->d_ids;
    }
    if (embeds) gids = nullptr;
    GraphKey key{B, kv, kv_batch, kv_max, logits, next_ids, gids, embeds != nullptr, masked, n_steps, tokens};
    GraphEntry& ge = x->graphs[key];
    if (!ge.exec) {
        if (ge.seen++ == 0) {  // first call with this key: run eagerly (sets kernel attributes)
            if ((rc = body(s, gids, kv_max, false))) return rc;
            LAUNCHCHK();
            advanced();
            return 0;
        }
        HIPCHK(hipStreamSynchronize(s));
        hipGraph_t g;
        HIPCHK(hipStreamBeginCapture(x->cap_stream, hipStreamCaptureModeThreadLocal));
        rc = body(x->cap_stream, gids, kv_max, false);
        HIPCHK(hipStreamEndCapture(x->cap_stream, &g));
        if (rc) return rc;
        HIPCHK(hipGraphInstantiate(&ge.exec, g, nullptr, nullptr, 0));
        (void)hipGraphDestroy(g);
    }
    HIPCHK(hipGraphLaunch(ge.exec, s));
    LAUNCHCHK();
    advanced();
    return 0;
}

int pgmi_decode(pgmi_ctx* x, const int64_t* ids, int B, void* kv, int kv_batch, int kv_max, int kv_len, int position,
                float* logits, int64_t* next_ids, int use_graph, void* stream) {
    if (!ids) return fail(PGMI_E_ARG, "null argument");
    return decode_step(x, ids, nullptr, B, kv, kv_batch, kv_max, kv_len, position, logits, next_ids, use_graph, stream);
}

int pgmi_decode_steps(pgmi_ctx* x, int64_t* ids, int B, void* kv, int kv_batch, int kv_max, int kv_len, int position,
                      int n_steps, float* logits, int64_t* tokens, int use_graph, void* stream) {
    if (!ids) return fail(PGMI_E_ARG, "null argument");
    return decode_step(x, ids, nullptr, B, kv, kv_batch, kv_max, kv_len, position, logits, ids, use_graph, stream,
                       nullptr, n_steps, tokens);
}

int pgmi_decode_embeds(pgmi_ctx* x, const void* embeds, int B, void* kv, int kv_batch, int kv_max, int kv_len,
                       int position, float* logits, int64_t* next_ids, int use_graph, void* stream) {
    if (!embeds) return fail(PGMI_E_ARG, "null argument");
    return decode_step(x, nullptr, embeds, B, kv, kv_batch, kv_max, kv_len, position, logits, next_ids, use_graph,
                       stream);
}

int pgmi_decode_embeds_dev(pgmi_ctx* x, const void* embeds, int B, void* kv, int kv_batch, int kv_max, int kv_len,
                           const void* position, int position_dtype, const void* mask, int mask_dtype,
                           int64_t mask_b_stride, float* logits, int64_t* next_ids, int use_graph, void* stream) {
    if (!embeds || !position) return fail(PGMI_E_ARG, "null argument");
    if (position_dtype != PGMI_DTYPE_BF16 && position_dtype != PGMI_DTYPE_F32 && position_dtype != 10 &&
        position_dtype != 11 && position_dtype != 12)
        return fail(PGMI_E_ARG, "position dtype must be bf16, fp32, fp64, int64 or int32");
    if (mask && mask_dtype != PGMI_DTYPE_BF16 && mask_dtype != PGMI_DTYPE_F32)
        return fail(PGMI_E_ARG, "mask dtype must be bf16 or fp32");
    if (B != 1) return fail(PGMI_E_ARG, "device-side positions: one sequence per step (B = 1)");
    DevStepIn d;
    d.pos = position; d.pos_dtype = position_dtype; d.mask = mask; d.mask_dtype = mask_dtype;
    d.mask_b_stride = (long)mask_b_stride;
    return decode_step(x, nullptr, embeds, B, kv, kv_batch, kv_max, kv_len, -1, logits, next_ids, use_graph, stream,
                       &d);
}

int pgmi_lm_head(pgmi_ctx* x, const void* normed, int rows, float* logits, void* stream) {
    int rc;
    if ((rc = ensure_prepared(x))) return rc;
    if (!normed || !logits) return fail(PGMI_E_ARG, "null argument");
    if (rows < 1) return fail(PGMI_E_ARG, "lm_head: no rows");
    const pgmi_config& c = x->c;
    EpiArgs l{};
    l.out_f32 = logits;
    l.ldo = c.t_vocab;
    gemm((hipStream_t)stream, reinterpret_cast<const uint16_t*>(normed), c.t_hidden,
         W(x, "language_model.model.embed_tokens.weight"), c.t_hidden, rows, c.t_vocab, c.t_hidden, EPI_F32, l, x->ws,
         x->ws_bytes);
    LAUNCHCHK();
    return 0;
}

int pgmi_lm_final_hidden(pgmi_ctx* x, void* out, int rows, void* stream) {
    int rc;
    if ((rc = ensure_prepared(x))) return rc;
    if (!out) return fail(PGMI_E_ARG, "null argument");
    if (rows < 1 || rows > x->c.max_batch * x->c.max_seq) return fail(PGMI_E_ARG, "rows exceed the prefill workspace");
    if (rows > x->tn_rows)
        return fail(PGMI_E_STATE, "the last pgmi_lm_forward did not keep these rows' final hidden states (logits_rows 2)");
    HIPCHK(hipMemcpyAsync(out, x->Tn, (size_t)rows * x->c.t_hidden * 2, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return 0;
}

// ---------------------------------------------------------------- replicas: load-time broadcast
#define RCCL_READY()                                                                       \
    do {                                                                                   \
        const Rccl& r_ = rccl();                                                           \
        if (!r_.get_unique_id || !r_.comm_init_rank || !r_.comm_destroy || !r_.broadcast || !r_.error_string) \
            return fail(PGMI_E_STATE, std::string("librccl could not be loaded (dlopen librccl.so.1): ") + \
                        (r_.h ? "missing nccl* symbols" : r_.why));                        \
    } while (0)

#define NCCLCHK(expr)                                                                      \
    do {                                                                                   \
        ncclResult_t r_ = (expr);                                                          \
        if (r_ != ncclSuccess) return fail(PGMI_E_HIP, std::string(#expr) + ": " + rccl().error_string(r_)); \
    } while (0)

int pgmi_comm_unique_id(void* id_out) {
    if (!id_out) return fail(PGMI_E_ARG, "null argument");
    RCCL_READY();
    static_assert(sizeof(ncclUniqueId) == PGMI_COMM_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId id;
    NCCLCHK(rccl().get_unique_id(&id));
    std::memcpy(id_out, &id, sizeof(id));
    return 0;
}

int pgmi_comm_init(int device, int nranks, int rank, const void* id, void** comm_out) {
    if (!id || !comm_out) return fail(PGMI_E_ARG, "null argument");
    if (nranks < 1 || rank < 0 || rank >= nranks) return fail(PGMI_E_ARG, "bad rank / world size");
    RCCL_READY();
    // the communicator binds to the current device: switch for the init, then give the caller's
    // thread its own current device back (torch keeps its own notion of it)
    int prev = 0;
    HIPCHK(hipGetDevice(&prev));
    HIPCHK(hipSetDevice(device));
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    ncclComm_t comm = nullptr;
    const ncclResult_t r = rccl().comm_init_rank(&comm, nranks, uid, rank);
    HIPCHK(hipSetDevice(prev));
    if (r != ncclSuccess) return fail(PGMI_E_HIP, std::string("ncclCommInitRank: ") + rccl().error_string(r));
    *comm_out = comm;
    return 0;
}

int pgmi_comm_destroy(void* comm) {
    if (!comm) return 0;
    RCCL_READY();
    NCCLCHK(rccl().comm_destroy(reinterpret_cast<ncclComm_t>(comm)));
    return 0;
}

int pgmi_broadcast_weights(pgmi_ctx* x, void* comm, int root, void* stream) {
    if (!x || !comm) return fail(PGMI_E_ARG, "null argument");
    if (!x->slab) return fail(PGMI_E_STATE, "weights are not bound (pgmi_bind_weights)");
    RCCL_READY();
    int prev = 0;
    HIPCHK(hipGetDevice(&prev));
    HIPCHK(hipSetDevice(x->device));
    // the whole slab in one in-place collective: rank `root`'s bytes land in every replica
    const ncclResult_t r = rccl().broadcast(x->slab, x->slab, (size_t)x->slab_bytes, ncclUint8, root,
                                            reinterpret_cast<ncclComm_t>(comm), (hipStream_t)stream);
    HIPCHK(hipSetDevice(prev));
    if (r != ncclSuccess) return fail(PGMI_E_HIP, std::string("ncclBroadcast: ") + rccl().error_string(r));
    x->prepared = false;  // derived tensors are rebuilt from the received weights by pgmi_prepare
    return 0;
}

int pgmi_argmax(pgmi_ctx* x, const float* logits, int rows, int V, int64_t* out, void* stream) {
    if (!x || !logits || !out) return fail(PGMI_E_ARG, "null argument");
    if (rows <= 0 || V <= 0) return fail(PGMI_E_ARG, "argmax: empty logits");
    if (!x->amax_v) return fail(PGMI_E_STATE, "argmax scratch missing");
    argmax_rows((hipStream_t)stream, logits, rows, V, x->amax_v, x->amax_i, out);
    LAUNCHCHK();
    return 0;
}

int pgmi_eos_update(pgmi_ctx* x, int64_t* next_ids, int32_t* finished, int B, int64_t eos_id, int64_t pad_id,
                    int32_t* n_alive, void* stream) {
    if (!x || !next_ids || !finished) return fail(PGMI_E_ARG, "null argument");
    if (B <= 0) return fail(PGMI_E_ARG, "eos_update: empty batch");
    eos_update((hipStream_t)stream, next_ids, finished, B, eos_id, pad_id, n_alive);
    LAUNCHCHK();
    return 0;
}

int pgmi_decode_kernel(pgmi_ctx* x, int which, int layer, int B, void* stream) {
    int rc;
    if ((rc = ensure_prepared(x))) return rc;
    const pgmi_config& c = x->c;
    if (B < 1 || B > c.max_batch) return fail(PGMI_E_ARG, "batch exceeds max_batch");
    if (layer < 0 || layer >= c.t_layers) return fail(PGMI_E_ARG, "layer out of range");
    hipStream_t s = (hipStream_t)stream;
    const float eps = c.t_rms_eps;
    const int H = c.t_hidden;
    switch (which) {
        case 1: gemv_res(s, B, c.t_heads * c.t_head_dim, x->dAO, TL(x, layer, "self_attn.o_proj.weight"), H, x->dH, x->ws); break;
        case 2:
            gemv_geglu(s, B, x->dH, TL(x, layer, "post_attention_layernorm.weight"), eps, TL(x, layer, "mlp.gate_proj.weight"),
                       c.t_intermediate, x->dACT);
            break;
        case 3: gemv_res(s, B, c.t_intermediate, x->dACT, TL(x, layer, "mlp.down_proj.weight"), H, x->dH, x->ws); break;
        case 4: {
            int nparts = 0;
            gemv_logits(s, B, x->dH, W(x, "language_model.model.norm.weight"), eps,
                        W(x, "language_model.model.embed_tokens.weight"), c.t_vocab, x->dlogits, x->pmax, x->pidx, &nparts);
            break;
        }
        default: return fail(PGMI_E_ARG, "unknown kernel id");
    }
    LAUNCHCHK();
    return 0;
}

int pgmi_preprocess(pgmi_ctx* x, const void* src_hwc, int H, int W, int out_h, int out_w, float* out_chw,
                    void* stream) {
    if (!x || !src_hwc || !out_chw) return fail(PGMI_E_ARG, "null argument");
    if (H < 1 || W < 1 || out_h < 1 || out_w < 1) return fail(PGMI_E_ARG, "empty image");
    if (!x->ws) return fail(PGMI_E_STATE, "workspace not allocated (pgmi_prepare)");
    if (preprocess_scratch_bytes(H, W, out_h, out_w) > x->ws_bytes)
        return fail(PGMI_E_ARG, "image too large for the preprocessing scratch");
    preprocess((hipStream_t)stream, reinterpret_cast<const uint8_t*>(src_hwc), H, W, out_h, out_w, out_chw, x->ws);
    LAUNCHCHK();
    return 0;
}

int pgmi_prefill_kernel(pgmi_ctx* x, int which, int layer, int rows, void* stream) {
    int rc;
    if ((rc = ensure_prepared(x))) return rc;
    const pgmi_config& c = x->c;
    if (rows < 1 || rows > c.max_batch * c.max_seq) return fail(PGMI_E_ARG, "rows exceed the prefill workspace");
    if (layer < 0 || layer >= c.t_layers) return fail(PGMI_E_ARG, "layer out of range");
    hipStream_t s = (hipStream_t)stream;
    const int H = c.t_hidden;
    switch (which) {
        case 0: {  // gate|up GEMM + GeGLU epilogue (modeling_gemma.py:134): Tn -> ACT
            EpiArgs g{};
            g.out = x->ACT; g.ldo = c.t_intermediate;
            gemm(s, x->Tn, H, TL(x, layer, "mlp.gate_proj.weight"), H, rows, c.t_intermediate, H, EPI_GEGLU, g, x->ws,
                 x->ws_bytes, c.t_intermediate);
            break;
        }
        case 1: {  // down GEMM as the prefill runs it: split-K partials (reduced by the next norm)
            EpiArgs d{};
            d.res = x->Hs; d.ldr = H; d.out = x->Hs; d.ldo = H;
            gemm(s, x->ACT, c.t_intermediate, TL(x, layer, "mlp.down_proj.weight"), c.t_intermediate, rows, H,
                 c.t_intermediate, EPI_RES, d, x->ws, x->ws_bytes, 0, true);
            break;
        }
        default: return fail(PGMI_E_ARG, "unknown kernel id");
    }
    LAUNCHCHK();
    return 0;
}

int pgmi_debug_gemm_tiles(int n_mt, int n_nt, int S, int BM, int BN, int K, int* mt, int* nt, int* z) {
    if (n_mt < 1 || n_nt < 1 || S < 1 || !mt || !nt || !z) return fail(PGMI_E_ARG, "bad argument");
    return gemm_tile_order(n_mt, n_nt, S, BM, BN, K, mt, nt, z);
}

int pgmi_tune_gemm(int cfg, int split) {
    if (cfg >= kGemmCfgs || split < 0 || split > 32) return fail(PGMI_E_ARG, "bad GEMM plan");
    gemm_force_plan(cfg, split);
    return 0;
}

int pgmi_tune_gemm_shape(int M, int N, int K, int dual, int cfg, int split) {
    if (cfg >= kGemmCfgs || split < 0 || split > 16) return fail(PGMI_E_ARG, "bad GEMM plan");
    if (gemm_force_shape(M, N, K, dual, cfg, split)) return fail(PGMI_E_ARG, "too many per-shape GEMM plans");
    return 0;
}

int pgmi_tune_attention(int variant) {
    static const int ok[] = {-1, 0, 7, 8, 41, 42, 21, 22, 44, 24, 9, 91, 92, 94, 81, 82};
    for (int v : ok)
        if (v == variant) {
            attention_force_variant(variant);
            return 0;
        }
    return fail(PGMI_E_ARG, "unknown attention variant");
}

int pgmi_sample_top_p(pgmi_ctx* x, const float* logits, int rows, int V, float temperature, float top_p,
                      const float* u, int64_t* out, float* kept_mass, void* stream) {
    if (!x || !logits || !u || !out) return fail(PGMI_E_ARG, "null argument");
    if (rows <= 0 || V <= 0) return fail(PGMI_E_ARG, "sample_top_p: empty probabilities");
    if (!(top_p >= 0.f)) return fail(PGMI_E_ARG, "sample_top_p: top_p must be >= 0");
    if (!x->ws) return fail(PGMI_E_STATE, "workspace not allocated (pgmi_prepare)");
    const int per = (int)std::min<size_t>((size_t)rows, x->ws_bytes / sample_scratch_bytes(1, V));
    if (per < 1) return fail(PGMI_E_ARG, "sample_top_p: vocabulary exceeds the scratch");
    for (int r0 = 0; r0 < rows; r0 += per) {  // row batches that fit the scratch (stream-ordered)
        const int nr = std::min(per, rows - r0);
        sample_top_p((hipStream_t)stream, logits + (size_t)r0 * V, nr, V, temperature, top_p, u + r0, x->ws,
                     out + r0, kept_mass ? kept_mass + r0 : nullptr);
    }
    LAUNCHCHK();
    return 0;
}

// ---------------------------------------------------------------- single ops (tests)
int pgmi_op_gemm(pgmi_ctx* x, const void* A, const void* Wt, int M, int N, int K, int epi, const void* bias,
                 const void* res, void* out, void* stream) {
    int rc;
    if ((rc = ensure_prepared(x))) return rc;
    if (K % 8 != 0) return fail(PGMI_E_ARG, "K must be a multiple of 8");
    EpiArgs e{};
    e.bias = reinterpret_cast<const uint16_t*>(bias);
    e.res = reinterpret_cast<const uint16_t*>(res);
    e.ldr = N;
    e.ldo = N;
    if (epi == EPI_F32) e.out_f32 = reinterpret_cast<float*>(out);
    else e.out = reinterpret_cast<uint16_t*>(out);
    gemm((hipStream_t)stream, reinterpret_cast<const uint16_t*>(A), K, reinterpret_cast<const uint16_t*>(Wt), K, M, N,
         K, (Epi)epi, e, x->ws, x->ws_bytes, epi == EPI_GEGLU ? N : 0);
    LAUNCHCHK();
    return 0;
}

int pgmi_op_gemm_strided(pgmi_ctx* x, const void* A, int lda, const void* Wt, int ldw, int M, int N, int K, int epi,
                         const void* bias, const void* res, void* out, void* stream) {
    int rc;
    if ((rc = ensure_prepared(x))) return rc;
    if (K % 8 != 0 || lda < K || ldw < K || lda % 8 != 0 || ldw % 8 != 0)
        return fail(PGMI_E_ARG, "K, lda, ldw must be multiples of 8 with lda, ldw >= K");
    EpiArgs e{};
    e.bias = reinterpret_cast<const uint16_t*>(bias);
    e.res = reinterpret_cast<const uint16_t*>(res);
    e.ldr = N;
    e.ldo = N;
    if (epi == EPI_F32) e.out_f32 = reinterpret_cast<float*>(out);
    else e.out = reinterpret_cast<uint16_t*>(out);
    gemm((hipStream_t)stream, reinterpret_cast<const uint16_t*>(A), lda, reinterpret_cast<const uint16_t*>(Wt), ldw, M,
         N, K, (Epi)epi, e, x->ws, x->ws_bytes, epi == EPI_GEGLU ? N : 0);
    LAUNCHCHK();
    return 0;
}

int pgmi_op_rmsnorm(pgmi_ctx* x, const void* in, const void* w, int rows, int D, float eps, void* out, void* stream) {
    if (!x) return fail(PGMI_E_ARG, "null ctx");
    rmsnorm((hipStream_t)stream, reinterpret_cast<const uint16_t*>(in), reinterpret_cast<const uint16_t*>(w), eps,
            reinterpret_cast<uint16_t*>(out), rows, D);
    LAUNCHCHK();
    return 0;
}

int pgmi_op_layernorm(pgmi_ctx* x, const void* in, const void* w, const void* b, int rows, int D, float eps, void* out,
                      void* stream) {
    if (!x) return fail(PGMI_E_ARG, "null ctx");
    layernorm((hipStream_t)stream, reinterpret_cast<const uint16_t*>(in), reinterpret_cast<const uint16_t*>(w),
              reinterpret_cast<const uint16_t*>(b), eps, reinterpret_cast<uint16_t*>(out), rows, D);
    LAUNCHCHK();
    return 0;
}

int pgmi_op_add(pgmi_ctx* x, const void* a, const void* b, int64_t n, void* out, void* stream) {
    if (!x) return fail(PGMI_E_ARG, "null ctx");
    if (!a || !b || !out || n < 0) return fail(PGMI_E_ARG, "bad argument");
    if (n % 8 != 0) return fail(PGMI_E_ARG, "n must be a multiple of 8");
    if (n == 0) return 0;
    add_rows((hipStream_t)stream, reinterpret_cast<const uint16_t*>(a), reinterpret_cast<const uint16_t*>(b), (long)n,
             reinterpret_cast<uint16_t*>(out));
    LAUNCHCHK();
    return 0;
}

int pgmi_op_patch_embed(pgmi_ctx* x, const void* pixels, int pixel_dtype, int B, int C, int H, int P, const void* conv_w,
                        const void* conv_b, const void* pos, int D, void* out, void* stream) {
    int rc;
    if ((rc = ensure_prepared(x))) return rc;
    if (!pixels || !conv_w || !conv_b || !pos || !out) return fail(PGMI_E_ARG, "null argument");
    if (pixel_dtype != PGMI_DTYPE_F32 && pixel_dtype != PGMI_DTYPE_BF16) return fail(PGMI_E_ARG, "pixels must be fp32 or bf16");
    if (B < 1 || C < 1 || P < 1 || H < P || H % P != 0 || D < 1 || D % 8 != 0) return fail(PGMI_E_ARG, "bad shape");
    const int N = (H / P) * (H / P), K = C * P * P, Kpad = (K + 63) / 64 * 64;
    // scratch: the conv weight padded to Kpad columns, then the patch rows (modeling_siglip.py:67 as a GEMM)
    const size_t wbytes = ((size_t)D * Kpad * 2 + 255) & ~(size_t)255, pbytes = ((size_t)B * N * Kpad * 2 + 255) & ~(size_t)255;
    if (wbytes + pbytes > x->ws_bytes) return fail(PGMI_E_ARG, "batch too large for the scratch");
    hipStream_t s = (hipStream_t)stream;
    uint16_t* wpad = reinterpret_cast<uint16_t*>(x->ws);
    uint16_t* rows = reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(x->ws) + wbytes);
    pad_rows(s, reinterpret_cast<const uint16_t*>(conv_w), D, K, Kpad, wpad);
    patchify(s, pixels, pixel_dtype == PGMI_DTYPE_F32, B, C, H, H, P, Kpad, rows);
    EpiArgs e{};
    e.bias = reinterpret_cast<const uint16_t*>(conv_b);
    e.pos = reinterpret_cast<const uint16_t*>(pos);
    e.npos = N;
    e.out = reinterpret_cast<uint16_t*>(out);
    e.ldo = D;
    float* gws = reinterpret_cast<float*>(reinterpret_cast<char*>(x->ws) + wbytes + pbytes);
    gemm(s, rows, Kpad, wpad, Kpad, B * N, D, Kpad, EPI_BIAS_POS, e, gws, x->ws_bytes - wbytes - pbytes);
    LAUNCHCHK();
    return 0;
}

int pgmi_op_attention(pgmi_ctx* x, const void* q, const void* k, const void* v, void* o, int B, int Lq, int Lk, int H,
                      int Hkv, int hd, float scale, void* stream) {
    if (!x) return fail(PGMI_E_ARG, "null ctx");
    if (hd != 256 && hd != 72) return fail(PGMI_E_ARG, "head_dim must be 72 or 256");
    if (H % Hkv != 0 || H / Hkv > 16) return fail(PGMI_E_ARG, "bad head grouping");
    AttnArgs a{};
    a.q = reinterpret_cast<const uint16_t*>(q); a.q_b_stride = (long)Lq * H * hd; a.q_row_stride = H * hd; a.q_head_stride = hd;
    a.k = reinterpret_cast<const uint16_t*>(k); a.k_b_stride = (long)Lk * Hkv * hd; a.k_row_stride = Hkv * hd; a.k_head_stride = hd;
    a.v = reinterpret_cast<const uint16_t*>(v); a.v_b_stride = a.k_b_stride; a.v_row_stride = Hkv * hd; a.v_head_stride = hd;
    a.o = reinterpret_cast<uint16_t*>(o); a.o_b_stride = a.q_b_stride; a.o_row_stride = H * hd; a.o_head_stride = hd;
    a.Lq = Lq; a.Lk = Lk; a.G = H / Hkv; a.n_kv = Hkv; a.B = B; a.scale = scale;
    a.ws = x->ws; a.ws_floats = (long)(x->ws_bytes / sizeof(float));
    attention_prefill((hipStream_t)stream, hd, a);
    LAUNCHCHK();
    return 0;
}

int pgmi_op_attention_ex(pgmi_ctx* x, const void* q, const void* k, const void* v, void* o, int B, int Lq, int Lk,
                         int H, int Hkv, int hd, int kv_layout, float scale, int scale_div, const void* mask,
                         int mask_dtype, int64_t m_b_stride, int64_t m_h_stride, int64_t m_q_stride, void* probs,
                         void* stream) {
    if (!x) return fail(PGMI_E_ARG, "null ctx");
    if (!q || !k || !v || !o) return fail(PGMI_E_ARG, "null argument");
    if (B < 1 || Lq < 1 || Lk < 1 || H < 1 || Hkv < 1 || H % Hkv != 0) return fail(PGMI_E_ARG, "bad shape");
    if (hd < 1 || hd > 256) return fail(PGMI_E_ARG, "head_dim must be in [1, 256]");
    if (kv_layout != 0 && kv_layout != 1) return fail(PGMI_E_ARG, "kv_layout must be 0 (B,L,Hkv,hd) or 1 (B,Hkv,L,hd)");
    if (mask && mask_dtype != PGMI_DTYPE_BF16 && mask_dtype != PGMI_DTYPE_F32)
        return fail(PGMI_E_ARG, "mask must be bf16 or fp32");
    if (attention_exact_lds(Lk, hd) > 160 * 1024) return fail(PGMI_E_ARG, "too many keys for one workgroup's scores");
    ModAttnArgs a{};
    a.q = reinterpret_cast<const uint16_t*>(q);
    a.k = reinterpret_cast<const uint16_t*>(k);
    a.v = reinterpret_cast<const uint16_t*>(v);
    a.kv_b_stride = (long)Lk * Hkv * hd;
    a.kv_h_stride = kv_layout == 0 ? hd : (long)Lk * hd;
    a.kv_row_stride = kv_layout == 0 ? (long)Hkv * hd : hd;
    a.o = reinterpret_cast<uint16_t*>(o);
    a.probs = reinterpret_cast<uint16_t*>(probs);
    a.mask = mask;
    a.m_b_stride = m_b_stride;
    a.m_h_stride = m_h_stride;
    a.m_q_stride = m_q_stride;
    a.mask_f32 = mask_dtype == PGMI_DTYPE_F32;
    a.B = B; a.Lq = Lq; a.Lk = Lk; a.H = H; a.Hkv = Hkv; a.hd = hd;
    a.scale = scale;
    a.scale_div = scale_div != 0;
    attention_exact((hipStream_t)stream, a);
    LAUNCHCHK();
    return 0;
}

int pgmi_op_rope(pgmi_ctx* x, const void* in, const void* cos_rows, const void* sin_rows, int64_t rows, int heads,
                 int hd, void* out, void* stream) {
    if (!x) return fail(PGMI_E_ARG, "null ctx");
    if (!in || !cos_rows || !sin_rows || !out) return fail(PGMI_E_ARG, "null argument");
    if (rows < 0 || heads < 1 || hd < 2 || hd % 2 != 0) return fail(PGMI_E_ARG, "bad shape");
    if (rows == 0) return 0;
    rope_rows((hipStream_t)stream, reinterpret_cast<const uint16_t*>(in), reinterpret_cast<const uint16_t*>(cos_rows),
              reinterpret_cast<const uint16_t*>(sin_rows), (long)rows, heads, hd, reinterpret_cast<uint16_t*>(out));
    LAUNCHCHK();
    return 0;
}

int pgmi_op_scale(pgmi_ctx* x, const void* in, float a, int64_t n, void* out, void* stream) {
    if (!x) return fail(PGMI_E_ARG, "null ctx");
    if (!in || !out || n < 0) return fail(PGMI_E_ARG, "bad argument");
    if (n % 8 != 0) return fail(PGMI_E_ARG, "n must be a multiple of 8");
    if (n == 0) return 0;
    scale_rows((hipStream_t)stream, reinterpret_cast<const uint16_t*>(in), (long)n, a, reinterpret_cast<uint16_t*>(out));
    LAUNCHCHK();
    return 0;
}

int pgmi_op_gemv_res(pgmi_ctx* x, const void* in, const void* Wt, int B, int N, int K, void* h, void* stream) {
    if (!x) return fail(PGMI_E_ARG, "null ctx");
    if (K != 2048 && K != 16384) return fail(PGMI_E_ARG, "K must be 2048 or 16384");
    if (B < 1 || B > 8) return fail(PGMI_E_ARG, "B must be in [1, 8]");
    if (!x->ws) return fail(PGMI_E_STATE, "workspace not allocated (pgmi_prepare)");
    if ((size_t)4 * B * N * sizeof(float) > x->ws_bytes) return fail(PGMI_E_ARG, "N too large for the scratch");
    gemv_res((hipStream_t)stream, B, K, reinterpret_cast<const uint16_t*>(in), reinterpret_cast<const uint16_t*>(Wt), N,
             reinterpret_cast<uint16_t*>(h), x->ws);
    LAUNCHCHK();
    return 0;
}

}  // extern "C"
