"""oracle/paligemma_np.py -- TEST INFRASTRUCTURE ONLY.

CPU restatement (numpy, float32 arithmetic with explicit bf16 rounding) of the
reference's PaliGemma inference path.  It rounds to bf16 exactly where the
reference's bf16 modules do (SURVEY.md sec.8a "rounding points" column), so it
is the checker for the HIP path.  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may use it; the product never imports it.

Every function cites the reference file:line it restates.  Pinned against
golden vectors captured from the reference itself (tests/golden/make_golden.py).
"""
from __future__ import annotations

import math

import numpy as np

F32 = np.float32
_FP32_TRUTH = [False]


class fp32_truth:
    """Context manager: every bf16 rounding point becomes the identity, i.e. the reference run
    with its modules in float32 on the same (bf16-valued) weights -- how make_golden.py produced
    the full_*_fp32.npz truths.  Used to measure the reference bf16's own error floor on the
    small configurations (smoke, tests/test_gpu_model_small.py)."""

    def __enter__(self):
        _FP32_TRUTH[0] = True
        return self

    def __exit__(self, *exc):
        _FP32_TRUTH[0] = False
        return False


# ---------------------------------------------------------------- bf16 helpers
def bf16(x) -> np.ndarray:
    """Round float32 -> bf16 (round-to-nearest-even), returned widened to float32."""
    x = np.ascontiguousarray(x, dtype=F32)
    if _FP32_TRUTH[0]:
        return x
    u = x.view(np.uint32)
    r = (u + np.uint32(0x7FFF) + ((u >> np.uint32(16)) & np.uint32(1))) & np.uint32(0xFFFF0000)
    return r.view(F32)


def bf16_bits(x) -> np.ndarray:
    return (bf16(x).view(np.uint32) >> np.uint32(16)).astype(np.uint16)


def from_bits(u16) -> np.ndarray:
    return (np.asarray(u16, dtype=np.uint16).astype(np.uint32) << np.uint32(16)).view(F32)


def linear(x, w, b=None):
    """nn.Linear in bf16: fp32 accumulate (+bias), one rounding
    (modeling_siglip.py:92-95, modeling_gemma.py:129-131,220-223,391,433)."""
    y = np.matmul(x.astype(F32), w.T.astype(F32))
    if b is not None:
        y = y + b
    return bf16(y)


def gelu_tanh(x):
    """nn.functional.gelu(approximate='tanh') on bf16 (fp32 math, one rounding)
    (modeling_siglip.py:162, modeling_gemma.py:134)."""
    x = x.astype(F32)
    k = F32(math.sqrt(2.0 / math.pi))
    inner = k * (x + F32(0.044715) * x * x * x)
    return bf16(F32(0.5) * x * (F32(1.0) + np.tanh(inner)))


def softmax_f32(s):
    """softmax(dim=-1, dtype=float32) (modeling_siglip.py:125, modeling_gemma.py:273)."""
    s = s.astype(F32)
    m = s.max(axis=-1, keepdims=True)
    e = np.exp(s - m)
    return e / e.sum(axis=-1, keepdims=True)


def layer_norm(x, w, b, eps):
    """nn.LayerNorm on bf16 input: fp32 statistics, one rounding
    (modeling_siglip.py:175,177,234)."""
    x = x.astype(F32)
    mu = x.mean(axis=-1, keepdims=True)
    var = ((x - mu) ** 2).mean(axis=-1, keepdims=True)
    return bf16((x - mu) / np.sqrt(var + F32(eps)) * w + b)


def rms_norm(x, w, eps):
    """GemmaRMSNorm: x.float() * rsqrt(mean(x^2)+eps) * (1 + w.float()), one rounding
    (modeling_gemma.py:107-120)."""
    x = x.astype(F32)
    r = F32(1.0) / np.sqrt((x * x).mean(axis=-1, keepdims=True) + F32(eps))
    return bf16((x * r) * (F32(1.0) + w))


# ---------------------------------------------------------------- SigLIP
def siglip_embeddings(P, cfg, pixel_values):
    """SiglipVisionEmbeddings.forward (modeling_siglip.py:62-79): 14x14/14 conv as a
    GEMM over (c, kh, kw)-ordered patches, + bias, round; + position embedding, round.
    pixel_values are cast to bf16 first (modeling_gemma.py:570)."""
    v = cfg["vision_config"]
    p = v["patch_size"]
    x = bf16(pixel_values)
    B, C, H, W = x.shape
    gh, gw = H // p, W // p
    patches = x.reshape(B, C, gh, p, gw, p).transpose(0, 2, 4, 1, 3, 5).reshape(B, gh * gw, C * p * p)
    pre = "vision_tower.vision_model.embeddings."
    wc = P[pre + "patch_embedding.weight"].reshape(v["hidden_size"], -1)
    y = linear(patches, wc, P[pre + "patch_embedding.bias"])
    return bf16(y + P[pre + "position_embedding.weight"][None])


def siglip_attention(P, pre, x, n_heads, taps=None):
    """SiglipAttention.forward (modeling_siglip.py:97-147); taps["probs"] = the attention
    probabilities the reference returns as its second output (:125,147)."""
    B, L, D = x.shape
    hd = D // n_heads
    q = linear(x, P[pre + "q_proj.weight"], P[pre + "q_proj.bias"])
    k = linear(x, P[pre + "k_proj.weight"], P[pre + "k_proj.bias"])
    vv = linear(x, P[pre + "v_proj.weight"], P[pre + "v_proj.bias"])
    q = q.reshape(B, L, n_heads, hd).transpose(0, 2, 1, 3)
    k = k.reshape(B, L, n_heads, hd).transpose(0, 2, 1, 3)
    vv = vv.reshape(B, L, n_heads, hd).transpose(0, 2, 1, 3)
    s = bf16(np.matmul(q, k.transpose(0, 1, 3, 2)))                # :116 matmul -> bf16
    s = bf16(s * F32(hd ** -0.5))                                    # :116 * scale -> bf16
    p = bf16(softmax_f32(s))                                         # :125
    if taps is not None:
        taps["probs"] = p
    o = bf16(np.matmul(p, vv))                                       # :131
    o = o.transpose(0, 2, 1, 3).reshape(B, L, D)                     # :140-142
    return linear(o, P[pre + "out_proj.weight"], P[pre + "out_proj.bias"])  # :145


def siglip_mlp(P, pre, x):
    """SiglipMLP.forward (modeling_siglip.py:157-167)."""
    h = linear(x, P[pre + "fc1.weight"], P[pre + "fc1.bias"])
    h = gelu_tanh(h)
    return linear(h, P[pre + "fc2.weight"], P[pre + "fc2.bias"])


def siglip_layer(P, cfg, i, x):
    """SiglipEncoderLayer.forward (modeling_siglip.py:179-204)."""
    v = cfg["vision_config"]
    eps = v.get("layer_norm_eps", 1e-6)
    pre = f"vision_tower.vision_model.encoder.layers.{i}."
    h = layer_norm(x, P[pre + "layer_norm1.weight"], P[pre + "layer_norm1.bias"], eps)
    h = siglip_attention(P, pre + "self_attn.", h, v["num_attention_heads"])
    x = bf16(h + x)
    h = layer_norm(x, P[pre + "layer_norm2.weight"], P[pre + "layer_norm2.bias"], eps)
    h = siglip_mlp(P, pre + "mlp.", h)
    return bf16(h + x)


def siglip_vision(P, cfg, pixel_values, taps=None):
    """SiglipVisionModel.forward (modeling_siglip.py:236-255)."""
    v = cfg["vision_config"]
    x = siglip_embeddings(P, cfg, pixel_values)
    if taps is not None:
        taps["vision_embeddings"] = x
    for i in range(v["num_hidden_layers"]):
        x = siglip_layer(P, cfg, i, x)
        if taps is not None:
            taps[f"vision_layer{i}"] = x
    pre = "vision_tower.vision_model.post_layernorm."
    return layer_norm(x, P[pre + "weight"], P[pre + "bias"], v.get("layer_norm_eps", 1e-6))


def project(P, feats):
    """PaliGemmaMultiModalProjector.forward (modeling_gemma.py:435-438)."""
    return linear(feats, P["multi_modal_projector.linear.weight"], P["multi_modal_projector.linear.bias"])


# ---------------------------------------------------------------- Gemma
def inv_freq(head_dim=256, base=10000.0):
    """GemmaRotaryEmbedding inv_freq (modeling_gemma.py:151), fp32."""
    e = np.arange(0, head_dim, 2, dtype=np.int64).astype(F32) / F32(head_dim)
    return (F32(1.0) / np.power(F32(base), e, dtype=F32)).astype(F32)


def rope_cos_sin(positions, invf, max_pos=8192):
    """GemmaRotaryEmbedding.forward (modeling_gemma.py:155-185): clamp, fp32
    freqs = inv_freq * pos, emb = cat(freqs, freqs), cos/sin -> bf16."""
    pos = np.clip(np.asarray(positions, dtype=F32), 0, max_pos - 1)
    freqs = pos[..., None].astype(F32) * invf[None, :]
    emb = np.concatenate([freqs, freqs], axis=-1).astype(F32)
    return bf16(np.cos(emb.astype(np.float64)).astype(F32)), bf16(np.sin(emb.astype(np.float64)).astype(F32))


def rotate_half(x):
    """modeling_gemma.py:187-191."""
    h = x.shape[-1] // 2
    return np.concatenate([-x[..., h:], x[..., :h]], axis=-1)


def apply_rope(x, cos, sin):
    """apply_rotary_pos_emb (modeling_gemma.py:193-199): three bf16 roundings."""
    return bf16(bf16(x * cos) + bf16(rotate_half(x) * sin))


class KV:
    """KVCache (modeling_gemma.py:10-36): per-layer K/V appended on the seq axis."""

    def __init__(self):
        self.k, self.v = [], []

    def num_items(self):
        return 0 if not self.k else self.k[0].shape[-2]

    def update(self, k, v, i):
        if len(self.k) <= i:
            self.k.append(k)
            self.v.append(v)
        else:
            self.k[i] = np.concatenate([self.k[i], k], axis=-2)
            self.v[i] = np.concatenate([self.v[i], v], axis=-2)
        return self.k[i], self.v[i]


def gemma_attention(P, cfg, i, x, positions, kv, invf, mask=None, taps=None):
    """GemmaAttention.forward (modeling_gemma.py:231-293).  mask: the additive attention mask
    (:269, bf16-valued, broadcast to (B, H, Lq, Lk)); None = the all-zero mask the merge builds
    (:506-511).  taps["probs"] = the probabilities the reference returns (:273,293)."""
    t = cfg["text_config"]
    NH, NKV, HD = t["num_attention_heads"], t["num_key_value_heads"], t.get("head_dim", 256)
    pre = f"language_model.model.layers.{i}.self_attn."
    B, L, _ = x.shape
    q = linear(x, P[pre + "q_proj.weight"]).reshape(B, L, NH, HD).transpose(0, 2, 1, 3)
    k = linear(x, P[pre + "k_proj.weight"]).reshape(B, L, NKV, HD).transpose(0, 2, 1, 3)
    v = linear(x, P[pre + "v_proj.weight"]).reshape(B, L, NKV, HD).transpose(0, 2, 1, 3)
    cos, sin = rope_cos_sin(positions, invf, t.get("max_position_embeddings", 8192))
    cos, sin = cos[:, None], sin[:, None]
    q = apply_rope(q, cos, sin)
    k = apply_rope(k, cos, sin)
    if kv is not None:
        k, v = kv.update(k, v, i)
    rep = NH // NKV
    k = np.repeat(k, rep, axis=1)                                    # repeat_kv :136-141
    v = np.repeat(v, rep, axis=1)
    s = bf16(np.matmul(q, k.transpose(0, 1, 3, 2)))                  # :266 matmul
    s = bf16(s / F32(math.sqrt(HD)))                                 # :266 / sqrt(d)
    if mask is not None:
        s = bf16(s + mask)                                           # :269
    p = bf16(softmax_f32(s))                                         # :273
    if taps is not None:
        taps["probs"] = p
    o = bf16(np.matmul(p, v))                                        # :277
    o = o.transpose(0, 2, 1, 3).reshape(B, L, NH * HD)
    return linear(o, P[pre + "o_proj.weight"])                       # :291


def gemma_mlp(P, i, x):
    """GemmaMLP.forward (modeling_gemma.py:133-134): down(gelu_tanh(gate(x)) * up(x))."""
    pre = f"language_model.model.layers.{i}.mlp."
    g = gelu_tanh(linear(x, P[pre + "gate_proj.weight"]))
    u = linear(x, P[pre + "up_proj.weight"])
    return linear(bf16(g * u), P[pre + "down_proj.weight"])


def gemma_forward(P, cfg, embeds, positions, kv, invf=None, taps=None, all_logits=True, mask=None):
    """GemmaForCausalLM.forward (modeling_gemma.py:399-427) over GemmaModel.forward
    (:357-382) and GemmaDecoderLayer.forward (:307-338); mask: the additive attention mask every
    layer adds (:269), None = the merge's zero mask."""
    t = cfg["text_config"]
    eps = t.get("rms_norm_eps", 1e-6)
    if invf is None:
        invf = inv_freq(t.get("head_dim", 256), t.get("rope_theta", 10000.0))
    normalizer = bf16(np.array([math.sqrt(t["hidden_size"])], F32))[0]   # :367 (bf16 45.25)
    h = bf16(embeds * normalizer)                                        # :368
    for i in range(t["num_hidden_layers"]):
        pre = f"language_model.model.layers.{i}."
        x = rms_norm(h, P[pre + "input_layernorm.weight"], eps)
        x = gemma_attention(P, cfg, i, x, positions, kv, invf, mask=mask)
        h = bf16(x + h)
        x = rms_norm(h, P[pre + "post_attention_layernorm.weight"], eps)
        x = gemma_mlp(P, i, x)
        h = bf16(x + h)
        if taps is not None:
            taps[f"text_layer{i}"] = h
    h = rms_norm(h, P["language_model.model.norm.weight"], eps)          # :379
    if not all_logits:
        h = h[:, -1:]
    return linear(h, P["language_model.model.embed_tokens.weight"])      # :417-418 (tied)


def merge(P, cfg, image_features, input_ids):
    """_merge_input_ids_with_image_features (modeling_gemma.py:468-537), embedding side:
    text rows from embed_tokens, image rows = features / sqrt(hidden), pad rows zero."""
    E = P["language_model.model.embed_tokens.weight"]
    ids = np.asarray(input_ids)
    emb = E[ids]                                                         # :565
    img_idx, pad = cfg["image_token_index"], cfg.get("pad_token_id", 0)
    pad = -1 if pad is None else pad
    out = np.zeros_like(emb)
    text = (ids != img_idx) & (ids != pad)
    out[text] = emb[text]
    if image_features is not None and image_features.shape[1] > 0:
        scaled = bf16(image_features / F32(cfg["hidden_size"] ** 0.5))  # :481
        imask = ids == img_idx
        out[imask] = scaled.reshape(-1, scaled.shape[-1])[: int(imask.sum())]
    return out


def paligemma_prefill(P, cfg, input_ids, pixel_values, taps=None, all_logits=True):
    """PaliGemmaForConditionalGeneration.forward with an empty KVCache
    (modeling_gemma.py:539-617; positions 0..L-1 :532-535, non-causal mask :506-507)."""
    feats = None
    if pixel_values is not None:
        feats = project(P, siglip_vision(P, cfg, pixel_values, taps))
        if taps is not None:
            taps["image_features"] = feats
    emb = merge(P, cfg, feats, input_ids)
    B, L = np.asarray(input_ids).shape
    kv = KV()
    pos = np.broadcast_to(np.arange(L), (B, L))
    logits = gemma_forward(P, cfg, emb, pos, kv, taps=taps, all_logits=all_logits)
    return logits, kv


def paligemma_decode(P, cfg, next_ids, kv, mask_len):
    """One decode step with inference.py semantics: input_ids (B,1), attention_mask has
    `mask_len` ones, position = cumsum(mask)[-1] = mask_len (modeling_gemma.py:516-528),
    which after prefill of L tokens is L+1 (the position-id gap)."""
    ids = np.asarray(next_ids).reshape(-1, 1)
    emb = merge(P, cfg, None, ids)
    pos = np.full((ids.shape[0], 1), mask_len, dtype=np.int64)
    return gemma_forward(P, cfg, emb, pos, kv)


def greedy_generate(P, cfg, input_ids, pixel_values, n_tokens, eos=None):
    """inference.py:test_inference greedy loop (inference.py:55-78)."""
    logits, kv = paligemma_prefill(P, cfg, input_ids, pixel_values, all_logits=False)
    L = np.asarray(input_ids).shape[1]
    toks, step_logits = [], []
    mask_len = L
    for _ in range(n_tokens):
        last = logits[:, -1, :]
        step_logits.append(last)
        nxt = np.argmax(last, axis=-1)
        toks.append(nxt)
        if eos is not None and int(nxt[0]) == eos:
            break
        mask_len += 1
        logits = paligemma_decode(P, cfg, nxt, kv, mask_len)
    return np.stack(toks, axis=1), np.stack(step_logits, axis=1)


def ablation_generate(P, cfg, input_ids, pixel_values, n_tokens, kv_mode):
    """The ablation harness's greedy loop (ablation_study_fixed.py:168-251, run_inference with
    temperature 0.0) under load_model_simple's two patches (:335-342):
      * the patched merge (:99-142): with a filled cache EVERY query row sits at the single position
        cumsum(mask)[:, -1:] (:130-133) and attends cached + q_len keys (:124-126); otherwise
        positions 0..L-1 clamped to max_position_embeddings - 1 (:135-140);
      * the patched rotary (:144-166): positions clamped, fp32 angles cast to bf16 (= rope_cos_sin).
    KV mode: a discarded prefill (:194-199), then step 0 re-feeds prompt + pixels into the filled
    cache, then one-token steps without pixels (:238-243).  no-KV mode: every step is a fresh
    prefill over prompt + generated with the pixels (:244-251).
    run_inference's `model = model.to(config["dtype"])` (:182) casts every floating buffer, the
    rotary inv_freq included, so the angles come from bf16-rounded inverse frequencies.
    Returns (tokens (n,), last-row logits (n, V))."""
    ids0 = np.asarray(input_ids)
    B, L = ids0.shape
    t = cfg["text_config"]
    max_pos = t.get("max_position_embeddings", 8192)
    invf = bf16(inv_freq(t.get("head_dim", 256), t.get("rope_theta", 10000.0)))
    feats = project(P, siglip_vision(P, cfg, pixel_values))
    toks, steps = [], []
    if kv_mode:
        kv = KV()
        emb = merge(P, cfg, feats, ids0)
        gemma_forward(P, cfg, emb, np.broadcast_to(np.minimum(np.arange(L), max_pos - 1), (B, L)), kv, invf,
                      all_logits=False)                                          # discarded prefill
        cur, mask_len, with_px = ids0, L, True
        for _ in range(n_tokens):
            emb = merge(P, cfg, feats if with_px else None, cur)
            q = cur.shape[1]
            pos = np.full((B, q), mask_len, dtype=np.int64)                      # cumsum(mask)[:, -1:]
            last = gemma_forward(P, cfg, emb, pos, kv, invf, all_logits=False)[:, -1, :]
            nxt = np.argmax(last, axis=-1)
            steps.append(last)
            toks.append(nxt)
            cur, mask_len, with_px = nxt.reshape(B, 1), mask_len + 1, False
    else:
        gen = []
        for _ in range(n_tokens):
            cur = np.concatenate([ids0, np.array(gen, dtype=np.int64).reshape(B, -1)], axis=1) if gen else ids0
            n = cur.shape[1]
            emb = merge(P, cfg, feats, cur)
            last = gemma_forward(P, cfg, emb, np.broadcast_to(np.minimum(np.arange(n), max_pos - 1), (B, n)), KV(),
                                 invf, all_logits=False)[:, -1, :]
            nxt = np.argmax(last, axis=-1)
            steps.append(last)
            toks.append(nxt)
            gen.append(int(nxt[0]))
    return np.stack(toks, axis=1), np.stack(steps, axis=1)
