"""Per-layer module forwards of the drop-in model (SigLIP layers; GemmaRMSNorm, GemmaMLP, GemmaAttention,
GemmaDecoderLayer, GemmaModel) on libpgmi's single-op C-ABI entries (include/pgmi.h: pgmi_op_gemm /
_layernorm / _rmsnorm / _attention / _attention_ex / _rope / _add / _scale / _patch_embed).

The whole-model forwards (PaliGemmaForConditionalGeneration, SiglipVisionModel, GemmaForCausalLM) run
the fused engine and never call these; they exist so that a submodule called on its own -- and any
forward hook registered on it -- behaves as the reference module does (modeling_siglip.py:62-223,
modeling_gemma.py:107-134), with the reference's bf16 rounding points:
  * nn.Linear + bias         -> bf16(acc + bias)                        (GEMM epilogue 1)
  * fc1 + gelu(tanh)         -> bf16(gelu(bf16(acc + bias)))            (epilogue 2)
  * gate/up + GeGLU          -> bf16(bf16(gelu(bf16(g))) * bf16(u))     (epilogue 7, gate|up rows stacked)
  * residual adds            -> bf16(a + b)                             (pgmi_op_add)
  * rotary                   -> bf16(bf16(x*cos) + bf16(rotate_half(x)*sin)) (pgmi_op_rope)
  * attention                -> bf16(q.k), bf16(* scale | / sqrt(hd)), bf16(+ mask), bf16(softmax_fp32),
                                bf16(p.v); the probabilities are returned as the reference returns them
                                (pgmi_op_attention_ex)
Every op runs on a small context of its own per (device, stream) -- the context's scratch holds split-K
partials, so two streams never share one (weights are passed by pointer); inputs and parameters are bf16
on the GPU (other float dtypes are rounded to bf16, as the fused path does).
"""
from __future__ import annotations

import math
from collections import OrderedDict

import torch

from . import _native as N
from .engine import Engine

EPI_STORE, EPI_BIAS, EPI_BIAS_GELU, EPI_BIAS_RES, EPI_RES, EPI_GEGLU = 0, 1, 2, 3, 4, 7
_CTX: "OrderedDict" = OrderedDict()   # (device, stream handle) -> (Engine, the torch stream)
_CTX_MAX = 8  # contexts kept (least recently used evicted): callers that make streams per call stay bounded
_RETIRED: list = []  # evicted contexts still possibly read by their stream: (event, Engine)


def _reap() -> None:
    """Free the evicted contexts whose stream has passed the event recorded at eviction."""
    keep = []
    for ev, e in _RETIRED:
        if not ev.query():
            keep.append((ev, e))
    _RETIRED[:] = keep


def _ctx(device: torch.device) -> Engine:
    """Context for the single-op entries on (device, current stream): a zero-layer model whose scratch
    (split-K partials, patch-embedding staging, attention partials) is used from offset 0 by every op,
    so ops issued on different streams get different contexts and never overwrite each other's.  At most
    _CTX_MAX contexts are kept; an evicted one is freed once its stream has passed an event recorded at
    eviction (no device-wide synchronisation in the middle of an op; nothing is evicted while the current
    stream is being captured into a CUDA graph)."""
    dev = device.index if device.index is not None else torch.cuda.current_device()
    cur = torch.cuda.current_stream(dev)
    key = (dev, cur.cuda_stream)
    hit = _CTX.get(key)
    if hit is not None:
        _CTX.move_to_end(key)
        return hit[0]
    capturing = torch.cuda.is_current_stream_capturing()
    if not capturing:
        _reap()
        while len(_CTX) >= _CTX_MAX:
            _, (old, ostream) = _CTX.popitem(last=False)
            # its scratch may still be read by kernels queued on its stream (torch streams are pooled, never
            # destroyed, so the handle stays valid): freed once that stream passes this event
            ev = torch.cuda.Event()
            ev.record(ostream)
            _RETIRED.append((ev, old))
    from .binding import _DUMMY_TEXT, _DUMMY_VISION
    from .synthetic import init_policy
    cfg = {"vision_config": dict(_DUMMY_VISION), "text_config": dict(_DUMMY_TEXT), "image_token_index": 7,
           "projection_dim": 2048, "pad_token_id": None}
    e = Engine(cfg, device=torch.device("cuda", dev), max_batch=1, max_seq=64, max_kv=64)
    e.fill_synthetic(0, init_policy)
    e.prepare()
    _CTX[key] = (e, cur)
    return e


def _bf(t: torch.Tensor) -> torch.Tensor:
    if t.device.type != "cuda":
        raise RuntimeError("libpgmi runs on an MI355X GPU only (no CPU fallback): move the module and its "
                           "input to the GPU first")
    return t.to(torch.bfloat16).contiguous()


def linear(x: torch.Tensor, weight: torch.Tensor, bias=None, epi: int = EPI_STORE, res=None) -> torch.Tensor:
    """x (..., K) @ weight (N, K)^T with the epilogue `epi` -> (..., N) bf16."""
    xs = _bf(x)
    K = xs.shape[-1]
    M = xs.numel() // K
    w = _bf(weight)
    Nn = w.shape[0] // (2 if epi == EPI_GEGLU else 1)
    out = torch.empty((*xs.shape[:-1], Nn), dtype=torch.bfloat16, device=xs.device)
    b = _bf(bias) if bias is not None else None
    r = _bf(res) if res is not None else None
    e = _ctx(xs.device)
    N.check(e.lib.pgmi_op_gemm(e.ctx, xs.data_ptr(), w.data_ptr(), M, Nn, K, epi, N.ptr(b), N.ptr(r),
                               out.data_ptr(), N.stream_handle(xs.device)), "pgmi_op_gemm")
    return out


def layer_norm(x: torch.Tensor, weight, bias, eps: float) -> torch.Tensor:
    xs = _bf(x)
    D = xs.shape[-1]
    out = torch.empty_like(xs)
    e = _ctx(xs.device)
    N.check(e.lib.pgmi_op_layernorm(e.ctx, xs.data_ptr(), _bf(weight).data_ptr(), _bf(bias).data_ptr(),
                                    xs.numel() // D, D, float(eps), out.data_ptr(), N.stream_handle(xs.device)),
            "pgmi_op_layernorm")
    return out


def rms_norm(x: torch.Tensor, weight, eps: float) -> torch.Tensor:
    xs = _bf(x)
    D = xs.shape[-1]
    out = torch.empty_like(xs)
    e = _ctx(xs.device)
    N.check(e.lib.pgmi_op_rmsnorm(e.ctx, xs.data_ptr(), _bf(weight).data_ptr(), xs.numel() // D, D, float(eps),
                                  out.data_ptr(), N.stream_handle(xs.device)), "pgmi_op_rmsnorm")
    return out


def add(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    xa, xb = _bf(a), _bf(b)
    if xa.shape != xb.shape:
        raise ValueError(f"shape mismatch {tuple(xa.shape)} vs {tuple(xb.shape)}")
    out = torch.empty_like(xa)
    e = _ctx(xa.device)
    N.check(e.lib.pgmi_op_add(e.ctx, xa.data_ptr(), xb.data_ptr(), xa.numel(), out.data_ptr(),
                              N.stream_handle(xa.device)), "pgmi_op_add")
    return out


def attention(q, k, v, n_heads: int, n_kv: int, head_dim: int, scale: float) -> torch.Tensor:
    """q (B, Lq, H*hd), k/v (B, Lk, Hkv*hd) -> (B, Lq, H*hd): bf16(bf16(softmax(bf16(bf16(q.k)*scale))) . v)."""
    qs, ks, vs = _bf(q), _bf(k), _bf(v)
    B, Lq, Lk = qs.shape[0], qs.shape[1], ks.shape[1]
    out = torch.empty_like(qs)
    e = _ctx(qs.device)
    N.check(e.lib.pgmi_op_attention(e.ctx, qs.data_ptr(), ks.data_ptr(), vs.data_ptr(), out.data_ptr(), B, Lq, Lk,
                                    n_heads, n_kv, head_dim, float(scale), N.stream_handle(qs.device)),
            "pgmi_op_attention")
    return out


def attention_ex(q, k, v, n_heads: int, n_kv: int, head_dim: int, scale: float, scale_div: bool = False,
                 kv_layout: int = 0, mask=None):
    """Reference-order attention returning (o, probs): q (B, Lq, H*hd) rows; k/v (B, Lk, Hkv*hd) rows
    (kv_layout 0) or (B, Hkv, Lk, hd) (kv_layout 1, the KVCache layout); mask additive, broadcastable
    to (B, H, Lq, Lk) -> o (B, Lq, H*hd), probs (B, H, Lq, Lk) bf16."""
    qs, ks, vs = _bf(q), _bf(k), _bf(v)
    B, Lq = qs.shape[0], qs.shape[1]
    Lk = ks.shape[1] if kv_layout == 0 else ks.shape[2]
    out = torch.empty((B, Lq, n_heads * head_dim), dtype=torch.bfloat16, device=qs.device)
    probs = torch.empty((B, n_heads, Lq, Lk), dtype=torch.bfloat16, device=qs.device)
    mp, mdt, ms = None, N.DTYPE_BF16, (0, 0, 0)
    if mask is not None:
        m = torch.as_tensor(mask, device=qs.device)
        if m.dtype not in (torch.bfloat16, torch.float32):
            m = m.float()                                   # torch promotes bf16 + (fp16 | fp64) past bf16
        m = m.broadcast_to((B, n_heads, Lq, Lk))
        if m.stride(-1) != 1:
            m = m.contiguous()
        mp, mdt, ms = m, (N.DTYPE_F32 if m.dtype == torch.float32 else N.DTYPE_BF16), m.stride()[:3]
    e = _ctx(qs.device)
    N.check(e.lib.pgmi_op_attention_ex(e.ctx, qs.data_ptr(), ks.data_ptr(), vs.data_ptr(), out.data_ptr(), B, Lq, Lk,
                                       n_heads, n_kv, head_dim, kv_layout, float(scale), int(bool(scale_div)),
                                       N.ptr(mp), mdt, ms[0], ms[1], ms[2], probs.data_ptr(),
                                       N.stream_handle(qs.device)), "pgmi_op_attention_ex")
    return out, probs


def rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, heads: int, head_dim: int) -> torch.Tensor:
    """apply_rotary_pos_emb on one projection: x (B, L, heads*hd), cos/sin broadcastable to (B, L, hd)."""
    xs = _bf(x)
    B, L = xs.shape[0], xs.shape[1]
    c = _bf(cos.broadcast_to((B, L, head_dim)))
    s_ = _bf(sin.broadcast_to((B, L, head_dim)))
    out = torch.empty_like(xs)
    e = _ctx(xs.device)
    N.check(e.lib.pgmi_op_rope(e.ctx, xs.data_ptr(), c.data_ptr(), s_.data_ptr(), B * L, heads, head_dim,
                               out.data_ptr(), N.stream_handle(xs.device)), "pgmi_op_rope")
    return out


def scale(x: torch.Tensor, a: float) -> torch.Tensor:
    """bf16(x * a), a already in the reference's precision (GemmaModel's bf16 normalizer)."""
    xs = _bf(x)
    out = torch.empty_like(xs)
    e = _ctx(xs.device)
    N.check(e.lib.pgmi_op_scale(e.ctx, xs.data_ptr(), float(a), xs.numel(), out.data_ptr(), N.stream_handle(xs.device)),
            "pgmi_op_scale")
    return out


# ---------------------------------------------------------------- module forwards

def siglip_embeddings_forward(self, pixel_values: torch.FloatTensor) -> torch.Tensor:
    """SiglipVisionEmbeddings.forward (modeling_siglip.py:62-79): patch conv + bias + position embedding."""
    px = pixel_values
    if px.device.type != "cuda":
        raise RuntimeError("libpgmi runs on an MI355X GPU only (no CPU fallback)")
    if px.dtype not in (torch.float32, torch.bfloat16):
        px = px.float()
    px = px.contiguous()
    B, C, H, _ = px.shape
    Pp, D = self.patch_size, self.embed_dim
    out = torch.empty((B, (H // Pp) ** 2, D), dtype=torch.bfloat16, device=px.device)
    e = _ctx(px.device)
    cw, cb, pe = _bf(self.patch_embedding.weight), _bf(self.patch_embedding.bias), _bf(self.position_embedding.weight)
    N.check(e.lib.pgmi_op_patch_embed(e.ctx, px.data_ptr(), 2 if px.dtype == torch.float32 else 0, B, C, H, Pp,
                                      cw.data_ptr(), cb.data_ptr(), pe.data_ptr(), D, out.data_ptr(),
                                      N.stream_handle(px.device)), "pgmi_op_patch_embed")
    return out


def siglip_attention_forward(self, hidden_states: torch.Tensor):
    """SiglipAttention.forward (modeling_siglip.py:97-147): (attn_output, attn_weights), the
    probabilities (B, H, L, L) bf16 as the reference returns them (:125,147)."""
    q = linear(hidden_states, self.q_proj.weight, self.q_proj.bias, EPI_BIAS)
    k = linear(hidden_states, self.k_proj.weight, self.k_proj.bias, EPI_BIAS)
    v = linear(hidden_states, self.v_proj.weight, self.v_proj.bias, EPI_BIAS)
    o, probs = attention_ex(q, k, v, self.num_heads, self.num_heads, self.head_dim, self.scale)
    return linear(o, self.out_proj.weight, self.out_proj.bias, EPI_BIAS), probs


def siglip_mlp_forward(self, hidden_states: torch.Tensor) -> torch.Tensor:
    """SiglipMLP.forward (modeling_siglip.py:157-167): fc2(gelu_tanh(fc1(x)))."""
    h = linear(hidden_states, self.fc1.weight, self.fc1.bias, EPI_BIAS_GELU)
    return linear(h, self.fc2.weight, self.fc2.bias, EPI_BIAS)


def siglip_encoder_layer_forward(self, hidden_states: torch.Tensor) -> torch.Tensor:
    """SiglipEncoderLayer.forward (modeling_siglip.py:179-204): the submodules are called as modules,
    so their forward hooks fire as in the reference."""
    residual = hidden_states
    h = self.layer_norm1(hidden_states)
    h, _ = self.self_attn(hidden_states=h)
    h = add(residual, h)
    residual = h
    h = self.layer_norm2(h)
    h = self.mlp(h)
    return add(residual, h)


def siglip_encoder_forward(self, inputs_embeds: torch.Tensor) -> torch.Tensor:
    """SiglipEncoder.forward (modeling_siglip.py:215-223)."""
    h = inputs_embeds
    for layer in self.layers:
        h = layer(h)
    return h


def gemma_rmsnorm_forward(self, x: torch.Tensor) -> torch.Tensor:
    """GemmaRMSNorm.forward (modeling_gemma.py:107-120): x * rsqrt(mean(x^2) + eps) * (1 + w), in fp32,
    rounded to bf16."""
    return rms_norm(x, self.weight, self.eps)


def gemma_mlp_forward(self, x: torch.Tensor) -> torch.Tensor:
    """GemmaMLP.forward (modeling_gemma.py:133-134): down(gelu_tanh(gate(x)) * up(x)); gate and up rows
    stacked into one GEMM (the slab keeps them adjacent; otherwise they are stacked here)."""
    g, u = self.gate_proj.weight, self.up_proj.weight
    if (g.dtype == torch.bfloat16 and u.dtype == torch.bfloat16 and g.is_contiguous() and u.is_contiguous()
            and g.untyped_storage().data_ptr() == u.untyped_storage().data_ptr()
            and u.data_ptr() == g.data_ptr() + g.numel() * g.element_size()):
        gu = g.as_strided((2 * g.shape[0], g.shape[1]), (g.shape[1], 1))  # the slab's adjacent gate|up rows
    else:
        gu = torch.cat([_bf(g), _bf(u)], 0)
    act = linear(x, gu, None, EPI_GEGLU)
    return linear(act, self.down_proj.weight, None, EPI_STORE)


def _proj(x, lin):
    return linear(x, lin.weight, lin.bias, EPI_BIAS if lin.bias is not None else EPI_STORE)


def gemma_attention_forward(self, hidden_states: torch.Tensor, attention_mask=None, position_ids=None,
                            kv_cache=None, **kwargs):
    """GemmaAttention.forward (modeling_gemma.py:231-293): q/k/v projections, the module's own
    rotary_emb (monkey-patchable, ablation_study_fixed.py:144-166) applied by pgmi_op_rope,
    kv_cache.update (:258-259), repeat_kv folded into the attention's head mapping, the additive
    mask, o_proj.  Returns (attn_output, attn_weights)."""
    bsz, q_len, _ = hidden_states.size()
    H, Hkv, hd = self.num_heads, self.num_key_value_heads, self.head_dim
    q = _proj(hidden_states, self.q_proj)
    k = _proj(hidden_states, self.k_proj)
    v = _proj(hidden_states, self.v_proj)
    value_states = v.view(bsz, q_len, Hkv, hd).transpose(1, 2)
    cos, sin = self.rotary_emb(value_states, position_ids, seq_len=None)   # (B|1, L, hd)
    q = rope(q, cos, sin, H, hd)
    k = rope(k, cos, sin, Hkv, hd)
    key_states = k.view(bsz, q_len, Hkv, hd).transpose(1, 2)
    if kv_cache is not None:
        key_states, value_states = kv_cache.update(key_states, value_states, self.layer_idx)
    assert attention_mask is not None                                      # :268
    o, probs = attention_ex(q, key_states.contiguous(), value_states.contiguous(), H, Hkv, hd, math.sqrt(hd),
                            scale_div=True, kv_layout=1, mask=attention_mask)
    if o.size() != (bsz, q_len, H * hd):
        raise ValueError(f" attn_output should be of size {(bsz, H, q_len, hd)}, but is {tuple(o.shape)}")
    return _proj(o, self.o_proj), probs


def gemma_decoder_layer_forward(self, hidden_states=None, attention_mask=None, position_ids=None, kv_cache=None):
    """GemmaDecoderLayer.forward (modeling_gemma.py:307-338): the submodules are called as modules,
    so their forward hooks fire as in the reference."""
    residual = hidden_states
    h = self.input_layernorm(hidden_states)
    h, _ = self.self_attn(hidden_states=h, attention_mask=attention_mask, position_ids=position_ids, kv_cache=kv_cache)
    h = add(residual, h)
    residual = h
    h = self.post_attention_layernorm(h)
    h = self.mlp(h)
    return add(residual, h)


def gemma_model_forward(self, attention_mask=None, position_ids=None, inputs_embeds=None, kv_cache=None):
    """GemmaModel.forward (modeling_gemma.py:357-382): x bf16(sqrt(hidden)) (:367-368, the normalizer
    rounded to the embeddings' dtype as torch.tensor(..., dtype=...) does), the layers, the final norm."""
    h = inputs_embeds
    normalizer = float(torch.tensor(self.config.hidden_size ** 0.5, dtype=torch.bfloat16))
    h = scale(h, normalizer)
    for decoder_layer in self.layers:
        h = decoder_layer(h, attention_mask=attention_mask, position_ids=position_ids, kv_cache=kv_cache)
    return self.norm(h)
