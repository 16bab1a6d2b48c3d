"""Per-layer module forwards of the drop-in model (SigLIP layers, GemmaRMSNorm, GemmaMLP) on libpgmi's
single-op C-ABI entries (include/pgmi.h: pgmi_op_gemm / _layernorm / _rmsnorm / _attention / _add /
_patch_embed).

The whole-model forwards (PaliGemmaForConditionalGeneration, SiglipVisionModel, GemmaForCausalLM) run
the fused engine and never call these; they exist so that a submodule called on its own -- and any
forward hook registered on it -- behaves as the reference module does (modeling_siglip.py:62-223,
modeling_gemma.py:107-134), with the reference's bf16 rounding points:
  * nn.Linear + bias         -> bf16(acc + bias)                        (GEMM epilogue 1)
  * fc1 + gelu(tanh)         -> bf16(gelu(bf16(acc + bias)))            (epilogue 2)
  * gate/up + GeGLU          -> bf16(bf16(gelu(bf16(g))) * bf16(u))     (epilogue 7, gate|up rows stacked)
  * residual adds            -> bf16(a + b)                             (pgmi_op_add)
Every op runs on a small per-device context of its own (weights are passed by pointer); inputs and
parameters are bf16 on the GPU (other float dtypes are rounded to bf16, as the fused path does).
"""
from __future__ import annotations

import torch

from . import _native as N
from .engine import Engine

EPI_STORE, EPI_BIAS, EPI_BIAS_GELU, EPI_BIAS_RES, EPI_RES, EPI_GEGLU = 0, 1, 2, 3, 4, 7
_CTX = {}


def _ctx(device: torch.device) -> Engine:
    """Per-device context for the single-op entries (a zero-layer model: only its scratch is used)."""
    key = device.index if device.index is not None else torch.cuda.current_device()
    e = _CTX.get(key)
    if e is None:
        from .binding import _DUMMY_TEXT, _DUMMY_VISION
        from .synthetic import init_policy
        cfg = {"vision_config": dict(_DUMMY_VISION), "text_config": dict(_DUMMY_TEXT), "image_token_index": 7,
               "projection_dim": 2048, "pad_token_id": None}
        e = Engine(cfg, device=torch.device("cuda", key), max_batch=1, max_seq=64, max_kv=64)
        e.fill_synthetic(0, init_policy)
        e.prepare()
        _CTX[key] = e
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
    """SiglipAttention.forward (modeling_siglip.py:97-147).  Returns (attn_output, None): the fused
    attention never materialises the (B, H, L, L) probability matrix the reference also returns."""
    q = linear(hidden_states, self.q_proj.weight, self.q_proj.bias, EPI_BIAS)
    k = linear(hidden_states, self.k_proj.weight, self.k_proj.bias, EPI_BIAS)
    v = linear(hidden_states, self.v_proj.weight, self.v_proj.bias, EPI_BIAS)
    o = attention(q, k, v, self.num_heads, self.num_heads, self.head_dim, self.scale)
    return linear(o, self.out_proj.weight, self.out_proj.bias, EPI_BIAS), None


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
