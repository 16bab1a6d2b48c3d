"""Torch-CPU restatement of the KV-cached Gemma decode step -- the CPU "beside" number of bench.py.

TEST / MEASUREMENT INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg and tests/ use it; the product path
(libpgmi) never imports it.  It is a builder-written port, not the reference's code: the same arithmetic as
one inference.py loop iteration (inference.py:56-78) through GemmaForCausalLM (modeling_gemma.py:357-427) in
bf16 on the host, with the rounding points of the reference's modules:

  embedding x bf16(sqrt(hidden))                                   modeling_gemma.py:367-368
  RMSNorm in fp32, (1 + w), cast back to bf16                      :114-120
  q|k|v projections (bf16 linear), RoPE with fp32 angles -> bf16   :241-256, :178-185, :193-199
  attention: bf16(q.k) / sqrt(256), softmax in fp32 -> bf16, p.v   :266-277 (MQA: one KV head, :136-141)
  o_proj, residual, RMSNorm, GeGLU MLP (tanh GELU), residual       :291, :327-336, :133-134
  final RMSNorm, tied lm_head, .float()                            :379, :417-418

Engineering choices of this port (not the reference's): the q|k|v and gate|up weight rows are concatenated
so each is one linear call, and the KV cache is a preallocated [layer][token][256] slab written in place
(the reference concatenates per step, KVCache.update :22-36).  tests/test_cpu_oracle.py holds it to the
numpy oracle (oracle/paligemma_np.py) on the same synthetic weights.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

from oracle import weights as OW


def _bf16(a: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(a.view(np.int16).copy()).view(torch.bfloat16)


class TorchCpuDecoder:
    """Gemma text model of `cfg` on synthetic weights (oracle/wgen.c, seed), bf16, decode only."""

    def __init__(self, cfg: dict, seed: int, max_kv: int):
        t = cfg["text_config"]
        self.H, self.I = t["hidden_size"], t["intermediate_size"]
        self.nh, self.nkv, self.hd = t["num_attention_heads"], t["num_key_value_heads"], t.get("head_dim", 256)
        self.eps = t.get("rms_norm_eps", 1e-6)
        self.max_pos = t.get("max_position_embeddings", 8192)
        self.L = t["num_hidden_layers"]
        shapes = {n: s for n, s in OW.param_shapes(cfg).items() if n.startswith("language_model")}
        P = {n: _bf16(OW.gen_bf16(n, s, seed)) for n, s in shapes.items()}
        self.E = P["language_model.model.embed_tokens.weight"]
        self.norm = P["language_model.model.norm.weight"]
        self.layers = []
        for i in range(self.L):
            p = f"language_model.model.layers.{i}."
            self.layers.append({
                "ln1": P[p + "input_layernorm.weight"], "ln2": P[p + "post_attention_layernorm.weight"],
                "qkv": torch.cat([P[p + "self_attn.q_proj.weight"], P[p + "self_attn.k_proj.weight"],
                                  P[p + "self_attn.v_proj.weight"]], 0).contiguous(),
                "o": P[p + "self_attn.o_proj.weight"],
                "gu": torch.cat([P[p + "mlp.gate_proj.weight"], P[p + "mlp.up_proj.weight"]], 0).contiguous(),
                "down": P[p + "mlp.down_proj.weight"]})
        self.K = torch.zeros(self.L, max_kv, self.nkv, self.hd, dtype=torch.bfloat16)
        self.V = torch.zeros_like(self.K)
        self.kv_len = 0
        base = t.get("rope_theta", 10000.0)
        self.inv_freq = 1.0 / (base ** (torch.arange(0, self.hd, 2, dtype=torch.int64).float() / self.hd))
        self.normalizer = torch.tensor(self.H ** 0.5, dtype=torch.bfloat16)

    def fill_cache(self, n: int, seed: int = 0) -> None:
        """n cached tokens of random K/V (the decode step's cost depends on the cache length only)."""
        g = torch.Generator().manual_seed(seed)
        self.K[:, :n] = torch.randn(self.L, n, self.nkv, self.hd, generator=g).to(torch.bfloat16)
        self.V[:, :n] = torch.randn(self.L, n, self.nkv, self.hd, generator=g).to(torch.bfloat16)
        self.kv_len = n

    def _rms(self, x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
        xf = x.float()
        y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + self.eps)
        return (y * (1.0 + w.float())).to(x.dtype)

    def _rope(self, x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
        h = x.shape[-1] // 2
        rot = torch.cat((-x[..., h:], x[..., :h]), -1)
        return x * cos + rot * sin

    @torch.no_grad()
    def step(self, token: int, position: int) -> torch.Tensor:
        """One decode step: token at rotary `position`, K/V appended at kv_len; returns fp32 logits (V,)."""
        h = self.E[token].unsqueeze(0) * self.normalizer                         # (1, H) bf16
        pos = min(max(position, 0), self.max_pos - 1)
        ang = self.inv_freq * float(pos)
        emb = torch.cat((ang, ang), -1)
        cos, sin = emb.cos().to(torch.bfloat16), emb.sin().to(torch.bfloat16)
        T = self.kv_len + 1
        nq = self.nh * self.hd
        for i, ly in enumerate(self.layers):
            x = self._rms(h, ly["ln1"])
            qkv = F.linear(x, ly["qkv"])[0]
            q = self._rope(qkv[:nq].view(self.nh, self.hd), cos, sin)
            k = self._rope(qkv[nq:nq + self.nkv * self.hd].view(self.nkv, self.hd), cos, sin)
            self.K[i, self.kv_len] = k
            self.V[i, self.kv_len] = qkv[nq + self.nkv * self.hd:].view(self.nkv, self.hd)
            Kc, Vc = self.K[i, :T, 0], self.V[i, :T, 0]                           # MQA: the one KV head
            s = (q @ Kc.t()) / math.sqrt(self.hd)                                # (nh, T) bf16
            p = torch.softmax(s, -1, dtype=torch.float32).to(torch.bfloat16)
            o = (p @ Vc).reshape(1, nq)
            h = h + F.linear(o, ly["o"])
            x = self._rms(h, ly["ln2"])
            gu = F.linear(x, ly["gu"])
            a = F.gelu(gu[:, :self.I], approximate="tanh") * gu[:, self.I:]
            h = h + F.linear(a, ly["down"])
        self.kv_len = T
        return F.linear(self._rms(h, self.norm), self.E).float()[0]
