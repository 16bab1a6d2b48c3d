"""Drop-in for the reference's modeling_gemma.py (Gemma decoder, KV cache, PaliGemma), MI355X-native.

Same classes, constructor signatures, attributes and state-dict names as
/root/reference/modeling_gemma.py, so the reference's inference.py / utils.py /
ablation_study_fixed.py drive it unchanged.  The forwards of the three boundary modules run in
libpgmi (include/pgmi.h):

  PaliGemmaForConditionalGeneration.forward  (:539-617)  vision tower + projector + merge +
                                                         Gemma prefill, or one KV-cached decode step
  GemmaForCausalLM.forward                   (:399-427)  Gemma over given embeddings
  KVCache                                    (:10-36)    a preallocated bf16 slab
                                                         [layer][K|V][batch][tokens][256] with the
                                                         reference's key_cache/value_cache/num_items()

Kept reference semantics: non-causal prefill (zero mask, :506-511); decode position =
attention_mask.cumsum(-1)[:, -1] (:524-528, so the first decode position is L+1); image features
divided by sqrt(hidden) (:481) and the bf16 normalizer 45.25 (:367-368); fp32 logits (:418);
the error behaviour of :557-564 and :509.  A monkey-patched _merge_input_ids_with_image_features
(ablation_study_fixed.py:335-337) is honoured: its embeddings/positions are fed to libpgmi.
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

import torch
from torch import nn
from torch.nn import CrossEntropyLoss

from modeling_siglip import SiglipVisionConfig, SiglipVisionModel
from pgmi import binding as _binding
from pgmi import modules as _modules
from pgmi.lazy_logits import LazyLogits
from pgmi.lookahead import lookahead_for


class KVCache:
    """modeling_gemma.py:10-36.  When filled by the MI355X path the cache is one bf16 slab
    (layers, 2, B, capacity, kv_heads*head_dim) in HBM written in place (no torch.cat per
    step); key_cache[i] / value_cache[i] are (B, kv_heads, T, head_dim) views of it, as in the
    reference.  update() keeps the reference's behaviour for callers that drive it directly."""

    def __init__(self) -> None:
        self._lists_k: List[torch.Tensor] = []
        self._lists_v: List[torch.Tensor] = []
        self._slab: Optional[torch.Tensor] = None
        self._len = 0

    # -- reference API --------------------------------------------------------------------
    @property
    def key_cache(self) -> List[torch.Tensor]:
        if self._slab is None:
            return self._lists_k
        return [self._slab[i, 0, :, : self._len].unflatten(-1, (-1, 256)).transpose(1, 2)
                for i in range(self._slab.shape[0])]

    @property
    def value_cache(self) -> List[torch.Tensor]:
        if self._slab is None:
            return self._lists_v
        return [self._slab[i, 1, :, : self._len].unflatten(-1, (-1, 256)).transpose(1, 2)
                for i in range(self._slab.shape[0])]

    def num_items(self) -> int:
        if self._slab is not None:
            return self._len
        if len(self._lists_k) == 0:
            return 0
        return self._lists_k[0].shape[-2]

    def update(self, key_states: torch.Tensor, value_states: torch.Tensor, layer_idx: int
               ) -> Tuple[torch.Tensor, torch.Tensor]:
        if self._slab is not None:
            raise RuntimeError("this KVCache is owned by the MI355X path; update() is only for torch-driven caches")
        if len(self._lists_k) <= layer_idx:
            self._lists_k.append(key_states)
            self._lists_v.append(value_states)
        else:
            self._lists_k[layer_idx] = torch.cat([self._lists_k[layer_idx], key_states], dim=-2)
            self._lists_v[layer_idx] = torch.cat([self._lists_v[layer_idx], value_states], dim=-2)
        return self._lists_k[layer_idx], self._lists_v[layer_idx]

    # -- MI355X path ----------------------------------------------------------------------
    def _ensure(self, engine, batch: int, need: int) -> torch.Tensor:
        if self._lists_k:
            raise RuntimeError("KVCache was filled through update(); start generation with a fresh KVCache()")
        if self._slab is None:
            cap = max(engine.max_kv, need)
            self._slab = engine.new_kv(batch, cap)
        if self._slab.shape[2] != batch:
            raise ValueError(f"KVCache holds batch {self._slab.shape[2]}, got {batch}")
        if need > self._slab.shape[3]:
            raise ValueError(f"KVCache capacity {self._slab.shape[3]} exceeded ({need} tokens)")
        return self._slab


class GemmaConfig:
    """modeling_gemma.py:39-71."""

    def __init__(self, vocab_size, hidden_size, intermediate_size, num_hidden_layers, num_attention_heads,
                 num_key_value_heads, head_dim=256, max_position_embeddings=8192, rms_norm_eps=1e-6,
                 rope_theta=10000.0, attention_bias=False, attention_dropout=0.0, pad_token_id=None, **kwargs):
        super().__init__()
        self.vocab_size = vocab_size
        self.max_position_embeddings = max_position_embeddings
        self.hidden_size = hidden_size
        self.intermediate_size = intermediate_size
        self.num_hidden_layers = num_hidden_layers
        self.num_attention_heads = num_attention_heads
        self.head_dim = head_dim
        self.num_key_value_heads = num_key_value_heads
        self.rms_norm_eps = rms_norm_eps
        self.rope_theta = rope_theta
        self.attention_bias = attention_bias
        self.attention_dropout = attention_dropout
        self.pad_token_id = pad_token_id


class PaliGemmaConfig:
    """modeling_gemma.py:74-105."""

    def __init__(self, vision_config=None, text_config=None, ignore_index=-100, image_token_index=256000,
                 vocab_size=257152, projection_dim=2048, hidden_size=2048, pad_token_id=None, **kwargs):
        super().__init__()
        self.ignore_index = ignore_index
        self.image_token_index = image_token_index
        self.vocab_size = vocab_size
        self.projection_dim = projection_dim
        self.hidden_size = hidden_size
        self.vision_config = vision_config
        self.is_encoder_decoder = False
        self.pad_token_id = pad_token_id
        self.vision_config = SiglipVisionConfig(**vision_config)
        self.text_config = text_config
        self.text_config = GemmaConfig(**text_config, pad_token_id=pad_token_id)
        self.vocab_size = self.text_config.vocab_size
        self.text_config.num_image_tokens = (self.vision_config.image_size // self.vision_config.patch_size) ** 2
        self.vision_config.projection_dim = projection_dim


class GemmaRMSNorm(nn.Module):
    """modeling_gemma.py:107-120 (weight applied as (1 + w))."""

    def __init__(self, dim: int, eps: float = 1e-6):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.zeros(dim))

    forward = _modules.gemma_rmsnorm_forward  # callable on its own (pgmi_op_rmsnorm)


class GemmaMLP(nn.Module):
    """modeling_gemma.py:122-134: down(gelu_tanh(gate(x)) * up(x))."""

    def __init__(self, config):
        super().__init__()
        self.config = config
        self.hidden_size = config.hidden_size
        self.intermediate_size = config.intermediate_size
        self.gate_proj = nn.Linear(self.hidden_size, self.intermediate_size, bias=False)
        self.up_proj = nn.Linear(self.hidden_size, self.intermediate_size, bias=False)
        self.down_proj = nn.Linear(self.intermediate_size, self.hidden_size, bias=False)

    forward = _modules.gemma_mlp_forward  # callable on its own (pgmi_op_gemm: GeGLU, then down)


def repeat_kv(hidden_states: torch.Tensor, n_rep: int) -> torch.Tensor:
    """modeling_gemma.py:136-141 (utility; the MI355X kernels never materialise the repeat)."""
    batch, num_key_value_heads, slen, head_dim = hidden_states.shape
    if n_rep == 1:
        return hidden_states
    hidden_states = hidden_states[:, :, None, :, :].expand(batch, num_key_value_heads, n_rep, slen, head_dim)
    return hidden_states.reshape(batch, num_key_value_heads * n_rep, slen, head_dim)


class GemmaRotaryEmbedding(nn.Module):
    """modeling_gemma.py:143-185.  The engine builds its RoPE table from this module's
    inv_freq buffer with the same fp32 arithmetic as forward(); forward() itself is kept as a
    utility (and remains monkey-patchable, ablation_study_fixed.py:339-341)."""

    def __init__(self, dim, max_position_embeddings=2048, base=10000, device=None):
        super().__init__()
        self.dim = dim
        self.max_position_embeddings = max_position_embeddings
        self.base = base
        inv_freq = 1.0 / (self.base ** (torch.arange(0, self.dim, 2, dtype=torch.int64).float() / self.dim))
        self.register_buffer("inv_freq", tensor=inv_freq, persistent=False)

    @torch.no_grad()
    def forward(self, x, position_ids, seq_len=None):
        if position_ids.dim() == 1:
            position_ids = position_ids.unsqueeze(0)
        position_ids = torch.clamp(position_ids, 0, self.max_position_embeddings - 1)
        inv = self.inv_freq.to(x.device)[None, :, None].float().expand(position_ids.shape[0], -1, 1)
        pos = position_ids[:, None, :].float()
        freqs = (inv @ pos).transpose(1, 2)
        emb = torch.cat((freqs, freqs), dim=-1)
        return emb.cos().to(dtype=x.dtype), emb.sin().to(dtype=x.dtype)


def rotate_half(x):
    """modeling_gemma.py:187-191."""
    x1 = x[..., : x.shape[-1] // 2]
    x2 = x[..., x.shape[-1] // 2:]
    return torch.cat((-x2, x1), dim=-1)


def apply_rotary_pos_emb(q, k, cos, sin, unsqueeze_dim=1):
    """modeling_gemma.py:193-199."""
    cos = cos.unsqueeze(unsqueeze_dim)
    sin = sin.unsqueeze(unsqueeze_dim)
    return (q * cos) + (rotate_half(q) * sin), (k * cos) + (rotate_half(k) * sin)


class GemmaAttention(nn.Module):
    """modeling_gemma.py:201-293 (MQA: 8 query heads share 1 KV head in PaliGemma-3B)."""

    def __init__(self, config: GemmaConfig, layer_idx: Optional[int] = None):
        super().__init__()
        self.config = config
        self.layer_idx = layer_idx
        self.attention_dropout = config.attention_dropout
        self.hidden_size = config.hidden_size
        self.num_heads = config.num_attention_heads
        self.head_dim = config.head_dim
        self.num_key_value_heads = config.num_key_value_heads
        self.num_key_value_groups = self.num_heads // self.num_key_value_heads
        self.max_position_embeddings = config.max_position_embeddings
        self.rope_theta = config.rope_theta
        self.is_causal = True
        assert self.hidden_size % self.num_heads == 0
        self.q_proj = nn.Linear(self.hidden_size, self.num_heads * self.head_dim, bias=config.attention_bias)
        self.k_proj = nn.Linear(self.hidden_size, self.num_key_value_heads * self.head_dim, bias=config.attention_bias)
        self.v_proj = nn.Linear(self.hidden_size, self.num_key_value_heads * self.head_dim, bias=config.attention_bias)
        self.o_proj = nn.Linear(self.num_heads * self.head_dim, self.hidden_size, bias=config.attention_bias)
        self.rotary_emb = GemmaRotaryEmbedding(self.head_dim, max_position_embeddings=self.max_position_embeddings,
                                               base=self.rope_theta)

    # callable on its own (pgmi/modules.py: q/k/v GEMMs, the module's rotary_emb + pgmi_op_rope,
    # kv_cache.update, pgmi_op_attention_ex with the mask, o_proj); returns (out, attn_weights)
    forward = _modules.gemma_attention_forward


class GemmaDecoderLayer(nn.Module):
    """modeling_gemma.py:295-338."""

    def __init__(self, config: GemmaConfig, layer_idx: int):
        super().__init__()
        self.hidden_size = config.hidden_size
        self.self_attn = GemmaAttention(config=config, layer_idx=layer_idx)
        self.mlp = GemmaMLP(config)
        self.input_layernorm = GemmaRMSNorm(config.hidden_size, eps=config.rms_norm_eps)
        self.post_attention_layernorm = GemmaRMSNorm(config.hidden_size, eps=config.rms_norm_eps)

    forward = _modules.gemma_decoder_layer_forward  # calls its submodules as modules (hooks fire)


class GemmaModel(nn.Module):
    """modeling_gemma.py:340-382."""

    def __init__(self, config: GemmaConfig):
        super().__init__()
        self.config = config
        self.padding_idx = config.pad_token_id
        self.vocab_size = config.vocab_size
        self.embed_tokens = nn.Embedding(config.vocab_size, config.hidden_size, self.padding_idx)
        self.layers = nn.ModuleList([GemmaDecoderLayer(config, i) for i in range(config.num_hidden_layers)])
        self.norm = GemmaRMSNorm(config.hidden_size, eps=config.rms_norm_eps)

    def get_input_embeddings(self):
        return self.embed_tokens

    # callable on its own, layer by layer through the module forwards (GemmaForCausalLM and
    # PaliGemmaForConditionalGeneration run the fused engine instead)
    forward = _modules.gemma_model_forward


def _positions_2d(position_ids, B, L) -> torch.Tensor:
    """Rotary positions as a host int64 (B, L) tensor; accepts the reference's (1, L), (B, L),
    (B, 1) (decode, float from the mask cumsum) and 1-D forms (modeling_gemma.py:160-161)."""
    pos = torch.as_tensor(position_ids).detach().to("cpu")
    if pos.dim() == 1:
        pos = pos.unsqueeze(0)
    pos = pos.to(torch.float64).round().to(torch.int64)
    return pos.expand(B, L).contiguous()


def _dev_mask_ok(mask, n_keys: int) -> bool:
    """A merge's mask the device-side decode step can take: none, or one additive row over the n_keys
    attended keys (shape (1, 1, 1, n_keys) as the reference's merge builds it, modeling_gemma.py:512-518)."""
    if mask is None:
        return True
    return torch.is_tensor(mask) and mask.numel() == n_keys and mask.shape[-1] == n_keys and mask.is_floating_point()


def _merged_positions(position_ids, mask, B, L) -> torch.Tensor:
    """Host int64 (B, L) positions of a (patched) merge's output, read together with a check of
    its attention mask in ONE device->host copy.  libpgmi attends every cached key with no
    additive mask -- the reference's zero mask (modeling_gemma.py:506-511,
    ablation_study_fixed.py:122-128) -- so a merge returning any non-zero mask entry is refused
    rather than silently ignored."""
    pid = torch.as_tensor(position_ids)
    dev = pid.device if pid.device.type != "cpu" else (mask.device if torch.is_tensor(mask) else pid.device)
    parts = [pid.detach().to(dev, torch.float64).reshape(-1)]
    if torch.is_tensor(mask):
        parts.append((mask != 0).any().to(dev, torch.float64).reshape(1))
    host = torch.cat(parts).cpu()
    if torch.is_tensor(mask) and host[-1].item() != 0:
        raise NotImplementedError("libpgmi attends every cached key with no additive mask (the reference's zero "
                                  "mask); the merge returned a non-zero attention mask")
    n = parts[0].numel()
    return _positions_2d(host[:n].reshape(pid.shape), B, L)


class GemmaForCausalLM(nn.Module):
    """modeling_gemma.py:384-427."""

    def __init__(self, config):
        super().__init__()
        self.config = config
        self.model = GemmaModel(config)
        self.vocab_size = config.vocab_size
        self.lm_head = nn.Linear(config.hidden_size, config.vocab_size, bias=False)

    def get_input_embeddings(self):
        return self.model.embed_tokens

    def tie_weights(self):
        self.lm_head.weight = self.model.embed_tokens.weight

    def pgmi_rebind(self):
        """Forget the engine binding (after replacing Parameter objects; pgmi/binding.py)."""
        _binding.unbind(self)

    def _pgmi_engine(self, full_check: bool = False):
        owner = _binding.owner_of(self)
        if owner is not None:
            return owner._pgmi_engine(full_check)
        _check_tied(self)
        return _binding.bind(self, lambda: _binding.text_cfg(self.config), "language_model.",
                             inv_freq=self.model.layers[0].self_attn.rotary_emb.inv_freq if self.model.layers else None,
                             full_check=full_check)

    def forward(self, attention_mask: Optional[torch.Tensor] = None, position_ids: Optional[torch.LongTensor] = None,
                inputs_embeds: Optional[torch.FloatTensor] = None, kv_cache: Optional[KVCache] = None, **kwargs) -> dict:
        """Gemma over merged embeddings (x bf16(sqrt(hidden)) inside), KV appended at
        kv_cache.num_items().  attention_mask is the additive mask every layer adds to its scores
        (modeling_gemma.py:268-269, passed down at :370-377, :409-414) and, as there, must be given.
        The all-zero mask the merge builds (:506-518) runs the fused engine (attention over the whole
        cache); any other mask runs the per-layer module forwards, whose attention adds it
        (pgmi_op_attention_ex), and the tied lm_head GEMM -- bf16 logits cast to fp32, as :416-418."""
        if inputs_embeds is None:
            raise ValueError("inputs_embeds must be provided")
        assert attention_mask is not None                                  # modeling_gemma.py:268
        B, L = inputs_embeds.shape[:2]
        if position_ids is None:
            position_ids = torch.arange(L).unsqueeze(0)
        if not torch.is_tensor(attention_mask) or bool((attention_mask != 0).any()):
            return self._forward_masked(attention_mask, position_ids, inputs_embeds, kv_cache)
        eng = self._pgmi_engine(full_check=kv_cache is None or kv_cache.num_items() == 0)
        pos = _positions_2d(position_ids, B, L)
        logits = _run_lm(eng, kv_cache, B, L, pos, embeds=inputs_embeds, logits_rows=kwargs.get("logits_rows", 0))
        out = {"logits": logits}
        if kv_cache is not None:
            out["kv_cache"] = kv_cache
        return out

    def _forward_masked(self, attention_mask, position_ids, inputs_embeds, kv_cache):
        """A non-zero additive mask (causal, padding): GemmaModel's module forwards (each layer's
        GemmaAttention adds the mask to its scores, :269) and the lm_head, :409-418."""
        if kv_cache is not None and kv_cache._slab is not None:
            raise NotImplementedError("a KVCache filled by the fused path attends every cached key; a non-zero "
                                      "attention mask needs a fresh KVCache() (filled through update())")
        _check_tied(self)
        dev = self.lm_head.weight.device
        mask = torch.as_tensor(attention_mask, device=dev)
        pos = torch.as_tensor(position_ids, device=dev)
        h = self.model(attention_mask=mask, position_ids=pos, inputs_embeds=inputs_embeds.to(dev), kv_cache=kv_cache)
        logits = _modules.linear(h, self.lm_head.weight).float()
        out = {"logits": logits}
        if kv_cache is not None:
            out["kv_cache"] = kv_cache
        return out


def _check_tied(lm: "GemmaForCausalLM"):
    w, e = lm.lm_head.weight, lm.model.embed_tokens.weight
    if w.data_ptr() == e.data_ptr():
        return
    if w.shape != e.shape or not torch.equal(w.detach(), e.detach()):
        raise NotImplementedError("libpgmi computes logits with the tied embedding (modeling_gemma.py:396-397); "
                                  "call tie_weights() first, as utils.load_hf_model does")


class _PaddingCheck:
    """`assert torch.all(attention_mask == 1)` (modeling_gemma.py:558) without a host sync AHEAD of the
    GPU work: for a device mask the comparison runs on a side stream (behind an event of the caller's
    stream, so it sees the mask the caller's kernels produced) and its result is copied to pinned host
    memory behind an event; wait() reads it -- raising the reference's AssertionError -- after this
    call's kernels are enqueued and before any Python-side state (the KVCache length) changes.
    launch() may come after the step's own launch (the KV-cached decode step): the check's host cost
    then overlaps the step instead of delaying it; nothing is committed before wait()."""

    _flags = {}
    _streams = {}
    _events = {}  # per device: (the caller-stream event, the side-stream event), reused call after call

    def __init__(self, mask: torch.Tensor):
        self.mask, self.ev, self.bad, self.flag = mask, None, False, None
        if mask.device.type == "cuda":
            evs = _PaddingCheck._events.get(mask.device)
            if evs is None:
                evs = _PaddingCheck._events[mask.device] = (torch.cuda.Event(), torch.cuda.Event())
            self.ready, self.done = evs
            self.ready.record()
        else:
            self.bad = bool((mask != 1).any())

    def launch(self):
        mask = self.mask
        if mask.device.type != "cuda" or self.ev is not None:
            return
        dev = mask.device
        flag = _PaddingCheck._flags.get(dev)
        if flag is None:
            flag = _PaddingCheck._flags[dev] = torch.zeros((), dtype=torch.bool).pin_memory()
            _PaddingCheck._streams[dev] = torch.cuda.Stream(device=dev)
        side = _PaddingCheck._streams[dev]
        side.wait_event(self.ready)
        with torch.cuda.stream(side):
            mask.record_stream(side)
            flag.copy_((mask != 1).any(), non_blocking=True)
            self.ev = self.done
            self.ev.record(side)
        self.flag = flag

    def wait(self):
        self.launch()
        if self.ev is not None:
            self.ev.synchronize()
            self.bad, self.ev = bool(self.flag), None
        self.mask = None
        assert not self.bad, "The input cannot be padded"


def _run_lm(eng, kv_cache, B, L, pos, ids=None, image_feats=None, embeds=None, logits_rows=0, before_commit=None):
    """GemmaModel + lm_head with the cache semantics of KVCache.update (append at num_items());
    before_commit() runs after the forward is enqueued and before the cache length advances."""
    if kv_cache is None:
        kv = eng.scratch_kv(B, L)
        start = 0
    else:
        start = kv_cache.num_items()
        kv = kv_cache._ensure(eng, B, start + L)
    logits = eng.lm_forward(kv, start, pos, ids=ids, image_feats=image_feats, embeds=embeds, logits_rows=logits_rows)
    if before_commit is not None:
        before_commit()
    if kv_cache is not None:
        kv_cache._len = start + L
    return logits


class PaliGemmaMultiModalProjector(nn.Module):
    """modeling_gemma.py:429-438."""

    def __init__(self, config: PaliGemmaConfig):
        super().__init__()
        self.linear = nn.Linear(config.vision_config.hidden_size, config.vision_config.projection_dim, bias=True)

    def forward(self, image_features):
        owner = _binding.owner_of(self)
        if owner is None:
            raise NotImplementedError("the projector runs on the PaliGemma model's engine")
        return owner._pgmi_engine().project(image_features)


class PaliGemmaForConditionalGeneration(nn.Module):
    """modeling_gemma.py:440-617."""

    # knobs of the MI355X path (not in the reference): decode steps replay a captured hipGraph;
    # prefill logits: "lazy" (default: the (B, L, V) result computes its last row at once and the
    # other rows only when something reads them -- pgmi/lazy_logits.py), "all" (every row eagerly,
    # the reference's behaviour) or "last" (a (B, 1, V) tensor)
    pgmi_use_graph: bool = True
    pgmi_prefill_logits: str = "lazy"
    # KV-cached decode steps run the greedy continuation one step ahead of the caller (pgmi/lookahead.py):
    # bit-identical results, the host's per-token work overlaps the next step; off after two misses per cache
    pgmi_lookahead: bool = True

    def __init__(self, config: PaliGemmaConfig):
        super().__init__()
        self.config = config
        self.vision_tower = SiglipVisionModel(config.vision_config)
        self.multi_modal_projector = PaliGemmaMultiModalProjector(config)
        self.vocab_size = config.vocab_size
        self.language_model = GemmaForCausalLM(config.text_config)
        self.pad_token_id = self.config.pad_token_id if self.config.pad_token_id is not None else -1
        for child in (self.vision_tower.vision_model, self.multi_modal_projector, self.language_model):
            _binding.set_owner(child, self)

    def tie_weights(self):
        return self.language_model.tie_weights()

    def get_output_embeddings(self):
        return self.language_model.lm_head

    def prepare_inputs_for_generation(self, input_ids=None, **kwargs):
        return {"input_ids": input_ids, **kwargs}

    def pgmi_rebind(self):
        """Forget the engine binding (after replacing Parameter objects): the next forward copies
        the current parameters into a new weight slab (pgmi/binding.py)."""
        _binding.unbind(self)

    def _pgmi_engine(self, full_check: bool = False):
        _check_tied(self.language_model)
        layers = self.language_model.model.layers
        return _binding.bind(self, lambda: _pgmi_cfg(self.config), "",
                             inv_freq=layers[0].self_attn.rotary_emb.inv_freq if len(layers) else None,
                             full_check=full_check)

    def _merge_input_ids_with_image_features(self, image_features: torch.Tensor, inputs_embeds: torch.Tensor,
                                             input_ids: torch.Tensor, attention_mask: torch.Tensor,
                                             kv_cache: Optional[KVCache] = None):
        """modeling_gemma.py:468-537, same semantics (torch ops).  The default forward performs
        this merge on the device inside pgmi_lm_forward; this method is only called when it
        has been monkey-patched (or inputs_embeds were supplied)."""
        _, _, embed_dim = image_features.shape
        batch_size, sequence_length = input_ids.shape
        dtype, device = inputs_embeds.dtype, inputs_embeds.device
        scaled_image_features = image_features / (self.config.hidden_size ** 0.5)
        final_embedding = torch.zeros(batch_size, sequence_length, embed_dim, dtype=dtype, device=device)
        text_mask = (input_ids != self.config.image_token_index) & (input_ids != self.pad_token_id)
        image_mask = input_ids == self.config.image_token_index
        pad_mask = input_ids == self.pad_token_id
        final_embedding = torch.where(text_mask.unsqueeze(-1).expand(-1, -1, embed_dim), inputs_embeds, final_embedding)
        final_embedding = final_embedding.masked_scatter(image_mask.unsqueeze(-1).expand(-1, -1, embed_dim),
                                                         scaled_image_features.to(dtype))
        final_embedding = torch.where(pad_mask.unsqueeze(-1).expand(-1, -1, embed_dim),
                                      torch.zeros_like(final_embedding), final_embedding)
        q_len = inputs_embeds.shape[1]
        if kv_cache is None or kv_cache.num_items() == 0:
            causal_mask = torch.full((batch_size, q_len, q_len), fill_value=0, dtype=dtype, device=device)
        else:
            assert q_len == 1
            kv_len = kv_cache.num_items() + q_len
            causal_mask = torch.full((batch_size, q_len, kv_len), fill_value=0, dtype=dtype, device=device)
        causal_mask = causal_mask.unsqueeze(1)
        if kv_cache is not None and kv_cache.num_items() > 0:
            position_ids = attention_mask.cumsum(-1)[:, -1]
            if position_ids.dim() == 1:
                position_ids = position_ids.unsqueeze(0)
        else:
            seq_len = attention_mask.shape[1]
            position_ids = torch.arange(seq_len, device=device).unsqueeze(0).expand(attention_mask.shape[0], -1)
            position_ids = position_ids.masked_fill((attention_mask == 0), 0)
        return final_embedding, causal_mask, position_ids

    def _merge_is_patched(self) -> bool:
        return "_merge_input_ids_with_image_features" in self.__dict__ or \
            type(self)._merge_input_ids_with_image_features is not \
            PaliGemmaForConditionalGeneration._merge_input_ids_with_image_features

    def forward(self, input_ids: Optional[torch.LongTensor] = None, pixel_values: Optional[torch.FloatTensor] = None,
                attention_mask: Optional[torch.Tensor] = None, inputs_embeds: Optional[torch.FloatTensor] = None,
                kv_cache: Optional[KVCache] = None, labels: Optional[torch.LongTensor] = None,
                return_dict: bool = True, **kwargs) -> Tuple:
        # validation as the reference (modeling_gemma.py:557-564); the padding check is read after this
        # call's GPU work is enqueued (_PaddingCheck), still before anything is committed or returned
        if attention_mask is None:
            raise ValueError("attention_mask must be provided")
        chk = _PaddingCheck(attention_mask)
        decode_step = (kv_cache is not None and inputs_embeds is None and input_ids is not None and
                       kv_cache.num_items() > 0 and not self._merge_is_patched())
        if not decode_step:
            chk.launch()
        if inputs_embeds is None and input_ids is None:
            chk.wait()
            raise ValueError("You must provide either input_ids or inputs_embeds")
        cache_len = kv_cache.num_items() if kv_cache is not None else 0
        # a prefill also checks every weight the parameter sample cannot vouch for (pgmi/binding.py)
        eng = self._pgmi_engine(full_check=cache_len == 0)
        dev = eng.device
        src = input_ids if input_ids is not None else inputs_embeds
        B, L = src.shape[0], src.shape[1]
        mode = self.pgmi_prefill_logits
        if mode not in ("lazy", "all", "last"):
            raise ValueError(f"pgmi_prefill_logits must be 'lazy', 'all' or 'last', not {mode!r}")
        rows = 0 if mode == "all" else 1

        if self._merge_is_patched() or inputs_embeds is not None:
            # generic path: the (patched) merge decides embeddings / positions
            own_embeds = None
            if inputs_embeds is None:
                inputs_embeds = own_embeds = eng.embed(input_ids)
            if pixel_values is not None:
                img = eng.project(eng.vision(pixel_values))
            else:
                img = torch.zeros(B, 0, inputs_embeds.shape[-1], dtype=inputs_embeds.dtype, device=dev)
            merged, mask, position_ids = self._merge_input_ids_with_image_features(
                image_features=img, inputs_embeds=inputs_embeds.to(dev), input_ids=input_ids.to(dev),
                attention_mask=attention_mask, kv_cache=kv_cache)
            if (kv_cache is not None and cache_len > 0 and L == 1 and B == 1 and torch.is_tensor(position_ids)
                    and position_ids.numel() == 1 and _dev_mask_ok(mask, cache_len + 1)):
                # a one-sequence q_len == 1 step over a filled cache (the ablation harness's decode steps,
                # ablation_study_fixed.py:215-221,239-243): the graphed decode step reads the merge's
                # position and additive mask on the device -- no host read before the step is enqueued
                slab = kv_cache._ensure(eng, B, cache_len + 1)
                if self.pgmi_lookahead and self.pgmi_use_graph and own_embeds is not None:
                    # the greedy continuation one step ahead of the harness (pgmi/lookahead.py): used when the
                    # merge passed this token's embedding through at the predicted position with a zero mask
                    logits = lookahead_for(eng, B).step_embeds(kv_cache, slab, input_ids, own_embeds, merged[:, 0],
                                                               position_ids, mask if torch.is_tensor(mask) else None,
                                                               cache_len, True)
                else:
                    logits = eng.decode_embeds_dev(merged[:, 0], slab, cache_len, position_ids,
                                                   mask if torch.is_tensor(mask) else None, logits=eng.logits_buffer(B),
                                                   graph=self.pgmi_use_graph).clone().unsqueeze(1)
                chk.wait()
                kv_cache._len = cache_len + 1
                return self._pack(logits, labels, kv_cache, return_dict)
            chk.wait()
            pos = _merged_positions(position_ids, mask, B, L)
            if kv_cache is not None and cache_len > 0 and L == 1 and bool((pos == pos[0, 0]).all()):
                # a q_len == 1 step over a filled cache (the ablation harness's decode steps,
                # ablation_study_fixed.py:215-221,239-243): the graphed decode step over the merged row
                slab = kv_cache._ensure(eng, B, cache_len + 1)
                logits = eng.decode_embeds(merged[:, 0], slab, cache_len, int(pos[0, 0]), logits=eng.logits_buffer(B),
                                           graph=self.pgmi_use_graph).clone().unsqueeze(1)
                kv_cache._len = cache_len + 1
            else:
                logits = _run_lm(eng, kv_cache, B, L, pos, embeds=merged, logits_rows=rows)
                if mode == "lazy":
                    logits = LazyLogits(logits, eng.final_hidden(B * L), eng.lm_head, B, L)
        elif cache_len == 0 or kv_cache is None:
            # prefill (modeling_gemma.py:532-535: positions 0..L-1), merge on the device
            img = eng.project(eng.vision(pixel_values)) if pixel_values is not None else None
            pos = torch.arange(L).unsqueeze(0).expand(B, L)
            logits = _run_lm(eng, kv_cache, B, L, pos, ids=input_ids, image_feats=img, logits_rows=rows,
                             before_commit=chk.wait)
            if mode == "lazy":
                logits = LazyLogits(logits, eng.final_hidden(B * L), eng.lm_head, B, L)
        else:
            # KV-cached decode step; pixel_values of inference.py's loop would only produce image
            # features that the merge discards (the new token is not <image>), so they are skipped
            assert L == 1  # modeling_gemma.py:509
            position = int(attention_mask.shape[-1])  # cumsum of an all-ones mask, :526
            slab = kv_cache._ensure(eng, B, cache_len + 1)
            if self.pgmi_lookahead and self.pgmi_use_graph:
                # the greedy continuation runs one step ahead of the caller (pgmi/lookahead.py); the padding
                # check is enqueued behind the asked step and read before anything is committed
                logits = lookahead_for(eng, B).step(kv_cache, slab, input_ids, cache_len, position, True,
                                                    after_launch=chk.launch)
            else:
                logits = eng.decode(input_ids, slab, cache_len, position, logits=eng.logits_buffer(B),
                                    graph=self.pgmi_use_graph)
                chk.launch()  # behind the step's launch: its host cost overlaps the step
                logits = logits.clone().unsqueeze(1)
            chk.wait()
            kv_cache._len = cache_len + 1

        return self._pack(logits, labels, kv_cache, return_dict)

    def _pack(self, logits, labels, kv_cache, return_dict):
        """The loss and return conventions of modeling_gemma.py:598-617."""
        loss = None
        if labels is not None:
            shift_logits = logits[..., :-1, :].contiguous()
            shift_labels = labels[..., 1:].contiguous().to(logits.device)
            loss = CrossEntropyLoss(ignore_index=self.config.ignore_index)(
                shift_logits.view(-1, shift_logits.size(-1)), shift_labels.view(-1))
        if return_dict:
            out = {"logits": logits}
            if loss is not None:
                out["loss"] = loss
            if kv_cache is not None:
                out["kv_cache"] = kv_cache
            return out
        to_return = (logits,)
        if loss is not None:
            to_return = (loss,) + to_return
        return to_return


def _pgmi_cfg(config: PaliGemmaConfig) -> dict:
    v, t = config.vision_config, config.text_config
    return {
        "vision_config": {k: getattr(v, k) for k in ("hidden_size", "intermediate_size", "num_hidden_layers",
                                                     "num_attention_heads", "num_channels", "image_size",
                                                     "patch_size", "layer_norm_eps")},
        "text_config": {k: getattr(t, k) for k in ("vocab_size", "hidden_size", "intermediate_size",
                                                   "num_hidden_layers", "num_attention_heads", "num_key_value_heads",
                                                   "head_dim", "max_position_embeddings", "rms_norm_eps",
                                                   "rope_theta")},
        "image_token_index": config.image_token_index, "projection_dim": config.projection_dim,
        "hidden_size": config.hidden_size, "pad_token_id": config.pad_token_id,
    }
