"""oracle/weights.py -- TEST INFRASTRUCTURE ONLY (checker side, never the product).

Synthetic-weight policy + configs for parity testing.  PaliGemma-3B weights are
not available offline, so the oracle, the golden fixtures (made by running the
reference modules in the survey container) and the HIP path all run on the same
deterministic synthetic weights produced by ``wgen.c``.

State-dict names/shapes follow the reference module tree
(/root/reference/modeling_gemma.py:440-456,
/root/reference/modeling_siglip.py:36-255).
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "libwgen.so")

# HF google/paligemma-3b-pt-224 config.json, as consumed by PaliGemmaConfig
# (/root/reference/modeling_gemma.py:74-105).
FULL_224 = {
    "vision_config": {
        "hidden_size": 1152, "intermediate_size": 4304, "num_hidden_layers": 27,
        "num_attention_heads": 16, "num_channels": 3, "image_size": 224,
        "patch_size": 14, "layer_norm_eps": 1e-6, "projection_dim": 2048,
    },
    "text_config": {
        "vocab_size": 257216, "hidden_size": 2048, "intermediate_size": 16384,
        "num_hidden_layers": 18, "num_attention_heads": 8, "num_key_value_heads": 1,
        "head_dim": 256, "max_position_embeddings": 8192, "rms_norm_eps": 1e-6,
        "rope_theta": 10000.0,
    },
    "image_token_index": 257152, "vocab_size": 257216, "projection_dim": 2048,
    "hidden_size": 2048, "pad_token_id": 0, "bos_token_id": 2, "eos_token_id": 1,
}


def full_config(image_size: int = 224) -> dict:
    import copy
    c = copy.deepcopy(FULL_224)
    c["vision_config"]["image_size"] = image_size
    return c


def small_config(vision_layers: int = 2, text_layers: int = 2, vocab: int = 16384,
                 image_size: int = 224) -> dict:
    """Full PaliGemma widths, fewer layers and a reduced vocabulary: every kernel
    shape of the 3B model is exercised at a size the numpy oracle finishes in
    seconds."""
    c = full_config(image_size)
    c["vision_config"]["num_hidden_layers"] = vision_layers
    c["text_config"]["num_hidden_layers"] = text_layers
    c["text_config"]["vocab_size"] = vocab
    c["vocab_size"] = vocab
    c["image_token_index"] = vocab - 64
    return c


def num_image_tokens(cfg: dict) -> int:
    v = cfg["vision_config"]
    return (v["image_size"] // v["patch_size"]) ** 2


def param_shapes(cfg: dict) -> "dict[str, tuple]":
    """Every persistent parameter of PaliGemmaForConditionalGeneration(cfg), keyed by
    the reference state-dict name (lm_head is tied to embed_tokens,
    modeling_gemma.py:396-397, and so is not listed)."""
    v, t = cfg["vision_config"], cfg["text_config"]
    D, I, C, P = v["hidden_size"], v["intermediate_size"], v.get("num_channels", 3), v["patch_size"]
    N = (v["image_size"] // P) ** 2
    out = {}
    vp = "vision_tower.vision_model."
    out[vp + "embeddings.patch_embedding.weight"] = (D, C, P, P)
    out[vp + "embeddings.patch_embedding.bias"] = (D,)
    out[vp + "embeddings.position_embedding.weight"] = (N, D)
    for i in range(v["num_hidden_layers"]):
        lp = f"{vp}encoder.layers.{i}."
        for nm in ("q_proj", "k_proj", "v_proj", "out_proj"):
            out[lp + f"self_attn.{nm}.weight"] = (D, D)
            out[lp + f"self_attn.{nm}.bias"] = (D,)
        out[lp + "layer_norm1.weight"] = (D,)
        out[lp + "layer_norm1.bias"] = (D,)
        out[lp + "mlp.fc1.weight"] = (I, D)
        out[lp + "mlp.fc1.bias"] = (I,)
        out[lp + "mlp.fc2.weight"] = (D, I)
        out[lp + "mlp.fc2.bias"] = (D,)
        out[lp + "layer_norm2.weight"] = (D,)
        out[lp + "layer_norm2.bias"] = (D,)
    out[vp + "post_layernorm.weight"] = (D,)
    out[vp + "post_layernorm.bias"] = (D,)
    PD = cfg.get("projection_dim", 2048)
    out["multi_modal_projector.linear.weight"] = (PD, D)
    out["multi_modal_projector.linear.bias"] = (PD,)
    H, TI, V = t["hidden_size"], t["intermediate_size"], t["vocab_size"]
    NH, NKV, HD = t["num_attention_heads"], t["num_key_value_heads"], t.get("head_dim", 256)
    out["language_model.model.embed_tokens.weight"] = (V, H)
    for i in range(t["num_hidden_layers"]):
        lp = f"language_model.model.layers.{i}."
        out[lp + "self_attn.q_proj.weight"] = (NH * HD, H)
        out[lp + "self_attn.k_proj.weight"] = (NKV * HD, H)
        out[lp + "self_attn.v_proj.weight"] = (NKV * HD, H)
        out[lp + "self_attn.o_proj.weight"] = (H, NH * HD)
        out[lp + "mlp.gate_proj.weight"] = (TI, H)
        out[lp + "mlp.up_proj.weight"] = (TI, H)
        out[lp + "mlp.down_proj.weight"] = (H, TI)
        out[lp + "input_layernorm.weight"] = (H,)
        out[lp + "post_attention_layernorm.weight"] = (H,)
    out["language_model.model.norm.weight"] = (H,)
    return out


# Gains of the synthetic init (tuned so that the 18-layer bf16 model stays close to its
# fp32 counterpart -- i.e. parity is measurable -- while greedy decoding stays varied).
GAINS = {"embed": 0.02, "pos_embed": 0.1, "proj": 2.0, "qk": 3.0, "o_down": 8.0}


def init_policy(name: str, shape: tuple) -> "tuple[float, float]":
    """(scale, offset) of the synthetic init: w = bf16(offset + U[-1,1) * scale).

    gain/sqrt(fan_in) for projections; norms get small
    random deviations so the (1 + w) RMSNorm path (modeling_gemma.py:119) and the
    LayerNorm affine are exercised."""
    g = GAINS
    if name.endswith("embed_tokens.weight"):
        return g["embed"], 0.0
    if name.endswith("position_embedding.weight"):
        return g["pos_embed"], 0.0
    if "layernorm" in name or "layer_norm" in name or name.endswith("model.norm.weight"):
        if name.startswith("language_model"):
            return 0.1, 0.0            # GemmaRMSNorm multiplies by (1 + w)
        if name.endswith(".weight"):
            return 0.1, 1.0            # LayerNorm gamma around 1
        return 0.05, 0.0               # LayerNorm beta
    if name.endswith(".bias"):
        return 0.02, 0.0
    fan_in = int(np.prod(shape[1:]))
    gain = g["proj"]
    if name.startswith("language_model"):
        if name.endswith("o_proj.weight") or name.endswith("down_proj.weight"):
            gain = g["o_down"]   # residual stream dominated by layer outputs, not the tied embedding
        elif name.endswith("q_proj.weight") or name.endswith("k_proj.weight"):
            gain = g["qk"]       # position-dependent attention (else greedy repeats one token)
    return float(np.float32(gain / math.sqrt(fan_in))), 0.0


def build_lib(force: bool = False) -> str:
    src = os.path.join(_HERE, "wgen.c")
    if force or not os.path.exists(_LIB) or os.path.getmtime(_LIB) < os.path.getmtime(src):
        subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-shared", "-fPIC", src, "-o", _LIB])
    return _LIB


_lib = None


def _load():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(build_lib())
        _lib.wgen_fill_bf16.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_float, ctypes.c_float,
                                        ctypes.c_void_p, ctypes.c_int64]
        _lib.wgen_fill_f32.argtypes = _lib.wgen_fill_bf16.argtypes
        _lib.wgen_name_hash.argtypes = [ctypes.c_char_p]
        _lib.wgen_name_hash.restype = ctypes.c_uint64
    return _lib


def gen_bf16(name: str, shape: tuple, seed: int) -> np.ndarray:
    """bf16 bit patterns (uint16) of one synthetic tensor."""
    scale, offset = init_policy(name, shape)
    out = np.empty(int(np.prod(shape)), dtype=np.uint16)
    _load().wgen_fill_bf16(name.encode(), seed, scale, offset, out.ctypes.data, out.size)
    return out.reshape(shape)


def gen_f32(name: str, shape: tuple, seed: int) -> np.ndarray:
    """The same tensor widened to float32 (exact bf16 values)."""
    scale, offset = init_policy(name, shape)
    out = np.empty(int(np.prod(shape)), dtype=np.float32)
    _load().wgen_fill_f32(name.encode(), seed, scale, offset, out.ctypes.data, out.size)
    return out.reshape(shape)


def synthetic_state_dict_f32(cfg: dict, seed: int) -> "dict[str, np.ndarray]":
    return {n: gen_f32(n, s, seed) for n, s in param_shapes(cfg).items()}


def name_hash(name: str) -> int:
    return int(_load().wgen_name_hash(name.encode()))
