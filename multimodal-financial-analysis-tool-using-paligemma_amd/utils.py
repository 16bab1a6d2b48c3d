"""Drop-in for the reference's utils.py: load_hf_model(model_path, device) -> (model, tokenizer).

Replaces the reference's full random init + accelerate dispatch (/root/reference/utils.py:6-46)
with: config.json -> PaliGemmaConfig, the module tree built on the meta device (no 3B random
init), safetensors read straight into bf16 device parameters, non-persistent buffers
recomputed, weights tied (utils.py:44).  There is no "load without weights" fallback: a missing
tensor raises (the reference's strict=False / ImportError paths silently kept random weights).
"""
from __future__ import annotations

import glob
import json
import os

import torch

from modeling_gemma import PaliGemmaConfig, PaliGemmaForConditionalGeneration


def _reset_buffers(model):
    for layer in model.language_model.model.layers:
        re = layer.self_attn.rotary_emb
        re.inv_freq = (1.0 / (re.base ** (torch.arange(0, re.dim, 2, dtype=torch.int64).float() / re.dim))).to(
            re.inv_freq.device)
    emb = model.vision_tower.vision_model.embeddings
    emb.position_ids = torch.arange(emb.num_positions, device=emb.position_ids.device).expand((1, -1))


def build_model(config: PaliGemmaConfig, device="cuda", dtype=torch.bfloat16):
    """PaliGemmaForConditionalGeneration(config) with uninitialised device parameters."""
    with torch.device("meta"):
        model = PaliGemmaForConditionalGeneration(config)
    model = model.to_empty(device=device).to(dtype)
    _reset_buffers(model)
    return model


def load_safetensors(model, model_path: str, strict: bool = True):
    from safetensors import safe_open
    files = sorted(glob.glob(os.path.join(model_path, "*.safetensors")))
    if not files:
        raise FileNotFoundError(f"no *.safetensors under {model_path}")
    params = dict(model.named_parameters(remove_duplicate=False))
    seen = set()
    with torch.no_grad():
        for f in files:
            with safe_open(f, framework="pt", device="cpu") as sf:
                for k in sf.keys():
                    if k not in params:
                        continue
                    params[k].copy_(sf.get_tensor(k).to(params[k].dtype))
                    seen.add(k)
    missing = [k for k in params if k not in seen and not k.endswith("lm_head.weight")]
    if strict and missing:
        raise KeyError(f"{len(missing)} weights missing from {model_path}: {missing[:4]}")
    return model


def load_weights_native(model, model_path: str, strict: bool = True):
    """The checkpoint read by libpgmi straight into the model's engine slab (pgmi_load_safetensors:
    mmap, shape checks, bf16 conversion on the device); the module's bf16 parameters are views of
    that slab, so they see the loaded values."""
    eng = model._pgmi_engine()
    eng.load_safetensors(model_path, strict=strict)
    return model


def load_hf_model(model_path, device="cuda", native: bool = True):
    from transformers import AutoTokenizer
    tokenizer = AutoTokenizer.from_pretrained(model_path, padding_side="right")
    model = load_model(model_path, device=device, native=native)
    return model, tokenizer


def load_model(model_path, device="cuda", native: bool = True):
    """config.json + *.safetensors -> PaliGemmaForConditionalGeneration (utils.py:6-46 without the
    tokenizer).  native: libpgmi's reader fills the engine slab; else safe_open per tensor."""
    with open(f"{model_path}/config.json", "r") as f:
        config = PaliGemmaConfig(**json.load(f))
    model = build_model(config, device=device)
    if native and torch.device(device).type == "cuda":
        model.tie_weights()  # the engine binds the tied tree (lm_head = embed_tokens, utils.py:44)
        load_weights_native(model, model_path)
    else:
        load_safetensors(model, model_path)
        model.tie_weights()
    return model
