"""Synthetic-weight policy for benchmarks (random-init weights of the PaliGemma-3B
architecture; no checkpoint is available offline).

Same recipe as the test oracle (oracle/wgen.c + oracle/weights.py GAINS) so the benchmark
runs the exact weights the parity fixtures were made with; tests/test_cpu_host.py checks the
two policies agree name by name.  The values are generated on the device by
pgmi_fill_synthetic.
"""
from __future__ import annotations

import math

GAINS = {"embed": 0.02, "pos_embed": 0.1, "proj": 2.0, "qk": 3.0, "o_down": 8.0}


def _f32(x: float) -> float:
    import struct
    return struct.unpack("f", struct.pack("f", x))[0]


def init_policy(name: str, shape: tuple) -> "tuple[float, float]":
    """(scale, offset): w = bf16(offset + U[-1, 1) * scale)."""
    g = GAINS
    if name.endswith("embed_tokens.weight"):
        return g["embed"], 0.0
    if name.endswith("position_embedding.weight"):
        return g["pos_embed"], 0.0
    if "layernorm" in name or "layer_norm" in name or name.endswith("model.norm.weight"):
        if name.startswith("language_model"):
            return 0.1, 0.0
        if name.endswith(".weight"):
            return 0.1, 1.0
        return 0.05, 0.0
    if name.endswith(".bias"):
        return 0.02, 0.0
    fan_in = math.prod(shape[1:])
    gain = g["proj"]
    if name.startswith("language_model"):
        if name.endswith("o_proj.weight") or name.endswith("down_proj.weight"):
            gain = g["o_down"]
        elif name.endswith("q_proj.weight") or name.endswith("k_proj.weight"):
            gain = g["qk"]
    return _f32(gain / math.sqrt(fan_in)), 0.0


def paligemma_3b_config(image_size: int = 224) -> dict:
    """HF google/paligemma-3b-pt-{224,448} config.json (as PaliGemmaConfig consumes it)."""
    return {
        "vision_config": {"hidden_size": 1152, "intermediate_size": 4304, "num_hidden_layers": 27,
                          "num_attention_heads": 16, "num_channels": 3, "image_size": image_size,
                          "patch_size": 14, "layer_norm_eps": 1e-6, "projection_dim": 2048},
        "text_config": {"vocab_size": 257216, "hidden_size": 2048, "intermediate_size": 16384,
                        "num_hidden_layers": 18, "num_attention_heads": 8, "num_key_value_heads": 1,
                        "head_dim": 256, "max_position_embeddings": 8192, "rms_norm_eps": 1e-6,
                        "rope_theta": 10000.0},
        "image_token_index": 257152, "vocab_size": 257216, "projection_dim": 2048, "hidden_size": 2048,
        "pad_token_id": 0, "bos_token_id": 2, "eos_token_id": 1,
    }


def prompt_ids(image_token_index: int, n_image_tokens: int, vocab: int, n_text: int = 30, seed: int = 7):
    """<image>*N + <bos> + n_text synthetic ids + '\\n' (processing_paligemma.py:10-11)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    hi = min(image_token_index, vocab) - 1
    txt = rng.integers(3, hi, size=n_text)
    newline = 108 if hi > 108 else 5
    return np.array([[image_token_index] * n_image_tokens + [2] + txt.tolist() + [newline]], dtype=np.int64)
