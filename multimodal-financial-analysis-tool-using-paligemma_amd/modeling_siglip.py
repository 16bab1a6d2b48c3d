"""Drop-in for the reference's modeling_siglip.py (SigLIP vision tower), MI355X-native.

The module tree, constructor signatures and state-dict names are the reference's
(/root/reference/modeling_siglip.py:7-255), so checkpoints load unchanged.  The forward of
SiglipVisionModel runs the whole tower in libpgmi (pgmi_vision: im2col+MFMA patch embedding,
27 x [LayerNorm, fused QKV GEMM, MHA, out-proj+residual, LayerNorm, fc1+GELU, fc2+residual],
post-LayerNorm; csrc/engine.hip).  The per-layer submodules (embeddings, attention, MLP, encoder
layer, encoder) are callable on their own too, on libpgmi's single-op entries (pgmi/modules.py), so
forward hooks on them fire when they are called; the fused tower does not call them.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn as nn

from pgmi import binding as _binding
from pgmi import modules as _modules


class SiglipVisionConfig:
    """modeling_siglip.py:7-34 (same arguments and attributes)."""

    def __init__(self, hidden_size=768, intermediate_size=3072, num_hidden_layers=12, num_attention_heads=12,
                 num_channels=3, image_size=224, patch_size=16, layer_norm_eps=1e-6, attention_dropout=0.0,
                 num_image_tokens: int = None, **kwargs):
        super().__init__()
        self.hidden_size = hidden_size
        self.intermediate_size = intermediate_size
        self.num_hidden_layers = num_hidden_layers
        self.num_attention_heads = num_attention_heads
        self.num_channels = num_channels
        self.patch_size = patch_size
        self.image_size = image_size
        self.attention_dropout = attention_dropout
        self.layer_norm_eps = layer_norm_eps
        self.num_image_tokens = num_image_tokens


class _LayerNorm(nn.LayerNorm):
    """nn.LayerNorm (same parameters and state-dict names) whose own forward runs pgmi_op_layernorm."""

    def forward(self, x):
        return _modules.layer_norm(x, self.weight, self.bias, self.eps)


class SiglipVisionEmbeddings(nn.Module):
    """modeling_siglip.py:36-79: Conv2d(k=s=patch) + learned position embedding."""

    def __init__(self, config: SiglipVisionConfig):
        super().__init__()
        self.config = config
        self.embed_dim = config.hidden_size
        self.image_size = config.image_size
        self.patch_size = config.patch_size
        self.patch_embedding = nn.Conv2d(config.num_channels, self.embed_dim, kernel_size=self.patch_size,
                                         stride=self.patch_size, padding="valid")
        self.num_patches = (self.image_size // self.patch_size) ** 2
        self.num_positions = self.num_patches
        self.position_embedding = nn.Embedding(self.num_positions, self.embed_dim)
        self.register_buffer("position_ids", torch.arange(self.num_positions).expand((1, -1)), persistent=False)

    forward = _modules.siglip_embeddings_forward


class SiglipAttention(nn.Module):
    """modeling_siglip.py:81-147 (16 heads x 72 in PaliGemma-3B)."""

    def __init__(self, config):
        super().__init__()
        self.config = config
        self.embed_dim = config.hidden_size
        self.num_heads = config.num_attention_heads
        self.head_dim = self.embed_dim // self.num_heads
        self.scale = self.head_dim ** -0.5
        self.dropout = config.attention_dropout
        self.k_proj = nn.Linear(self.embed_dim, self.embed_dim)
        self.v_proj = nn.Linear(self.embed_dim, self.embed_dim)
        self.q_proj = nn.Linear(self.embed_dim, self.embed_dim)
        self.out_proj = nn.Linear(self.embed_dim, self.embed_dim)

    forward = _modules.siglip_attention_forward


class SiglipMLP(nn.Module):
    """modeling_siglip.py:149-167: fc1 -> gelu(tanh) -> fc2."""

    def __init__(self, config):
        super().__init__()
        self.config = config
        self.fc1 = nn.Linear(config.hidden_size, config.intermediate_size)
        self.fc2 = nn.Linear(config.intermediate_size, config.hidden_size)

    forward = _modules.siglip_mlp_forward


class SiglipEncoderLayer(nn.Module):
    """modeling_siglip.py:169-204: pre-LN attention and MLP blocks with residuals."""

    def __init__(self, config: SiglipVisionConfig):
        super().__init__()
        self.embed_dim = config.hidden_size
        self.self_attn = SiglipAttention(config)
        self.layer_norm1 = _LayerNorm(self.embed_dim, eps=config.layer_norm_eps)
        self.mlp = SiglipMLP(config)
        self.layer_norm2 = _LayerNorm(self.embed_dim, eps=config.layer_norm_eps)

    forward = _modules.siglip_encoder_layer_forward


class SiglipEncoder(nn.Module):
    """modeling_siglip.py:206-223."""

    def __init__(self, config: SiglipVisionConfig):
        super().__init__()
        self.config = config
        self.layers = nn.ModuleList([SiglipEncoderLayer(config) for _ in range(config.num_hidden_layers)])

    forward = _modules.siglip_encoder_forward


class SiglipVisionTransformer(nn.Module):
    """modeling_siglip.py:225-244."""

    def __init__(self, config: SiglipVisionConfig):
        super().__init__()
        self.config = config
        self.embeddings = SiglipVisionEmbeddings(config)
        self.encoder = SiglipEncoder(config)
        self.post_layernorm = _LayerNorm(config.hidden_size, eps=config.layer_norm_eps)

    def forward(self, pixel_values: torch.Tensor) -> torch.Tensor:
        return _binding.vision_forward(self, pixel_values, prefix="vision_tower.vision_model.")


class SiglipVisionModel(nn.Module):
    """modeling_siglip.py:246-255: (B, C, H, W) -> (B, num_patches, hidden) in bf16."""

    def __init__(self, config=SiglipVisionConfig):
        super().__init__()
        self.config = config
        self.vision_model = SiglipVisionTransformer(config)

    def forward(self, pixel_values) -> Tuple:
        return self.vision_model(pixel_values=pixel_values)
