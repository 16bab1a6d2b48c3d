"""Shared test helpers (no reference code: restatements of its preprocessing arithmetic)."""
import numpy as np


def pixels_from_u8(u8):
    """processing_paligemma.py:20-29,47-49 on the resized uint8 image: x/255 (float64 -> float32),
    (x - 0.5)/0.5 in float32, HWC -> CHW."""
    px = (u8 * (1 / 255.0)).astype(np.float32)
    return ((px - np.float32(0.5)) / np.float32(0.5)).transpose(2, 0, 1)


# ---- the ablation harness's two monkey-patches (ablation_study_fixed.py:99-142, 144-166), restated.
# load_model_simple (:335-342) installs them on the model instance / every layer's rotary module;
# tests install these on the drop-in model to drive it the way the paper's benchmark does.

def ablation_merge(self, image_features, inputs_embeds, input_ids, attention_mask, kv_cache=None):
    """Merge semantics of ablation_study_fixed.py:99-142: the reference merge with no q_len == 1
    assertion, kv_len = cached + q_len for a filled cache, the single position
    cumsum(mask)[:, -1:] for EVERY query row of a filled cache, and positions 0..L-1 (clamped to
    max_position_embeddings - 1) otherwise."""
    import torch
    B, L = input_ids.shape
    D = image_features.shape[-1]
    dt, dev = inputs_embeds.dtype, inputs_embeds.device
    img_id, pad_id = self.config.image_token_index, self.pad_token_id
    out = torch.zeros(B, L, D, dtype=dt, device=dev)
    is_img = input_ids == img_id
    is_pad = input_ids == pad_id
    is_txt = ~is_img & ~is_pad
    out = torch.where(is_txt[..., None].expand(-1, -1, D), inputs_embeds, out)
    out = out.masked_scatter(is_img[..., None].expand(-1, -1, D), image_features / (self.config.hidden_size ** 0.5))
    out = torch.where(is_pad[..., None].expand(-1, -1, D), torch.zeros_like(out), out)
    filled = kv_cache is not None and kv_cache.num_items() > 0
    kv_len = kv_cache.num_items() + L if filled else L
    mask = torch.zeros((B, L, kv_len), dtype=dt, device=dev).unsqueeze(1)
    if filled:
        pos = attention_mask.cumsum(-1)[:, -1:]
        if pos.dim() == 1:
            pos = pos.unsqueeze(0)
    else:
        n = attention_mask.shape[1]
        pos = torch.arange(n, device=dev, dtype=torch.long).unsqueeze(0).expand(B, -1)
        pos = pos.masked_fill(attention_mask == 0, 0)
        pos = torch.clamp(pos, 0, self.config.text_config.max_position_embeddings - 1)
    return out, mask, pos


def ablation_rotary(self, x, position_ids, seq_len=None):
    """Rotary semantics of ablation_study_fixed.py:144-166: positions clamped to
    max_position_embeddings - 1, fp32 angles, cos/sin cast to x's dtype."""
    import torch
    if position_ids.dim() == 1:
        position_ids = position_ids.unsqueeze(0)
    position_ids = torch.clamp(position_ids, 0, self.max_position_embeddings - 1)
    inv = self.inv_freq.to(x.device)[None, :, None].float().expand(position_ids.shape[0], -1, 1)
    ang = (inv @ position_ids[:, None, :].float()).transpose(1, 2)
    ang = torch.cat((ang, ang), dim=-1)
    return ang.cos().to(x.dtype), ang.sin().to(x.dtype)


def install_ablation_patches(model):
    import types
    model._merge_input_ids_with_image_features = types.MethodType(ablation_merge, model)
    for layer in model.language_model.model.layers:
        layer.self_attn.rotary_emb.forward = types.MethodType(ablation_rotary, layer.self_attn.rotary_emb)


def remove_ablation_patches(model):
    model.__dict__.pop("_merge_input_ids_with_image_features", None)
    for layer in model.language_model.model.layers:
        layer.self_attn.rotary_emb.__dict__.pop("forward", None)
