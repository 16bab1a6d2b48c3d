"""The drop-in reference API (modeling_gemma / modeling_siglip / utils) on the GPU, driven
exactly as the reference's harnesses drive it, against the golden vectors of the reference."""
import os
import types

import numpy as np
import pytest
import torch

from oracle import paligemma_np as O
from oracle import weights as W

pytestmark = pytest.mark.gpu
SEED = 1234


@pytest.fixture(scope="module")
def gold(golden_dir):
    return np.load(os.path.join(golden_dir, "small_bf16.npz"))


def _model(cfg):
    import modeling_gemma as MG
    import utils as U
    pcfg = MG.PaliGemmaConfig(**{k: v for k, v in cfg.items() if k not in ("bos_token_id", "eos_token_id")})
    m = U.build_model(pcfg, device="cuda")
    sd = {n: torch.from_numpy(W.gen_bf16(n, s, SEED).view(np.int16)).view(torch.bfloat16)
          for n, s in W.param_shapes(cfg).items()}
    m.load_state_dict(sd, strict=False)
    m.tie_weights()
    return m.eval()


@pytest.fixture(scope="module")
def model():
    return _model(W.small_config())


def _inputs(gold):
    px = torch.from_numpy(O.from_bits(gold["pixels_bits"])).cuda()
    ids = torch.from_numpy(gold["ids"]).cuda()
    return ids, px


def _margin_ok(toks, ref, ref_logits):
    s = np.sort(ref_logits, -1)
    margin = s[:, -1] - s[:, -2]
    diff = np.nonzero(np.asarray(toks) != np.asarray(ref))[0]
    return len(diff) == 0 or margin[diff[0]] < 0.25


@torch.no_grad()
def test_inference_loop(model, gold):
    """inference.py:test_inference's loop (inference.py:55-78): pixel_values re-passed every step,
    attention_mask grown by one float column per step, argmax of logits[:, -1, :]."""
    import modeling_gemma as MG
    ids, px = _inputs(gold)
    mask = torch.ones_like(ids)
    kv = MG.KVCache()
    toks = []
    for _ in range(16):
        out = model(input_ids=ids, pixel_values=px, attention_mask=mask, kv_cache=kv)
        kv = out["kv_cache"]
        nxt = torch.argmax(out["logits"][:, -1, :], dim=-1, keepdim=True)
        assert nxt.size() == (1, 1)
        nxt = nxt.squeeze(0)
        toks.append(int(nxt.item()))
        ids = nxt.unsqueeze(-1)
        mask = torch.cat([mask, torch.ones((1, 1), device=ids.device)], dim=-1)
    ref = gold["greedy_tokens"].tolist()
    assert _margin_ok(toks, ref, O.from_bits(gold["greedy_logits"])), (toks, ref)
    # the cache the API exposes is the reference's KVCache view: 18 layers x (B, 1, T, 256)
    assert kv.num_items() == gold["ids"].shape[1] + 15
    assert tuple(kv.key_cache[0].shape) == (1, 1, kv.num_items(), 256)


@torch.no_grad()
def test_prefill_logits_and_vision_api(model, gold):
    import modeling_gemma as MG
    ids, px = _inputs(gold)
    out = model(input_ids=ids, pixel_values=px, attention_mask=torch.ones_like(ids), kv_cache=MG.KVCache())
    lg = out["logits"]
    assert lg.dtype == torch.float32 and tuple(lg.shape) == (1, ids.shape[1], W.small_config()["vocab_size"])
    ref = gold["prefill_logits_last"]
    got = lg[:, -1].cpu().numpy()
    assert np.linalg.norm(got - ref) / np.linalg.norm(ref) < 3e-2
    feats = model.vision_tower(px)
    assert feats.shape == (1, 256, 1152)
    vref = O.from_bits(gold["tap_vision_out"])
    f = feats.float().cpu().numpy()[:, ::8]
    assert np.linalg.norm(f - vref) / np.linalg.norm(vref) < 1e-2


@torch.no_grad()
def test_no_kv_cache_mode(model, gold):
    """kv_cache=None (the ablation's no-KV mode) is a plain prefill over the given ids."""
    import modeling_gemma as MG
    ids, px = _inputs(gold)
    a = model(input_ids=ids, pixel_values=px, attention_mask=torch.ones_like(ids), kv_cache=None)["logits"]
    b = model(input_ids=ids, pixel_values=px, attention_mask=torch.ones_like(ids), kv_cache=MG.KVCache())["logits"]
    assert torch.equal(a, b)


@torch.no_grad()
def test_patched_merge_is_honoured(model, gold):
    """ablation_study_fixed.py:335-337 monkey-patches the merge; its positions must be used."""
    import modeling_gemma as MG
    ids, px = _inputs(gold)
    calls = []
    orig = MG.PaliGemmaForConditionalGeneration._merge_input_ids_with_image_features

    def patched(self, image_features, inputs_embeds, input_ids, attention_mask, kv_cache=None):
        calls.append(1)
        return orig(self, image_features, inputs_embeds, input_ids, attention_mask, kv_cache)

    model._merge_input_ids_with_image_features = types.MethodType(patched, model)
    try:
        a = model(input_ids=ids, pixel_values=px, attention_mask=torch.ones_like(ids), kv_cache=MG.KVCache())["logits"]
    finally:
        del model._merge_input_ids_with_image_features
    b = model(input_ids=ids, pixel_values=px, attention_mask=torch.ones_like(ids), kv_cache=MG.KVCache())["logits"]
    assert calls
    # same merge semantics through torch ops vs on the device: identical embeddings
    assert (a[:, -1] - b[:, -1]).abs().max().item() < 1e-3


def test_error_conventions(model, gold):
    import modeling_gemma as MG
    ids, px = _inputs(gold)
    with pytest.raises(ValueError):
        model(input_ids=ids, pixel_values=px, attention_mask=None)
    with pytest.raises(AssertionError):
        m = torch.ones_like(ids)
        m[0, -1] = 0
        model(input_ids=ids, pixel_values=px, attention_mask=m)
    with pytest.raises(ValueError):
        model(input_ids=None, pixel_values=px, attention_mask=torch.ones_like(ids))
    kv = MG.KVCache()
    model(input_ids=ids, pixel_values=px, attention_mask=torch.ones_like(ids), kv_cache=kv)
    with pytest.raises(AssertionError):  # decode with q_len != 1 (modeling_gemma.py:509)
        model(input_ids=ids[:, :2], attention_mask=torch.ones((1, ids.shape[1] + 2), device="cuda"), kv_cache=kv)


def test_submodule_forwards(model):
    """Every Gemma submodule runs on its own (tests/test_gpu_modules.py checks their values against the
    oracle) -- here on the bound model, whose parameters are slab views read in place (gate|up adjacent).
    GemmaAttention asserts a mask as the reference does (modeling_gemma.py:268)."""
    layer = model.language_model.model.layers[0]
    x = torch.randn(1, 3, 2048, device="cuda").bfloat16()
    mask = torch.zeros(1, 1, 3, 3, dtype=torch.bfloat16, device="cuda")
    pos = torch.arange(3, device="cuda")[None]
    y = layer(x, attention_mask=mask, position_ids=pos)
    assert y.shape == (1, 3, 2048) and y.dtype == torch.bfloat16 and bool(torch.isfinite(y.float()).all())
    with pytest.raises(AssertionError):
        layer.self_attn(hidden_states=x, attention_mask=None, position_ids=pos)
    y = layer.mlp(x)
    assert y.shape == (1, 3, 2048) and y.dtype == torch.bfloat16 and bool(torch.isfinite(y.float()).all())
    z = layer.input_layernorm(x)
    assert z.shape == x.shape and bool(torch.isfinite(z.float()).all())
