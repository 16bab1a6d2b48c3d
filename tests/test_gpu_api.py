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


def _greedy_logits(model, ids, px, B, steps=3):
    """The reference loop (inference.py:55-78) at batch B (rows = the same image and prompt): the last-row
    logits of the prefill and of `steps` greedy KV-cached steps, (B, steps + 1, V)."""
    import modeling_gemma as MG
    idsB, pxB = ids.expand(B, -1).contiguous(), px.expand(B, -1, -1, -1).contiguous()
    kv, mask = MG.KVCache(), torch.ones_like(idsB)
    out = model(input_ids=idsB, pixel_values=pxB, attention_mask=mask, kv_cache=kv)
    res = [out["logits"][:, -1].float().clone()]
    for _ in range(steps):
        nxt = torch.argmax(res[-1], -1, keepdim=True)
        mask = torch.cat([mask, torch.ones((B, 1), device=mask.device, dtype=mask.dtype)], -1)
        res.append(model(input_ids=nxt, attention_mask=mask, kv_cache=kv)["logits"][:, -1].float().clone())
    return torch.stack(res, 1)


@torch.no_grad()
def test_inplace_update_of_unsampled_weight_rebinds(gold):
    """An in-place update of a weight the binding's parameter sample does not hold (a text layer's q_proj)
    between two generations: the next prefill sees it (pgmi/binding.py full_check), drops the pending greedy
    lookahead and rebuilds the derived tensors -- the batched decode's fragment-major images among them -- so
    B = 1 and B = 8 logits equal those of a freshly bound model with the same weights (ablation_study_fixed.py
    :304-332 updates a bound model in place with load_state_dict)."""
    cfg = W.small_config()
    m = _model(cfg)
    ids, px = _inputs(gold)
    _greedy_logits(m, ids, px, 1)
    _greedy_logits(m, ids, px, 8)  # binds, builds the batched images, leaves a lookahead pending
    sampled = {id(p) for p in m.__dict__["_pgmi_bound"].sample}
    name, p = next((n, p) for n, p in m.named_parameters()
                   if n.startswith("language_model.") and n.endswith("self_attn.q_proj.weight") and id(p) not in sampled)
    p.mul_(0.5)
    a1, a8 = _greedy_logits(m, ids, px, 1), _greedy_logits(m, ids, px, 8)
    fresh = _model(cfg)
    fresh.load_state_dict(m.state_dict())
    fresh.tie_weights()
    b1, b8 = _greedy_logits(fresh, ids, px, 1), _greedy_logits(fresh, ids, px, 8)
    assert torch.equal(a1, b1), (name, (a1 - b1).abs().max().item())
    assert torch.equal(a8, b8), (name, (a8 - b8).abs().max().item())
    del fresh


@torch.no_grad()
def test_dropped_model_releases_engine_without_gc(gold):
    """A model dropped after lookahead decode steps frees its engine (context, weight slab, workspaces) at
    once: the greedy lookahead refers to its engine weakly, so no reference cycle waits for the collector."""
    import gc
    import weakref
    m = _model(W.small_config())
    ids, px = _inputs(gold)
    lg = _greedy_logits(m, ids, px, 1)
    eng = weakref.ref(m.__dict__["_pgmi_bound"].engine)
    assert eng() is not None and eng().__dict__.get("_lookahead") is not None
    gc.collect()
    gc.disable()
    try:
        del m, lg
        assert eng() is None
    finally:
        gc.enable()
