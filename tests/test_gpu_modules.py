"""Per-layer module forwards of the drop-in model (pgmi/modules.py on libpgmi's single-op C-ABI entries)
against the oracle's restatement of the same reference modules, on synthetic PaliGemma-3B-width
weights (oracle/wgen.c).  Tolerances: rel-L2 < 1e-2 for GEMM / attention chains,
2 bf16 ulp for the norms; the module tree's forward hooks fire when a layer runs its submodules
(modeling_siglip.py:179-204: the reference calls self_attn / mlp / layer_norm* as modules)."""
import types

import numpy as np
import pytest
import torch

from oracle import paligemma_np as O
from oracle import weights as W
from tests_helpers import assert_within_floor

pytestmark = pytest.mark.gpu
SEED = 77


def rel_l2(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def np32(t):
    return t.detach().float().cpu().numpy()


@pytest.fixture(scope="module")
def setup():
    import modeling_siglip as MS
    cfg = W.small_config(vision_layers=1, text_layers=1, vocab=1024)
    P = W.synthetic_state_dict_f32(cfg, SEED)
    tower = MS.SiglipVisionModel(MS.SiglipVisionConfig(**cfg["vision_config"]))
    with torch.no_grad():
        for name, p in tower.named_parameters():
            p.data = torch.from_numpy(P["vision_tower." + name]).to("cuda", torch.bfloat16)
    return cfg, P, tower


def _x(rng, *shape):
    return O.bf16(rng.uniform(-1, 1, shape).astype(np.float32))


@torch.no_grad()
def test_siglip_embeddings(setup):
    cfg, P, tower = setup
    px = np.random.default_rng(1).uniform(-1, 1, (2, 3, 224, 224)).astype(np.float32)
    got = tower.vision_model.embeddings(torch.from_numpy(px).cuda())
    assert got.shape == (2, 256, 1152) and got.dtype == torch.bfloat16
    assert rel_l2(np32(got), O.siglip_embeddings(P, cfg, px)) < 5e-3


@torch.no_grad()
def test_siglip_attention_and_mlp(setup):
    cfg, P, tower = setup
    layer = tower.vision_model.encoder.layers[0]
    pre = "vision_tower.vision_model.encoder.layers.0."
    x = _x(np.random.default_rng(2), 2, 256, 1152)
    out, weights = layer.self_attn(hidden_states=torch.from_numpy(x).cuda().bfloat16())
    taps = {}
    assert rel_l2(np32(out), O.siglip_attention(P, pre + "self_attn.", x, 16, taps)) < 1e-2
    # the probabilities the reference returns as its second output (modeling_siglip.py:125,147)
    assert weights.shape == (2, 16, 256, 256) and weights.dtype == torch.bfloat16
    assert rel_l2(np32(weights), taps["probs"]) < 1e-2
    h = layer.mlp(torch.from_numpy(x).cuda().bfloat16())
    assert rel_l2(np32(h), O.siglip_mlp(P, pre + "mlp.", x)) < 1e-2


@torch.no_grad()
def test_siglip_layer_norm_ulp(setup):
    cfg, P, tower = setup
    ln = tower.vision_model.encoder.layers[0].layer_norm1
    x = _x(np.random.default_rng(3), 64, 1152) * 4
    got = np32(ln(torch.from_numpy(x).cuda().bfloat16()))
    ref = O.layer_norm(x, np.asarray(P["vision_tower.vision_model.encoder.layers.0.layer_norm1.weight"]),
                       np.asarray(P["vision_tower.vision_model.encoder.layers.0.layer_norm1.bias"]), 1e-6)
    ulp = np.abs(got.view(np.int32) - ref.astype(np.float32).view(np.int32)) >> 16
    assert (ulp <= 2).mean() > 0.999


@torch.no_grad()
def test_siglip_encoder_layer_hooks_and_tower(setup):
    cfg, P, tower = setup
    layer = tower.vision_model.encoder.layers[0]
    seen = []
    hs = [m.register_forward_hook(lambda m, i, o, n=n: seen.append(n))
          for n, m in (("ln1", layer.layer_norm1), ("attn", layer.self_attn), ("ln2", layer.layer_norm2),
                       ("mlp", layer.mlp), ("layer", layer))]
    try:
        x = _x(np.random.default_rng(4), 1, 256, 1152)
        got = layer(torch.from_numpy(x).cuda().bfloat16())
    finally:
        for h in hs:
            h.remove()
    assert seen == ["ln1", "attn", "ln2", "mlp", "layer"]
    assert rel_l2(np32(got), O.siglip_layer(P, cfg, 0, x)) < 1e-2
    # the module-by-module tower equals the fused one (pgmi_vision)
    px = torch.from_numpy(np.random.default_rng(5).uniform(-1, 1, (1, 3, 224, 224)).astype(np.float32)).cuda()
    vm = tower.vision_model
    staged = vm.post_layernorm(vm.encoder(inputs_embeds=vm.embeddings(px)))
    fused = tower(px)
    assert rel_l2(np32(staged), np32(fused)) < 1e-2


@torch.no_grad()
def test_gemma_rmsnorm_and_mlp(setup):
    import modeling_gemma as MG
    cfg, P, _ = setup
    pre = "language_model.model.layers.0."
    norm = MG.GemmaRMSNorm(2048, eps=1e-6).cuda()
    norm.weight.data = torch.from_numpy(P[pre + "input_layernorm.weight"]).to("cuda", torch.bfloat16)
    x = _x(np.random.default_rng(6), 3, 40, 2048) * 3
    got = np32(norm(torch.from_numpy(x).cuda().bfloat16()))
    ref = O.rms_norm(x, np.asarray(P[pre + "input_layernorm.weight"]), 1e-6)
    ulp = np.abs(got.view(np.int32) - ref.astype(np.float32).view(np.int32)) >> 16
    assert (ulp <= 2).mean() > 0.999
    mlp = MG.GemmaMLP(types.SimpleNamespace(hidden_size=2048, intermediate_size=16384))
    ref = O.gemma_mlp(P, 0, x)
    g, u, d = (torch.from_numpy(P[pre + f"mlp.{n}.weight"]).to("cuda", torch.bfloat16) for n in ("gate_proj", "up_proj",
                                                                                              "down_proj"))
    # separate gate / up tensors (stacked for the GEMM), then gate|up adjacent in one buffer (read in place)
    for adjacent in (False, True):
        if adjacent:
            gu = torch.cat([g, u], 0)
            mlp.gate_proj.weight.data, mlp.up_proj.weight.data = gu[:16384], gu[16384:]
        else:
            mlp.gate_proj.weight.data, mlp.up_proj.weight.data = g.clone(), u.clone()
        mlp.down_proj.weight.data = d
        got = mlp(torch.from_numpy(x).cuda().bfloat16())
        assert got.shape == (3, 40, 2048)
        assert rel_l2(np32(got), ref) < 1e-2, adjacent


# ---------------------------------------------------------------- Gemma layer modules
def _gemma_layer(P, cfg, i=0):
    import modeling_gemma as MG
    gc = MG.GemmaConfig(**cfg["text_config"])
    layer = MG.GemmaDecoderLayer(gc, i)
    with torch.no_grad():
        for name, p in layer.named_parameters():
            p.data = torch.from_numpy(P[f"language_model.model.layers.{i}." + name]).to("cuda", torch.bfloat16)
    return layer.cuda()


@torch.no_grad()
def test_gemma_attention_vs_oracle(setup):
    """GemmaAttention.forward (modeling_gemma.py:231-293) on its own: zero mask, causal mask, and a KV
    cache filled by a prefill then extended by one decode token (KVCache.update, :258-259); outputs
    and the returned probabilities against the oracle."""
    import modeling_gemma as MG
    cfg, P, _ = setup
    attn = _gemma_layer(P, cfg).self_attn
    invf = O.inv_freq(256)
    B, L = 2, 40
    x = _x(np.random.default_rng(8), B, L, 2048) * 2
    pos = np.broadcast_to(np.arange(L), (B, L))
    xt, post = torch.from_numpy(x).cuda().bfloat16(), torch.from_numpy(pos.copy()).cuda()
    # zero mask (the merge's, modeling_gemma.py:506-511)
    zero = torch.zeros(B, 1, L, L, dtype=torch.bfloat16, device="cuda")
    out, w = attn(hidden_states=xt, attention_mask=zero, position_ids=post)
    taps = {}
    ref = O.gemma_attention(P, cfg, 0, x, pos, None, invf, taps=taps)
    with O.fp32_truth():
        truth = O.gemma_attention(P, cfg, 0, x, pos, None, invf)
    assert_within_floor("gemma_attention/zero_mask", np32(out), ref, truth)
    assert w.shape == (B, 8, L, L) and rel_l2(np32(w), taps["probs"]) < 1e-2
    # a causal additive mask (bf16 large negative above the diagonal)
    cm = np.triu(np.full((L, L), -1e4, np.float32), 1)
    cmask = torch.from_numpy(cm).to("cuda", torch.bfloat16)[None, None].expand(B, 1, L, L)
    out, w = attn(hidden_states=xt, attention_mask=cmask, position_ids=post)
    taps = {}
    ref = O.gemma_attention(P, cfg, 0, x, pos, None, invf, mask=O.bf16(cm)[None, None], taps=taps)
    with O.fp32_truth():
        truth = O.gemma_attention(P, cfg, 0, x, pos, None, invf, mask=O.bf16(cm)[None, None])
    assert_within_floor("gemma_attention/causal_mask", np32(out), ref, truth)
    assert rel_l2(np32(w), taps["probs"]) < 1e-2
    assert float(w[0, 0, 0, 1:].float().abs().max()) == 0.0
    # KV cache: prefill L tokens, then one decode token at position L (the cache grows to L + 1)
    kv, okv = MG.KVCache(), O.KV()
    attn(hidden_states=xt, attention_mask=zero, position_ids=post, kv_cache=kv)
    O.gemma_attention(P, cfg, 0, x, pos, okv, invf)
    x1 = _x(np.random.default_rng(9), B, 1, 2048) * 2
    p1 = np.full((B, 1), L)
    out, w = attn(hidden_states=torch.from_numpy(x1).cuda().bfloat16(),
                  attention_mask=torch.zeros(B, 1, 1, L + 1, dtype=torch.bfloat16, device="cuda"),
                  position_ids=torch.from_numpy(p1).cuda(), kv_cache=kv)
    assert kv.num_items() == L + 1 and kv.key_cache[0].shape == (B, 1, L + 1, 256)
    ref = O.gemma_attention(P, cfg, 0, x1, p1, okv, invf)
    assert rel_l2(np32(out), ref) < 2e-2
    assert rel_l2(np32(kv.key_cache[0]), okv.k[0]) < 1e-2


@torch.no_grad()
def test_gemma_decoder_layer_hooks_and_model(setup):
    """GemmaDecoderLayer.forward (modeling_gemma.py:307-338) runs its submodules as modules (their
    forward hooks fire in the reference's order) and GemmaModel.forward (:357-382) -- normalizer,
    the layers, the final norm -- against the oracle."""
    import modeling_gemma as MG
    cfg, P, _ = setup
    gc = MG.GemmaConfig(**cfg["text_config"])
    model = MG.GemmaModel(gc)
    with torch.no_grad():
        for name, p in model.named_parameters():
            p.data = torch.from_numpy(P["language_model.model." + name]).to("cuda", torch.bfloat16)
    model = model.cuda()
    layer = model.layers[0]
    seen = []
    hs = [m.register_forward_hook(lambda m, i, o, n=n: seen.append(n))
          for n, m in (("ln1", layer.input_layernorm), ("attn", layer.self_attn), ("ln2", layer.post_attention_layernorm),
                       ("mlp", layer.mlp), ("layer", layer), ("norm", model.norm))]
    B, L = 1, 33
    emb = _x(np.random.default_rng(10), B, L, 2048) * 0.05
    pos = np.broadcast_to(np.arange(L), (B, L))
    try:
        got = model(attention_mask=torch.zeros(B, 1, L, L, dtype=torch.bfloat16, device="cuda"),
                    position_ids=torch.from_numpy(pos.copy()).cuda(), inputs_embeds=torch.from_numpy(emb).cuda().bfloat16())
    finally:
        for h in hs:
            h.remove()
    assert seen == ["ln1", "attn", "ln2", "mlp", "layer", "norm"]
    def oracle():
        taps = {}
        O.gemma_forward(P, cfg, emb, pos, O.KV(), taps=taps, all_logits=False)
        return O.rms_norm(taps["text_layer0"], P["language_model.model.norm.weight"], 1e-6)
    ref = oracle()
    with O.fp32_truth():
        truth = oracle()
    assert_within_floor("gemma_model/1_layer_final_norm", np32(got), ref, truth)


@torch.no_grad()
def test_gemma_model_modules_equal_fused(setup):
    """The module-by-module GemmaModel + tied lm_head equals GemmaForCausalLM's fused forward
    (pgmi_lm_forward) on the same parameters and embeddings."""
    import modeling_gemma as MG
    cfg, P, _ = setup
    gc = MG.GemmaConfig(**cfg["text_config"])
    lm = MG.GemmaForCausalLM(gc)
    with torch.no_grad():
        for name, p in lm.named_parameters():
            key = "language_model." + name
            if key in P:
                p.data = torch.from_numpy(P[key]).to("cuda", torch.bfloat16)
    lm.tie_weights()
    lm = lm.cuda()
    B, L = 1, 48
    emb = torch.from_numpy(_x(np.random.default_rng(11), B, L, 2048) * 0.05).cuda().bfloat16()
    pos = torch.arange(L, device="cuda")[None]
    staged = lm.model(attention_mask=torch.zeros(B, 1, L, L, dtype=torch.bfloat16, device="cuda"), position_ids=pos,
                      inputs_embeds=emb)
    staged_logits = (staged.float() @ lm.lm_head.weight.float().T).bfloat16().float()
    # the reference's 4-D zero mask (the merge's, modeling_gemma.py:506-518): the fused engine
    zero = torch.zeros(B, 1, L, L, dtype=torch.bfloat16, device="cuda")
    fused = lm(attention_mask=zero, position_ids=pos, inputs_embeds=emb)["logits"]
    assert rel_l2(np32(staged_logits), np32(fused)) < 1e-2
    # the reference asserts a mask is given (modeling_gemma.py:268)
    with pytest.raises(AssertionError):
        lm(attention_mask=None, position_ids=pos, inputs_embeds=emb)


@torch.no_grad()
def test_gemma_causal_lm_honours_additive_mask(setup):
    """GemmaForCausalLM.forward adds a non-zero attention mask in every layer, as the reference does
    (modeling_gemma.py:268-269 via :370-377, :409-414): a causal mask against the oracle's Gemma forward
    with the same mask (every row's logits), and visibly different from the zero-mask result; a
    fused-path KVCache refuses it rather than ignoring it."""
    import modeling_gemma as MG
    cfg, P, _ = setup
    gc = MG.GemmaConfig(**cfg["text_config"])
    lm = MG.GemmaForCausalLM(gc)
    with torch.no_grad():
        for name, p in lm.named_parameters():
            key = "language_model." + name
            if key in P:
                p.data = torch.from_numpy(P[key]).to("cuda", torch.bfloat16)
    lm.tie_weights()
    lm = lm.cuda()
    B, L = 1, 40
    embn = _x(np.random.default_rng(12), B, L, 2048) * 0.05
    emb = torch.from_numpy(embn).cuda().bfloat16()
    posn = np.broadcast_to(np.arange(L), (B, L)).copy()
    pos = torch.from_numpy(posn).cuda()
    cm = O.bf16(np.triu(np.full((L, L), -1e4, np.float32), 1))[None, None]
    causal = torch.from_numpy(cm).to("cuda", torch.bfloat16)
    got = lm(attention_mask=causal, position_ids=pos, inputs_embeds=emb)["logits"]
    assert got.shape == (B, L, cfg["text_config"]["vocab_size"]) and got.dtype == torch.float32
    ref = O.gemma_forward(P, cfg, embn, posn, O.KV(), mask=cm)
    with O.fp32_truth():
        truth = O.gemma_forward(P, cfg, embn, posn, O.KV(), mask=cm)
    assert_within_floor("gemma_causal_lm/causal_mask", np32(got), ref, truth)
    # row 0 attends only itself under the causal mask: not the zero-mask (bidirectional) result
    zero = lm(attention_mask=torch.zeros(B, 1, L, L, dtype=torch.bfloat16, device="cuda"), position_ids=pos,
              inputs_embeds=emb)["logits"]
    assert rel_l2(np32(got[:, 0]), np32(zero[:, 0])) > 5e-2
    # a cache the fused path owns attends every cached key: a non-zero mask is refused, not ignored
    kv = MG.KVCache()
    lm(attention_mask=torch.zeros(B, 1, L, L, dtype=torch.bfloat16, device="cuda"), position_ids=pos,
       inputs_embeds=emb, kv_cache=kv)
    with pytest.raises(NotImplementedError):
        lm(attention_mask=torch.full((B, 1, 1, L + 1), -1e4, dtype=torch.bfloat16, device="cuda"),
           position_ids=torch.full((B, 1), L, device="cuda"), inputs_embeds=emb[:, :1], kv_cache=kv)
