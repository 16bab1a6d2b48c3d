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
    assert weights is None
    assert rel_l2(np32(out), O.siglip_attention(P, pre + "self_attn.", x, 16)) < 1e-2
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
