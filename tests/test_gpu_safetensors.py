"""Native safetensors loading (pgmi_load_safetensors): every slab
weight written from checkpoint shards in BF16 / F32 / F16 must equal torch's own conversion of
the tensor to bf16, bit for bit; names outside the slab (a tied lm_head) are skipped; the drop-in
utils.load_model builds a working model from config.json + shards."""
import json
import os

import numpy as np
import pytest
import torch
from safetensors.torch import save_file

from oracle import weights as W

pytestmark = pytest.mark.gpu


def _checkpoint(tmp_path, cfg, seed=0):
    from pgmi import Engine
    probe = Engine(cfg, max_batch=1, max_seq=300, max_kv=320)
    g = torch.Generator().manual_seed(seed)
    sd = {}
    for i, (n, v) in enumerate(probe.views.items()):
        t = torch.randn(tuple(v.shape), generator=g) * (0.5 / max(1.0, float(v.shape[-1]) ** 0.5))
        sd[n] = t.to((torch.bfloat16, torch.float32, torch.float16)[i % 3])
    del probe
    sd["language_model.lm_head.weight"] = sd["language_model.model.embed_tokens.weight"].clone()
    names = sorted(sd)
    half = len(names) // 2
    d = tmp_path / "ckpt"
    d.mkdir()
    save_file({k: sd[k].contiguous() for k in names[:half]}, str(d / "model-00001-of-00002.safetensors"))
    save_file({k: sd[k].contiguous() for k in names[half:]}, str(d / "model-00002-of-00002.safetensors"))
    with open(d / "config.json", "w") as f:
        json.dump(cfg, f)
    return d, sd


def test_shards_load_bit_exact(tmp_path):
    from pgmi import Engine
    cfg = W.small_config(vision_layers=1, text_layers=1, vocab=1024)
    d, sd = _checkpoint(tmp_path, cfg)
    eng = Engine(cfg, max_batch=1, max_seq=300, max_kv=320)
    eng.prepare()
    n = eng.load_safetensors(str(d))
    assert n == len(eng.views)
    for name, view in eng.views.items():
        want = sd[name].to(torch.bfloat16).cuda()
        assert torch.equal(view.view(torch.int16), want.view(torch.int16)), name
    # the loaded weights drive a forward (prepare re-runs for the derived tensors)
    px = torch.rand((1, 3, 224, 224), device="cuda") * 2 - 1
    feats = eng.vision(px)
    assert torch.isfinite(feats.float()).all()


def test_shape_mismatch_is_value_error(tmp_path):
    from pgmi import Engine
    cfg = W.small_config(vision_layers=1, text_layers=1, vocab=1024)
    eng = Engine(cfg, max_batch=1, max_seq=300, max_kv=320)
    p = str(tmp_path / "bad.safetensors")
    save_file({"multi_modal_projector.linear.bias": torch.zeros(7)}, p)
    with pytest.raises(ValueError):
        eng.load_safetensors(p, strict=False)
    with pytest.raises(KeyError):  # strict: the rest of the slab is missing
        save_file({"multi_modal_projector.linear.bias": torch.zeros(cfg["projection_dim"])}, p)
        eng.load_safetensors(p, strict=True)


def test_drop_in_load_model(tmp_path):
    import utils
    cfg = W.small_config(vision_layers=1, text_layers=1, vocab=1024)
    d, sd = _checkpoint(tmp_path, cfg, seed=3)
    model = utils.load_model(str(d), device="cuda")
    p = dict(model.named_parameters())
    for name in ("language_model.model.layers.0.mlp.down_proj.weight", "multi_modal_projector.linear.weight"):
        assert torch.equal(p[name].detach().view(torch.int16), sd[name].to(torch.bfloat16).cuda().view(torch.int16))
    L = W.num_image_tokens(cfg) + 4
    ids = torch.tensor([[cfg["image_token_index"]] * (L - 4) + [2, 17, 99, 108]], device="cuda")
    out = model(input_ids=ids, pixel_values=torch.rand((1, 3, 224, 224), device="cuda"),
                attention_mask=torch.ones_like(ids))
    assert out["logits"].shape == (1, L, cfg["text_config"]["vocab_size"])
    assert torch.isfinite(out["logits"]).all()
