"""Generate the golden fixtures under tests/golden/ by running the REFERENCE modules.

Runs only in the survey container (it imports /root/reference/modeling_gemma.py,
modeling_siglip.py, processing_paligemma.py and inference.py; the reference never
travels to the GPU box).  The committed .npz files are data: inputs and the
reference's outputs on deterministic synthetic weights (oracle/wgen.c).

    python tests/golden/make_golden.py [--skip-full]

What is captured:
  pixels.npz        reference process_images on the committed COCO jpgs (224, 448)
  small_bf16.npz    2+2-layer full-width model, bf16: per-op taps, prefill logits,
                    16 greedy tokens through inference.test_inference (vision re-run,
                    position gap), KV-cache samples
  full_bf16.npz     PaliGemma-3B-224 shapes, bf16: 64 greedy tokens via
                    inference.test_inference, per-step top-k / margins / sampled logits
  full_fp32.npz     the same token path teacher-forced in fp32 ("truth")
  full448_bf16.npz  PaliGemma-3B-448 shapes, bf16 prefill
  full_nokv_bf16.npz  KV cache disabled, ablation semantics (ablation_study_fixed.py:244-251)
  small_ablation_bf16.npz  the same on the 2+2-layer model, every logit kept (the oracle's check)
  full_ablation_bf16.npz  the ablation harness itself (run_inference with load_model_simple's two
                    patches): KV mode 64 tokens incl. the step-0 prompt re-feed, no-KV mode 48 tokens
  full_batch8_bf16.npz  configs[3]: 8 distinct images, each run alone through inference.test_inference
  full_batch8_fp32.npz  the fp32 truth of each of those 8 rows, teacher-forced on its bf16 token path
  full448_decode_{bf16,fp32}.npz  448 px (L = 1056): 16 greedy KV-cached tokens and their fp32 truth
"""
from __future__ import annotations

import argparse
import math
import os
import sys
import time
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, REF)

from oracle import weights as W  # noqa: E402

import modeling_gemma as RG  # noqa: E402
import processing_paligemma as RP  # noqa: E402

sys.modules.setdefault("fire", types.SimpleNamespace(Fire=lambda *a, **k: None))
import inference as RI  # noqa: E402

SEED = 1234
N_SAMPLE_IDX = 1024
COCO = [f"{REF}/ablation_results/images/coco_{i}.jpg" for i in
        ("000000000285", "000000005529", "000000012667", "000000013597", "000000024919")]


def bits(t: torch.Tensor) -> np.ndarray:
    return t.detach().to(torch.bfloat16).contiguous().view(torch.int16).numpy().view(np.uint16)


def build_model(cfg: dict, dtype: torch.dtype):
    pcfg = RG.PaliGemmaConfig(**{k: v for k, v in cfg.items() if k not in ("bos_token_id", "eos_token_id")})
    with torch.device("meta"):
        model = RG.PaliGemmaForConditionalGeneration(pcfg)
    model = model.to_empty(device="cpu").to(dtype)
    shapes = W.param_shapes(cfg)
    sd = dict(model.named_parameters())
    for name, shape in shapes.items():
        p = sd[name]
        assert tuple(p.shape) == tuple(shape), (name, p.shape, shape)
        t = torch.from_numpy(W.gen_bf16(name, shape, SEED).view(np.int16)).view(torch.bfloat16)
        with torch.no_grad():
            p.copy_(t.to(dtype))
    model.tie_weights()
    # non-persistent buffers (to_empty leaves them uninitialised): recompute exactly as
    # the reference constructors do; inv_freq stays fp32 (inference.py / load_hf_model path)
    for layer in model.language_model.model.layers:
        re = layer.self_attn.rotary_emb
        re.inv_freq = 1.0 / (re.base ** (torch.arange(0, re.dim, 2, dtype=torch.int64).float() / re.dim))
    emb = model.vision_tower.vision_model.embeddings
    emb.position_ids = torch.arange(emb.num_positions).expand((1, -1))
    return model.eval(), pcfg


def prompt_ids(cfg: dict, n_text: int = 30, seed: int = 7) -> np.ndarray:
    rng = np.random.default_rng(seed)
    hi = min(cfg["image_token_index"], cfg["text_config"]["vocab_size"]) - 1
    txt = rng.integers(3, hi, size=n_text)
    newline = 108 if hi > 108 else 5
    ids = [cfg["image_token_index"]] * W.num_image_tokens(cfg) + [2] + txt.tolist() + [newline]
    return np.array([ids], dtype=np.int64)


class FakeTokenizer:
    """Stands in for the absent Gemma tokenizer: PaliGemmaProcessor's calls
    (processing_paligemma.py:63-77,107-113) and inference.py's decode/eos."""

    def __init__(self, ids, image_token_index, eos=-1):
        self.ids, self.image_token_index, self.eos_token_id = ids, image_token_index, eos
        self.bos_token = "<bos>"
        self.decoded = None

    def add_special_tokens(self, d):
        pass

    def add_tokens(self, toks):
        pass

    def convert_tokens_to_ids(self, t):
        return self.image_token_index

    def __call__(self, strings, return_tensors="pt", padding=None, truncation=None):
        s = strings[0]
        n = int((self.ids == self.image_token_index).sum())
        assert s.startswith("<image>" * n + "<bos>") and s.endswith("\n"), s[:64]
        ids = torch.from_numpy(self.ids.copy())
        return {"input_ids": ids, "attention_mask": torch.ones_like(ids)}

    def decode(self, toks, skip_special_tokens=True):
        self.decoded = toks.detach().cpu().numpy().astype(np.int64)
        return ""


def run_test_inference(model, cfg, ids, image_path, n_tokens):
    """Drive the reference's own inference.test_inference (inference.py:34-85)."""
    tok = FakeTokenizer(ids, cfg["image_token_index"])
    proc = RP.PaliGemmaProcessor(tok, W.num_image_tokens(cfg), cfg["vision_config"]["image_size"])
    step_logits = []
    orig_forward = model.forward

    def spy(*a, **k):
        out = orig_forward(*a, **k)
        step_logits.append(out["logits"][:, -1, :].detach().clone())
        return out

    model.forward = spy
    try:
        with torch.no_grad():
            RI.test_inference(model, proc, "cpu", "p", image_path, n_tokens, 0.8, 0.9, False)
    finally:
        model.forward = orig_forward
    return tok.decoded, torch.cat(step_logits, 0).float().numpy()


def reference_pixels(image_path, size):
    from PIL import Image
    img = Image.open(image_path)
    return RP.process_images([img], size=(size, size), resample=Image.Resampling.BICUBIC,
                             rescale_factor=1 / 255.0, image_mean=RP.IMAGENET_STANDARD_MEAN,
                             image_std=RP.IMAGENET_STANDARD_STD)[0]


def pixels_from_u8(u8):
    """processing_paligemma.py:20-29,47-49 restated on the resized uint8 image: x/255 (float64
    -> float32), (x - 0.5) / 0.5 in float32, HWC -> CHW.  make_pixels() checks it is
    bit-identical to the reference's process_images."""
    px = (u8 * (1 / 255.0)).astype(np.float32)
    return ((px - np.float32(0.5)) / np.float32(0.5)).transpose(2, 0, 1)


def make_pixels():
    """Stores the BICUBIC-resized uint8 images (the only lossy step, done by PIL); the model
    input is pixels_from_u8(u8), verified equal to the reference's process_images here."""
    from PIL import Image
    out, px_all = {}, {}
    for i, p in enumerate(COCO):
        for size in (224, 448):
            if size == 448 and i > 0:
                continue
            img = Image.open(p)
            u8 = np.array(RP.resize(img, (size, size), resample=Image.Resampling.BICUBIC))
            px = reference_pixels(p, size).astype(np.float32)
            assert np.array_equal(pixels_from_u8(u8), px), p
            out[f"u8_{i}_{size}"] = u8
            px_all[f"px_{i}_{size}"] = px
    out["px_sum"] = np.array([px_all[k].astype(np.float64).sum() for k in sorted(px_all)])
    np.savez_compressed(os.path.join(HERE, "pixels.npz"), **out)
    print("pixels.npz written")
    return px_all


def topk(x, k):
    idx = np.argsort(-x, axis=-1, kind="stable")[..., :k]
    return idx, np.take_along_axis(x, idx, -1)


def sample_idx(V, seed=11):
    return np.sort(np.random.default_rng(seed).choice(V, size=min(N_SAMPLE_IDX, V), replace=False))


def make_small(pixels):
    cfg = W.small_config()
    model, _ = build_model(cfg, torch.bfloat16)
    ids = prompt_ids(cfg)
    px = pixels["px_0_224"][None]
    taps = {}
    hooks = []

    def tap(name):
        def h(mod, inp, out):
            o = out[0] if isinstance(out, tuple) else out
            taps[name] = o.detach().clone()
        return h

    vm = model.vision_tower.vision_model
    hooks.append(vm.embeddings.register_forward_hook(tap("vision_embeddings")))
    l0 = vm.encoder.layers[0]
    hooks.append(l0.layer_norm1.register_forward_hook(tap("v0_ln1")))
    hooks.append(l0.self_attn.q_proj.register_forward_hook(tap("v0_q")))
    hooks.append(l0.self_attn.register_forward_hook(tap("v0_attn")))
    hooks.append(l0.mlp.fc1.register_forward_hook(tap("v0_fc1")))
    hooks.append(l0.mlp.register_forward_hook(tap("v0_mlp")))
    for i, l in enumerate(vm.encoder.layers):
        hooks.append(l.register_forward_hook(tap(f"vision_layer{i}")))
    hooks.append(vm.post_layernorm.register_forward_hook(tap("vision_out")))
    hooks.append(model.multi_modal_projector.register_forward_hook(tap("image_features")))
    lm = model.language_model.model
    hooks.append(lm.layers[0].input_layernorm.register_forward_hook(tap("t0_ln_in")))
    hooks.append(lm.layers[0].self_attn.q_proj.register_forward_hook(tap("t0_q")))
    hooks.append(lm.layers[0].self_attn.register_forward_hook(tap("t0_attn")))
    hooks.append(lm.layers[0].mlp.gate_proj.register_forward_hook(tap("t0_gate")))
    hooks.append(lm.layers[0].mlp.register_forward_hook(tap("t0_mlp")))
    for i, l in enumerate(lm.layers):
        hooks.append(l.register_forward_hook(tap(f"text_layer{i}")))
    hooks.append(lm.norm.register_forward_hook(tap("final_norm")))

    def pre_lm(mod, args, kwargs):
        taps["merged_embeds"] = kwargs["inputs_embeds"].detach().clone()
    hooks.append(model.language_model.register_forward_pre_hook(pre_lm, with_kwargs=True))

    kv = RG.KVCache()
    with torch.no_grad():
        out = model(input_ids=torch.from_numpy(ids), pixel_values=torch.from_numpy(px),
                    attention_mask=torch.ones_like(torch.from_numpy(ids)), kv_cache=kv)
    for h in hooks:
        h.remove()
    logits = out["logits"].float()
    # row-subsampled (every 8th row) to keep the fixture small; checksums cover whole tensors
    res = {"ids": ids, "pixels_bits": bits(torch.from_numpy(px)),
           "prefill_logits_last": logits[:, -1, :].numpy(), "prefill_logits_rows": bits(logits[:, ::32, :]),
           "k0": bits(kv.key_cache[0][:, :, ::4]), "v0": bits(kv.value_cache[0][:, :, ::4]),
           "k_last": bits(kv.key_cache[-1][:, :, ::4]), "v_last": bits(kv.value_cache[-1][:, :, ::4])}
    for n, t in taps.items():
        res["tap_" + n] = bits(t[:, ::8])
        res["sum_" + n] = np.array([t.double().sum().item(), t.double().abs().sum().item()])
    toks, step_logits = run_test_inference(model, cfg, ids, COCO[0], 16)
    res["greedy_tokens"] = toks
    res["greedy_logits"] = bits(torch.from_numpy(step_logits))
    np.savez_compressed(os.path.join(HERE, "small_bf16.npz"), **res)
    print("small_bf16.npz written; tokens:", toks.tolist())


def summarize_steps(step_logits, sidx, k=8):
    ti, tv = topk(step_logits, k)
    return {"topk_idx": ti, "topk_val": tv, "margin": tv[:, 0] - tv[:, 1],
            "sample_vals": step_logits[:, sidx],
            "row_sum": step_logits.astype(np.float64).sum(-1), "row_sumsq": (step_logits.astype(np.float64) ** 2).sum(-1)}


def make_full(pixels, n_tokens=64):
    cfg = W.full_config(224)
    V = cfg["text_config"]["vocab_size"]
    sidx = sample_idx(V)
    ids = prompt_ids(cfg)
    t0 = time.time()
    model, _ = build_model(cfg, torch.bfloat16)
    print(f"built full bf16 model in {time.time() - t0:.1f}s")
    t0 = time.time()
    toks, step_logits = run_test_inference(model, cfg, ids, COCO[0], n_tokens)
    print(f"full bf16 greedy {n_tokens} tokens in {time.time() - t0:.1f}s: {toks.tolist()}")
    res = {"ids": ids, "tokens": toks, "sample_idx": sidx, **summarize_steps(step_logits, sidx)}
    np.savez_compressed(os.path.join(HERE, "full_bf16.npz"), **res)

    # KV disabled, ablation semantics (ablation_study_fixed.py:238-251): full recompute each step
    nk = 8
    px = torch.from_numpy(pixels["px_0_224"][None])
    cur = torch.from_numpy(ids)
    gen, nl = [], []
    t0 = time.time()
    with torch.no_grad():
        for _ in range(nk):
            out = model(input_ids=cur, pixel_values=px.to(torch.bfloat16), attention_mask=torch.ones_like(cur), kv_cache=None)
            last = out["logits"][:, -1, :].float()
            nl.append(last.numpy())
            nxt = torch.argmax(last, dim=-1, keepdim=True)
            gen.append(int(nxt))
            cur = torch.cat([torch.from_numpy(ids), torch.tensor([gen])], dim=-1)
    print(f"no-kv {nk} tokens in {time.time() - t0:.1f}s: {gen}")
    np.savez_compressed(os.path.join(HERE, "full_nokv_bf16.npz"), ids=ids, tokens=np.array(gen),
                        sample_idx=sidx, **summarize_steps(np.concatenate(nl, 0), sidx))
    del model

    # fp32 truth, teacher-forced along the bf16 token path
    model, _ = build_model(cfg, torch.float32)
    t0 = time.time()
    kv = RG.KVCache()
    mask = torch.ones((1, ids.shape[1]), dtype=torch.int64)
    cur = torch.from_numpy(ids)
    fl = []
    with torch.no_grad():
        for step in range(n_tokens):
            out = model(input_ids=cur, pixel_values=px, attention_mask=mask, kv_cache=kv)
            fl.append(out["logits"][:, -1, :].float().numpy())
            cur = torch.tensor([[int(toks[step])]])
            mask = torch.cat([mask, torch.ones((1, 1))], dim=-1)
    fl = np.concatenate(fl, 0)
    print(f"fp32 teacher-forced {n_tokens} steps in {time.time() - t0:.1f}s")
    bf = step_logits
    rel = np.linalg.norm(bf - fl, axis=-1) / np.linalg.norm(fl, axis=-1)
    np.savez_compressed(os.path.join(HERE, "full_fp32.npz"), sample_idx=sidx, ref_bf16_rel_l2=rel,
                        **summarize_steps(fl, sidx))
    print("ref bf16 vs fp32 rel-L2 per step: max %.4f mean %.4f" % (rel.max(), rel.mean()))
    del model

    cfg448 = W.full_config(448)
    model, _ = build_model(cfg448, torch.bfloat16)
    ids448 = prompt_ids(cfg448)
    px448 = torch.from_numpy(pixels["px_0_448"][None])
    t0 = time.time()
    with torch.no_grad():
        out = model(input_ids=torch.from_numpy(ids448), pixel_values=px448,
                    attention_mask=torch.ones_like(torch.from_numpy(ids448)), kv_cache=RG.KVCache())
    last = out["logits"][:, -1, :].float().numpy()
    print(f"448 prefill in {time.time() - t0:.1f}s")
    np.savez_compressed(os.path.join(HERE, "full448_bf16.npz"), ids=ids448, sample_idx=sidx,
                        **summarize_steps(last, sidx))


def seeded_image(i):
    """Synthetic RGB test image i (5..7 of the batch): seeded smooth gradients + noise at a
    non-square size, written as PNG so the reference's own Image.open / BICUBIC path reads it."""
    from PIL import Image
    rng = np.random.default_rng(100 + i)
    h, w = 300 + 17 * i, 260 + 29 * i
    yy, xx = np.mgrid[0:h, 0:w]
    base = np.stack([(yy * (1 + c) + xx * (3 - c)) % 256 for c in range(3)], -1).astype(np.float64)
    img = np.clip(base * 0.6 + rng.integers(0, 100, (h, w, 3)), 0, 255).astype(np.uint8)
    path = f"/tmp/pgmi_seeded_{i}.png"
    Image.fromarray(img).save(path)
    return path


def make_batch_images(n_tokens=64, n_sample=256):
    """configs[3] parity target: eight distinct images (the 5 COCO jpgs + 3 seeded PNGs), each with
    its own synthetic prompt, run ONE AT A TIME through inference.test_inference (the reference
    cannot batch: processing_paligemma.py:80, modeling_gemma.py:526-528).  The build runs them as
    one B = 8 batch and compares each row with its own image's fixture."""
    from PIL import Image
    cfg = W.full_config(224)
    V = cfg["text_config"]["vocab_size"]
    sidx = sample_idx(V)[:: max(1, N_SAMPLE_IDX // n_sample)]
    t0 = time.time()
    model, _ = build_model(cfg, torch.bfloat16)
    print(f"built full bf16 model in {time.time() - t0:.1f}s")
    paths = COCO + [seeded_image(i) for i in range(5, 8)]
    res = {"sample_idx": sidx}
    ids_all, u8_all, toks_all, ti_all, tv_all, mg_all, sv_all = [], [], [], [], [], [], []
    for i, p in enumerate(paths):
        ids = prompt_ids(cfg, seed=7 + i)
        u8 = np.array(RP.resize(Image.open(p), (224, 224), resample=Image.Resampling.BICUBIC))
        assert np.array_equal(pixels_from_u8(u8), reference_pixels(p, 224).astype(np.float32)), p
        t0 = time.time()
        toks, step_logits = run_test_inference(model, cfg, ids, p, n_tokens)
        print(f"image {i}: {n_tokens} tokens in {time.time() - t0:.1f}s: {toks.tolist()[:16]}...")
        s = summarize_steps(step_logits, sidx)
        ids_all.append(ids[0]), u8_all.append(u8), toks_all.append(toks.reshape(-1))
        ti_all.append(s["topk_idx"]), tv_all.append(s["topk_val"]), mg_all.append(s["margin"])
        sv_all.append(s["sample_vals"])
    res.update(ids=np.stack(ids_all), u8=np.stack(u8_all), tokens=np.stack(toks_all), topk_idx=np.stack(ti_all),
               topk_val=np.stack(tv_all), margin=np.stack(mg_all), sample_vals=np.stack(sv_all))
    np.savez_compressed(os.path.join(HERE, "full_batch8_bf16.npz"), **res)
    print("full_batch8_bf16.npz written")


def make_batch_fp32():
    """fp32 truth for every row of full_batch8_bf16.npz: the reference model in fp32, teacher-forced on
    that image's bf16 reference tokens (the path its inference.test_inference run took), the same
    sampled logit columns per step -- so each batched row gets SURVEY.md sec.8c's "<= 1.5x the
    reference-bf16 error vs fp32" rule, not image 0 alone."""
    G = np.load(os.path.join(HERE, "full_batch8_bf16.npz"))
    cfg = W.full_config(224)
    sidx = G["sample_idx"]
    model, _ = build_model(cfg, torch.float32)
    out_vals = []
    for i in range(G["ids"].shape[0]):
        ids = G["ids"][i][None]
        toks = G["tokens"][i].reshape(-1)
        px = torch.from_numpy(pixels_from_u8(G["u8"][i])[None])
        kv = RG.KVCache()
        mask = torch.ones((1, ids.shape[1]), dtype=torch.int64)
        cur = torch.from_numpy(ids)
        fl = []
        t0 = time.time()
        with torch.no_grad():
            for step in range(toks.shape[0]):
                out = model(input_ids=cur, pixel_values=px if step == 0 else None, attention_mask=mask, kv_cache=kv)
                fl.append(out["logits"][:, -1, :].float().numpy()[:, sidx])
                cur = torch.tensor([[int(toks[step])]])
                mask = torch.cat([mask, torch.ones((1, 1))], dim=-1)
        out_vals.append(np.concatenate(fl, 0))
        print(f"image {i}: fp32 teacher-forced {toks.shape[0]} steps in {time.time() - t0:.1f}s")
    np.savez_compressed(os.path.join(HERE, "full_batch8_fp32.npz"), sample_idx=sidx, sample_vals=np.stack(out_vals))
    print("full_batch8_fp32.npz written")


def make_long(pixels, n_tokens=256):
    """configs[1] as BASELINE.json states it: 256 greedy tokens with the KV cache (KV length up to
    L + 256 + 1), through inference.test_inference, plus the prefill's ALL-ROW logits
    (modeling_gemma.py:417-418: (1, L, 257216) fp32) summarised per row; then the fp32 truth
    teacher-forced on the same token path."""
    cfg = W.full_config(224)
    V = cfg["text_config"]["vocab_size"]
    sidx = sample_idx(V)
    ids = prompt_ids(cfg)
    model, _ = build_model(cfg, torch.bfloat16)
    prefill = {}
    orig_forward = model.forward

    def spy(*a, **k):
        out = orig_forward(*a, **k)
        if not prefill:
            lg = out["logits"][0].float().numpy()          # (L, V): every prefill row
            ti, tv = topk(lg, 8)
            prefill.update(rows_topk_idx=ti, rows_topk_val=tv, rows_sum=lg.astype(np.float64).sum(-1),
                           rows_sumsq=(lg.astype(np.float64) ** 2).sum(-1), rows_sample_vals=lg[::8][:, sidx])
        return out

    model.forward = spy
    t0 = time.time()
    try:
        toks, step_logits = run_test_inference(model, cfg, ids, COCO[0], n_tokens)
    finally:
        model.forward = orig_forward
    print(f"full bf16 greedy {n_tokens} tokens in {time.time() - t0:.1f}s")
    res = {"ids": ids, "tokens": toks.reshape(-1), "sample_idx": sidx, **summarize_steps(step_logits, sidx),
           **prefill}
    np.savez_compressed(os.path.join(HERE, "full256_bf16.npz"), **res)
    del model
    model, _ = build_model(cfg, torch.float32)
    px = torch.from_numpy(pixels["px_0_224"][None])
    kv = RG.KVCache()
    mask = torch.ones((1, ids.shape[1]), dtype=torch.int64)
    cur = torch.from_numpy(ids)
    fl = []
    with torch.no_grad():
        for step in range(n_tokens):
            out = model(input_ids=cur, pixel_values=px if step == 0 else None, attention_mask=mask, kv_cache=kv)
            fl.append(out["logits"][:, -1, :].float().numpy()[:, sidx])
            cur = torch.tensor([[int(toks.reshape(-1)[step])]])
            mask = torch.cat([mask, torch.ones((1, 1))], dim=-1)
    np.savez_compressed(os.path.join(HERE, "full256_fp32.npz"), sample_idx=sidx,
                        sample_vals=np.concatenate(fl, 0))
    print("full256_{bf16,fp32}.npz written")


def make_448_decode(pixels, n_tokens=16):
    """configs[4]'s shapes (448 px, L = 1056) through the KV-cached decode loop: n_tokens greedy tokens
    via inference.test_inference (step 0 is the prefill's last row), then the fp32 truth teacher-forced
    on the same token path (pixel_values at step 0 only: the later steps' image features are discarded
    by the merge, modeling_gemma.py:509-531)."""
    cfg = W.full_config(448)
    V = cfg["text_config"]["vocab_size"]
    sidx = sample_idx(V)
    ids = prompt_ids(cfg)
    model, _ = build_model(cfg, torch.bfloat16)
    t0 = time.time()
    toks, step_logits = run_test_inference(model, cfg, ids, COCO[0], n_tokens)
    toks = toks.reshape(-1)
    print(f"448 bf16 greedy {n_tokens} tokens in {time.time() - t0:.1f}s: {toks.tolist()}")
    np.savez_compressed(os.path.join(HERE, "full448_decode_bf16.npz"), ids=ids, tokens=toks, sample_idx=sidx,
                        **summarize_steps(step_logits, sidx))
    del model
    model, _ = build_model(cfg, torch.float32)
    px = torch.from_numpy(pixels["px_0_448"][None])
    kv = RG.KVCache()
    mask = torch.ones((1, ids.shape[1]), dtype=torch.int64)
    cur = torch.from_numpy(ids)
    fl = []
    t0 = time.time()
    with torch.no_grad():
        for step in range(n_tokens):
            out = model(input_ids=cur, pixel_values=px if step == 0 else None, attention_mask=mask, kv_cache=kv)
            fl.append(out["logits"][:, -1, :].float().numpy()[:, sidx])
            cur = torch.tensor([[int(toks[step])]])
            mask = torch.cat([mask, torch.ones((1, 1))], dim=-1)
    fl = np.concatenate(fl, 0)
    print(f"448 fp32 teacher-forced {n_tokens} steps in {time.time() - t0:.1f}s")
    np.savez_compressed(os.path.join(HERE, "full448_decode_fp32.npz"), sample_idx=sidx, sample_vals=fl)
    print("full448_decode_{bf16,fp32}.npz written")


def make_ablation(n_kv=64, n_nokv=48, small=False):
    """The paper's own harness (ablation_study_fixed.py:168-287 run_inference) on the reference model
    with BOTH of load_model_simple's patches applied (:335-342: the merge and every layer's rotary
    forward), bf16, greedy (temperature 0.0).

    KV mode: the discarded prefill (:194-199), then step 0 re-feeds the whole prompt + pixels into the
    filled cache -- every prompt row at the single position cumsum(mask)[:, -1:] = L (:130-133) and
    attending 2L keys (:124-126) -- then q_len == 1 steps at positions L+t over 2L+t keys.
    no-KV mode: every step re-runs vision + a bidirectional prefill over prompt + generated (:244-251).

    torch.cuda.synchronize (:204,211,253) is stubbed: there is no GPU in this container."""
    sys.path.insert(0, REF)
    import ablation_study_fixed as AB
    cfg = W.small_config() if small else W.full_config(224)
    V = cfg["text_config"]["vocab_size"]
    sidx = sample_idx(V)
    ids = prompt_ids(cfg)
    model, _ = build_model(cfg, torch.bfloat16)
    model._merge_input_ids_with_image_features = types.MethodType(AB.patched_merge_input_ids_with_image_features, model)
    for layer in model.language_model.model.layers:
        layer.self_attn.rotary_emb.forward = types.MethodType(AB.patched_rotary_forward, layer.self_attn.rotary_emb)
    tok = FakeTokenizer(ids, cfg["image_token_index"])
    proc = RP.PaliGemmaProcessor(tok, W.num_image_tokens(cfg), cfg["vision_config"]["image_size"])
    sync = torch.cuda.synchronize
    torch.cuda.synchronize = lambda *a, **k: None
    res = {"ids": ids, "sample_idx": sidx}
    try:
        for mode, n in (("kv", n_kv), ("nokv", n_nokv)):
            calls = []
            orig_forward = model.forward

            def spy(*a, **k):
                out = orig_forward(*a, **k)
                calls.append(out["logits"][:, -1, :].detach().float().clone())
                return out

            model.forward = spy
            t0 = time.time()
            try:
                with torch.no_grad():
                    r = AB.run_inference(model, proc, COCO[0], "p",
                                         {"dtype": torch.bfloat16, "kv_cache": mode == "kv", "max_tokens": n,
                                          "temperature": 0.0}, return_tokens=True)
            finally:
                del model.forward
            toks = np.array(r["token_ids"], dtype=np.int64).reshape(-1)
            step_logits = torch.cat(calls[1:], 0).numpy()      # calls[0] is the discarded prefill
            assert step_logits.shape[0] == n == toks.shape[0]
            print(f"ablation {mode}: {n} tokens in {time.time() - t0:.1f}s: {toks.tolist()[:24]}...")
            s = summarize_steps(step_logits, sidx)
            res.update({f"{mode}_tokens": toks, **{f"{mode}_{k}": v for k, v in s.items()}})
            if small:  # every logit of every step (small vocabulary): the oracle's CPU check
                res[f"{mode}_logits"] = bits(torch.from_numpy(step_logits))
            if mode == "kv":
                res["kv_prefill_topk_idx"], res["kv_prefill_topk_val"] = topk(calls[0].numpy(), 8)
    finally:
        torch.cuda.synchronize = sync
    name = "small_ablation_bf16.npz" if small else "full_ablation_bf16.npz"
    np.savez_compressed(os.path.join(HERE, name), **res)
    print(name, "written")


def make_nokv_fp32():
    """fp32 truth for full_nokv_bf16.npz (configs[2]): the reference model in fp32, KV cache disabled
    with the ablation's semantics (a full forward over prompt + generated tokens each step,
    ablation_study_fixed.py:244-251), teacher-forced on the bf16 run's greedy tokens."""
    g = np.load(os.path.join(HERE, "full_nokv_bf16.npz"))
    cfg = W.full_config(224)
    sidx = g["sample_idx"]
    ids = g["ids"]
    toks = g["tokens"].reshape(-1)
    P = np.load(os.path.join(HERE, "pixels.npz"))
    px = torch.from_numpy(pixels_from_u8(P["u8_0_224"])[None])
    model, _ = build_model(cfg, torch.float32)
    fl = []
    t0 = time.time()
    with torch.no_grad():
        for t in range(len(toks)):
            cur = torch.from_numpy(np.concatenate([ids, toks[None, :t]], 1))
            out = model(input_ids=cur, pixel_values=px, attention_mask=torch.ones_like(cur), kv_cache=None)
            fl.append(out["logits"][:, -1, :].float().numpy()[:, sidx])
    fl = np.concatenate(fl, 0)
    rel = np.linalg.norm(g["sample_vals"] - fl, axis=-1) / np.linalg.norm(fl, axis=-1)
    print(f"no-kv fp32 teacher-forced {len(toks)} steps in {time.time() - t0:.1f}s; ref bf16 vs fp32 rel-L2 "
          f"max {rel.max():.4f} mean {rel.mean():.4f}")
    np.savez_compressed(os.path.join(HERE, "full_nokv_fp32.npz"), sample_idx=sidx, sample_vals=fl)


def make_ablation_fp32():
    """fp32 truth for both modes of full_ablation_bf16.npz: the paper's harness itself
    (ablation_study_fixed.py run_inference, both load_model_simple patches) on the reference model in
    fp32, teacher-forced on the bf16 run's tokens.  run_inference picks each token by argmax of
    outputs["logits"][:, -1, :] (:226-229) and uses the logits for nothing else, so the spy records the
    fp32 row and hands the harness a one-hot row at the bf16 token: the harness's own loop (re-feeds,
    masks, positions, cache) then walks the bf16 token path."""
    sys.path.insert(0, REF)
    import ablation_study_fixed as AB
    g = np.load(os.path.join(HERE, "full_ablation_bf16.npz"))
    cfg = W.full_config(224)
    sidx = g["sample_idx"]
    ids = g["ids"]
    model, _ = build_model(cfg, torch.float32)
    model._merge_input_ids_with_image_features = types.MethodType(AB.patched_merge_input_ids_with_image_features, model)
    for layer in model.language_model.model.layers:
        layer.self_attn.rotary_emb.forward = types.MethodType(AB.patched_rotary_forward, layer.self_attn.rotary_emb)
    tok = FakeTokenizer(ids, cfg["image_token_index"])
    proc = RP.PaliGemmaProcessor(tok, W.num_image_tokens(cfg), cfg["vision_config"]["image_size"])
    sync = torch.cuda.synchronize
    torch.cuda.synchronize = lambda *a, **k: None
    res = {"sample_idx": sidx}
    try:
        for mode in ("kv", "nokv"):
            teacher = g[f"{mode}_tokens"].reshape(-1)
            rows, picks = [], []
            orig_forward = model.forward

            def spy(*a, **k):
                out = orig_forward(*a, **k)
                last = out["logits"][:, -1, :].detach().float()
                rows.append(last.numpy()[:, sidx].copy())
                picks.append(int(last.argmax()))
                step = len(rows) - 2                     # rows[0] is the discarded prefill
                if step >= 0:
                    forced = torch.zeros_like(out["logits"][:, -1:, :])
                    forced[..., int(teacher[step])] = 1.0
                    out = dict(out)
                    out["logits"] = forced
                return out

            model.forward = spy
            t0 = time.time()
            try:
                with torch.no_grad():
                    r = AB.run_inference(model, proc, COCO[0], "p",
                                         {"dtype": torch.float32, "kv_cache": mode == "kv", "max_tokens": len(teacher),
                                          "temperature": 0.0}, return_tokens=True)
            finally:
                del model.forward
            assert np.array_equal(np.array(r["token_ids"]).reshape(-1), teacher)
            fl = np.concatenate(rows[1:], 0)
            rel = np.linalg.norm(g[f"{mode}_sample_vals"] - fl, axis=-1) / np.linalg.norm(fl, axis=-1)
            agree = int((np.array(picks[1:]) == teacher).sum())
            print(f"ablation fp32 {mode}: {len(teacher)} steps in {time.time() - t0:.1f}s, fp32 argmax == bf16 "
                  f"token at {agree}/{len(teacher)}; ref bf16 vs fp32 rel-L2 max {rel.max():.4f} mean {rel.mean():.4f}")
            res[f"{mode}_sample_vals"] = fl
    finally:
        torch.cuda.synchronize = sync
    np.savez_compressed(os.path.join(HERE, "full_ablation_fp32.npz"), **res)
    print("full_ablation_fp32.npz written")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-full", action="store_true")
    ap.add_argument("--only", choices=["batch8", "batch8_fp32", "long", "ablation", "448decode", "r5", "r6"], default=None,
                    help="generate only one later round's fixtures (full_batch8 / full256 / full_ablation)")
    a = ap.parse_args()
    torch.set_num_threads(8)
    px = make_pixels() if a.only not in ("batch8", "batch8_fp32", "ablation", "r5", "r6") else None
    if a.only == "r5":
        # round 5: fp32 truths for configs[2] (no-KV) and both modes of the ablation harness; configs[3]'s
        # batched rows at their stated 256 output tokens, with their fp32 truths
        make_nokv_fp32()
        make_ablation_fp32()
        make_batch_images(n_tokens=256)
        make_batch_fp32()
    elif a.only == "r6":
        # round 6: configs[3]'s batched rows with the same 1,024 sampled vocabulary entries per step as every
        # other full-size fixture (256 before), and their fp32 truths
        make_batch_images(n_tokens=256, n_sample=N_SAMPLE_IDX)
        make_batch_fp32()
    elif a.only == "batch8":
        make_batch_images()
        make_batch_fp32()
    elif a.only == "batch8_fp32":
        make_batch_fp32()
    elif a.only == "ablation":
        make_ablation(16, 8, small=True)
        make_ablation()
    elif a.only == "long":
        make_long(px)
    elif a.only == "448decode":
        make_448_decode(px)
    else:
        make_small(px)
        if not a.skip_full:
            make_full(px)
            make_batch_images()
            make_batch_fp32()
            make_long(px)
            make_ablation(16, 8, small=True)
            make_ablation()
