"""The oracle (oracle/paligemma_np.py, numpy restatement of the reference) pinned against the
golden vectors the reference modules produced (tests/golden/make_golden.py).  CPU only."""
import os

import numpy as np
import pytest

from oracle import paligemma_np as O
from oracle import weights as W

SEED = 1234


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.fixture(scope="module")
def gold(golden_dir):
    return np.load(os.path.join(golden_dir, "small_bf16.npz"))


@pytest.fixture(scope="module")
def small():
    cfg = W.small_config()
    return cfg, W.synthetic_state_dict_f32(cfg, SEED)


@pytest.fixture(scope="module")
def prefill(small, gold):
    cfg, P = small
    taps = {}
    lg, kv = O.paligemma_prefill(P, cfg, gold["ids"], O.from_bits(gold["pixels_bits"]), taps=taps)
    return lg, kv, taps


def test_bf16_rounding_is_rne():
    x = np.array([1.0, 1.00390625, 1.005859375, -2.5e-3, 3.0e38], np.float32)
    b = O.bf16(x)
    assert b[0] == 1.0 and b[1] == 1.0 and b[2] == np.float32(1.0078125)
    assert np.array_equal(O.from_bits(O.bf16_bits(x)), b)


def test_vision_embeddings_exact(prefill, gold):
    """patch conv + bias + position embedding: bit-exact vs the reference."""
    _, _, taps = prefill
    assert np.array_equal(taps["vision_embeddings"][:, ::8], O.from_bits(gold["tap_vision_embeddings"]))


@pytest.mark.parametrize("name,tol", [("vision_layer0", 6e-3), ("vision_layer1", 1e-2), ("image_features", 1e-2),
                                      ("text_layer0", 3e-2), ("text_layer1", 4e-2)])
def test_layer_outputs(prefill, gold, name, tol):
    _, _, taps = prefill
    assert rel(taps[name][:, ::8], O.from_bits(gold["tap_" + name])) < tol


def test_per_op_teacher_forced(small, gold):
    """Each op restated on the reference's own inputs (taps) reproduces the reference's output."""
    cfg, P = small
    g = lambda k: O.from_bits(gold["tap_" + k])  # noqa: E731
    # text layer 0 input norm -> q projection (rows ::8 of the taps)
    x = g("t0_ln_in")
    q = O.linear(x, P["language_model.model.layers.0.self_attn.q_proj.weight"])
    assert rel(q, g("t0_q")) < 1e-3
    # vision layer 0: LN1 -> q
    qv = O.linear(g("v0_ln1"), P["vision_tower.vision_model.encoder.layers.0.self_attn.q_proj.weight"],
                  P["vision_tower.vision_model.encoder.layers.0.self_attn.q_proj.bias"])
    assert rel(qv, g("v0_q")) < 1e-3


def test_merge_exact(gold):
    """_merge_input_ids_with_image_features (modeling_gemma.py:468-537) restated: text rows and
    scaled image rows are bit-exact vs the embeddings the reference fed its language model."""
    cfg = W.small_config()
    P = {"language_model.model.embed_tokens.weight": _embed(cfg)}
    feats_rows = O.from_bits(gold["tap_image_features"])  # rows 0, 8, 16, ... of the image features
    ref = O.from_bits(gold["tap_merged_embeds"])           # rows 0, 8, 16, ... of the merged embeds
    m = O.merge(P, cfg, None, gold["ids"])                  # text rows (image rows left zero)
    text_rows = np.arange(0, gold["ids"].shape[1], 8) >= 256
    assert np.array_equal(m[:, ::8][:, text_rows], ref[:, text_rows])
    scaled = O.bf16(feats_rows / np.float32(cfg["hidden_size"] ** 0.5))
    assert np.array_equal(scaled[:, : int((~text_rows).sum())], ref[:, ~text_rows])


_EMB = {}


def _embed(cfg):
    if "e" not in _EMB:
        _EMB["e"] = W.gen_f32("language_model.model.embed_tokens.weight", W.param_shapes(cfg)[
            "language_model.model.embed_tokens.weight"], SEED)
    return _EMB["e"]


def test_prefill_logits(prefill, gold):
    lg, _, _ = prefill
    assert rel(lg[:, -1], gold["prefill_logits_last"]) < 3e-2
    assert rel(lg[:, ::32], O.from_bits(gold["prefill_logits_rows"])) < 3e-2


def test_kv_cache_rows(prefill, gold):
    _, kv, _ = prefill
    assert rel(kv.k[0][:, :, ::4], O.from_bits(gold["k0"])) < 1e-2
    assert rel(kv.v[-1][:, :, ::4], O.from_bits(gold["v_last"])) < 3e-2


def test_greedy_tokens(small, gold):
    """inference.py semantics (position gap L+1): tokens equal the reference's wherever the
    reference's top-2 margin exceeds 0.25."""
    cfg, P = small
    toks, _ = O.greedy_generate(P, cfg, gold["ids"], O.from_bits(gold["pixels_bits"]), 16)
    ref = gold["greedy_tokens"]
    s = np.sort(O.from_bits(gold["greedy_logits"]), -1)
    margin = s[:, -1] - s[:, -2]
    diff = np.nonzero(toks[0] != ref)[0]
    assert len(diff) == 0 or margin[diff[0]] < 0.25


def test_rope_tables():
    """inv_freq / cos / sin as GemmaRotaryEmbedding computes them (modeling_gemma.py:151,178-185)."""
    import torch
    inv_t = 1.0 / (10000.0 ** (torch.arange(0, 256, 2, dtype=torch.int64).float() / 256))
    inv = O.inv_freq()
    assert np.max(np.abs(inv - inv_t.numpy()) / inv_t.numpy()) < 2e-7
    pos = np.array([[0, 1, 287, 289, 8191]])
    c, s = O.rope_cos_sin(pos, inv_t.numpy())
    f = (inv_t[None, :, None] @ torch.tensor(pos, dtype=torch.float32)[:, None, :]).transpose(1, 2)
    emb = torch.cat((f, f), -1)
    ct, st = emb.cos().to(torch.bfloat16).float().numpy(), emb.sin().to(torch.bfloat16).float().numpy()
    assert (c != ct).mean() < 1e-3 and (s != st).mean() < 1e-3


def test_pixels_from_u8(golden_dir):
    """process_images restated on the stored BICUBIC output equals the reference's fp32 pixels
    (sums recorded by make_golden.py)."""
    d = np.load(os.path.join(golden_dir, "pixels.npz"))
    from tests_helpers import pixels_from_u8
    keys = sorted(k.replace("u8_", "px_") for k in d.files if k.startswith("u8_"))
    sums = [pixels_from_u8(d[k.replace("px_", "u8_")]).astype(np.float64).sum() for k in keys]
    assert np.allclose(sums, d["px_sum"], rtol=0, atol=1e-6)


def test_full_size_fixture_consistency(golden_dir):
    """The full-shape fixtures are self-consistent: reference bf16 vs fp32 error is small (the
    synthetic init is well conditioned) and the stored top-k agree with the stored tokens."""
    b = np.load(os.path.join(golden_dir, "full_bf16.npz"))
    f = np.load(os.path.join(golden_dir, "full_fp32.npz"))
    assert b["tokens"].shape[-1] == 64
    assert np.array_equal(b["topk_idx"][:, 0], b["tokens"].reshape(-1))
    assert float(f["ref_bf16_rel_l2"].max()) < 0.05


def test_resize_oracle_bit_exact_vs_pil(golden_dir):
    """oracle/resize_np.py (PIL Resample.c restated) vs PIL's outputs in preprocess.npz."""
    import sys
    sys.path.insert(0, golden_dir)
    from make_preprocess import SYNTH, synthetic_image
    from oracle import resize_np as R
    g = np.load(os.path.join(golden_dir, "preprocess.npz"))
    for s in (224, 448):
        assert np.array_equal(R.resize_bicubic_u8(g["coco0_src"], s, s), g[f"coco0_{s}"])
    for seed, h, w, s in SYNTH[:4]:
        assert np.array_equal(R.resize_bicubic_u8(synthetic_image(seed, h, w), s, s), g[f"syn{seed}_{h}x{w}_{s}"])
    # the COCO fixture agrees with the pixels.npz one (the reference's process_images input)
    px = np.load(os.path.join(golden_dir, "pixels.npz"))
    assert np.array_equal(g["coco0_224"], px["u8_0_224"]) and np.array_equal(g["coco0_448"], px["u8_0_448"])


@pytest.mark.parametrize("mode", ["kv", "nokv"])
def test_ablation_harness(small, gold, golden_dir, mode):
    """The ablation harness (ablation_study_fixed.py:168-251 with load_model_simple's two patches)
    restated by O.ablation_generate vs the reference's own run of it (small_ablation_bf16.npz):
    KV mode incl. the step-0 prompt re-feed at one position over 2L keys, and no-KV mode."""
    cfg, P = small
    g = np.load(os.path.join(golden_dir, "small_ablation_bf16.npz"))
    ref = O.from_bits(g[f"{mode}_logits"])
    n = ref.shape[0]
    px = O.bf16(O.from_bits(gold["pixels_bits"]))
    toks, steps = O.ablation_generate(P, cfg, g["ids"], px, n, kv_mode=(mode == "kv"))
    per_step = [rel(steps[0, t], ref[t]) for t in range(n)]
    assert max(per_step) < 2e-2, per_step
    diff = np.nonzero(toks[0] != g[f"{mode}_tokens"])[0]
    assert len(diff) == 0 or g[f"{mode}_margin"][diff[0]] < 0.25


def test_ablation_fixture_consistency(golden_dir):
    """The full-size ablation fixture: greedy tokens are the stored top-1 of every step."""
    g = np.load(os.path.join(golden_dir, "full_ablation_bf16.npz"))
    for mode, n in (("kv", 64), ("nokv", 48)):
        assert g[f"{mode}_tokens"].shape == (n,)
        assert np.array_equal(g[f"{mode}_topk_idx"][:, 0], g[f"{mode}_tokens"])


def test_batch8_fp32_fixture_consistency(golden_dir):
    """full_batch8_fp32.npz (fp32 truth of each batched row) is pinned to the same generator as the
    image-0 fixture: row 0 is bit-identical to full_fp32.npz at the shared logit columns, and every
    row's reference-bf16 error vs its truth is in the range the bf16 model shows on image 0."""
    b8 = np.load(os.path.join(golden_dir, "full_batch8_bf16.npz"))
    f8 = np.load(os.path.join(golden_dir, "full_batch8_fp32.npz"))
    n = f8["sample_vals"].shape[1]
    assert n == b8["tokens"].shape[1] == 256          # configs[3]: 256 output tokens per image
    # row 0 is image 0 with the prompt of full256_*: the same reference run, token for token
    b0 = np.load(os.path.join(golden_dir, "full256_bf16.npz"))
    f0 = np.load(os.path.join(golden_dir, "full256_fp32.npz"))
    assert np.array_equal(b8["tokens"][0], b0["tokens"].reshape(-1)[:n])
    assert np.array_equal(f8["sample_idx"], b8["sample_idx"])
    assert f8["sample_vals"].shape == b8["sample_vals"].shape
    col = {int(c): i for i, c in enumerate(f0["sample_idx"])}
    shared = [col[int(c)] for c in f8["sample_idx"]]
    assert np.array_equal(f8["sample_vals"][0], f0["sample_vals"][:n, shared])
    assert np.array_equal(b8["sample_vals"][0], b0["sample_vals"][:n, shared])
    bv, fv = b8["sample_vals"], f8["sample_vals"]  # (an NpzFile decompresses an array on every key access)
    for r in range(fv.shape[0]):
        e = np.mean(np.linalg.norm(bv[r] - fv[r], axis=-1) / np.linalg.norm(fv[r], axis=-1))
        assert 1e-3 < e < 5e-2, (r, e)


def test_448_decode_fixture_consistency(golden_dir):
    """full448_decode_{bf16,fp32}.npz: its step 0 is the 448 px prefill fixture bit for bit (same ids,
    pixels and weights), its tokens are the stored top-1, and the reference bf16 sits 1e-3..2e-2 from
    its fp32 truth at every step."""
    p = np.load(os.path.join(golden_dir, "full448_bf16.npz"))
    b = np.load(os.path.join(golden_dir, "full448_decode_bf16.npz"))
    f = np.load(os.path.join(golden_dir, "full448_decode_fp32.npz"))
    assert np.array_equal(p["ids"], b["ids"]) and np.array_equal(p["sample_idx"], b["sample_idx"])
    assert np.array_equal(p["sample_vals"][0], b["sample_vals"][0])
    assert np.array_equal(b["topk_idx"][:, 0], b["tokens"].reshape(-1))
    assert f["sample_vals"].shape == b["sample_vals"].shape == (16, b["sample_idx"].shape[0])
    e = np.linalg.norm(b["sample_vals"] - f["sample_vals"], axis=1) / np.linalg.norm(f["sample_vals"], axis=1)
    assert 1e-3 < e.min() and e.max() < 2e-2, e


def test_ablation_and_nokv_fp32_fixture_consistency(golden_dir):
    """full_ablation_fp32.npz / full_nokv_fp32.npz (fp32 truths of configs[2] and of the ablation harness,
    teacher-forced on the bf16 tokens): same columns and steps as their bf16 fixtures; the no-KV truth's
    step 0 is the KV-cached truth's step 0 bit for bit (the same prefill); the reference bf16 sits 1e-3..3e-2
    from the no-KV truth, and further (the harness's model.to(bf16) also casts the rotary inv_freq,
    ablation_study_fixed.py:182) from the harness's truth."""
    g = np.load(os.path.join(golden_dir, "full_ablation_bf16.npz"))
    f = np.load(os.path.join(golden_dir, "full_ablation_fp32.npz"))
    assert np.array_equal(g["sample_idx"], f["sample_idx"])
    for mode in ("kv", "nokv"):
        a, b = g[f"{mode}_sample_vals"], f[f"{mode}_sample_vals"]
        assert a.shape == b.shape == (len(g[f"{mode}_tokens"]), len(g["sample_idx"]))
        e = np.linalg.norm(a - b, axis=1) / np.linalg.norm(b, axis=1)
        assert 1e-3 < e.min() and e.max() < 0.15, (mode, e.min(), e.max())
    n = np.load(os.path.join(golden_dir, "full_nokv_bf16.npz"))
    nf = np.load(os.path.join(golden_dir, "full_nokv_fp32.npz"))
    f0 = np.load(os.path.join(golden_dir, "full_fp32.npz"))
    assert nf["sample_vals"].shape == n["sample_vals"].shape
    assert np.array_equal(nf["sample_vals"][0], f0["sample_vals"][0])
    e = np.linalg.norm(n["sample_vals"] - nf["sample_vals"], axis=1) / np.linalg.norm(nf["sample_vals"], axis=1)
    assert 1e-3 < e.min() and e.max() < 3e-2, e


def test_torch_cpu_decoder_matches_oracle():
    """oracle/torch_cpu.py (the bench's CPU baseline, a torch bf16 port of the decode step) against the numpy
    oracle on the same synthetic weights and the same cache: logits rel-L2 < 1e-2 and equal argmax over
    three greedy steps (both keep the reference's bf16 rounding points; only accumulation order differs)."""
    import torch
    from oracle.torch_cpu import TorchCpuDecoder
    cfg = W.small_config(vision_layers=1, text_layers=2, vocab=4096)
    seed, n = 5, 40
    P = W.synthetic_state_dict_f32(cfg, seed)
    dec = TorchCpuDecoder(cfg, seed, max_kv=64)
    dec.fill_cache(n)
    kv = O.KV()
    for i in range(2):
        kv.update(dec.K[i, :n].float().numpy().transpose(1, 0, 2)[None], dec.V[i, :n].float().numpy().transpose(1, 0, 2)[None], i)
    tok = 108
    for s in range(3):
        got = dec.step(tok, n + 1 + s).numpy()
        ref = O.paligemma_decode(P, cfg, np.array([tok]), kv, n + 1 + s)[0, -1]
        rel = np.linalg.norm(got - ref) / np.linalg.norm(ref)
        assert rel < 1e-2, (s, rel)
        assert int(got.argmax()) == int(ref.argmax())
        tok = int(ref.argmax())
    assert torch.equal(dec.K[0, n:n + 3].float(), torch.from_numpy(kv.k[0][0, :, n:n + 3].transpose(1, 0, 2)))
