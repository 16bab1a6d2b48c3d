"""Full PaliGemma-3B shapes (224 and 448 px) on the GPU vs the golden vectors the reference
produced (tests/golden/full_*.npz, tests/golden/make_golden.py).  Parity rules (SURVEY.md
sec.8c):
  * teacher-forced along the reference's greedy path, our argmax equals the reference's token
    wherever the reference's top-2 margin exceeds 0.25;
  * |our logit - reference logit| <= 0.25 at the reference's top-8 tokens of every step;
  * our bf16 error vs the fp32 reference is <= 1.5x the reference-bf16 error vs fp32
    (rel-L2 over the 1024 sampled vocabulary entries, averaged over the 64 steps);
  * per-step rel-L2 vs the reference bf16 <= 2e-2, or where the reference bf16 is itself further
    from its fp32 truth, <= 1.45x that step's reference error (mean over the steps <= 1.25x the
    reference's mean error): tests_helpers.assert_step_rule, measured table in DESIGN.md sec.5;
  * free-running greedy tokens equal the reference's up to the first low-margin step.
"""
import os

import numpy as np
import pytest
import torch

from oracle import weights as W
from tests_helpers import check_model_parity, logit_stats, pixels_from_u8

pytestmark = [pytest.mark.gpu, pytest.mark.slow]
SEED = 1234


@pytest.fixture(scope="module")
def G(golden_dir):
    load = lambda n: np.load(os.path.join(golden_dir, n))  # noqa: E731
    return {"bf16": load("full_bf16.npz"), "fp32": load("full_fp32.npz"), "nokv": load("full_nokv_bf16.npz"),
            "448": load("full448_bf16.npz"), "px": load("pixels.npz"), "bf16_256": load("full256_bf16.npz"), "nokv_fp32": load("full_nokv_fp32.npz"),
            "fp32_256": load("full256_fp32.npz"), "448d": load("full448_decode_bf16.npz"),
            "448d_fp32": load("full448_decode_fp32.npz")}


def _engine(image_size, max_seq=320, max_kv=576):
    from pgmi import Engine
    e = Engine(W.full_config(image_size), max_batch=1, max_seq=max_seq, max_kv=max_kv)
    e.fill_synthetic(SEED, W.init_policy)
    e.prepare()
    return e


@pytest.fixture(scope="module")
def eng224():
    e = _engine(224)
    yield e
    del e
    torch.cuda.empty_cache()


def _px(G, key):
    return torch.from_numpy(pixels_from_u8(G["px"][key])[None]).cuda()


def _teacher_forced(e, G, gb, gf, n, px_key="u8_0_224", kv_cap=576, label="full224"):
    ids = torch.from_numpy(gb["ids"]).cuda()
    L = ids.shape[1]
    ref_toks = gb["tokens"].reshape(-1)
    sidx = torch.from_numpy(gb["sample_idx"]).cuda()
    kv = e.new_kv(1, kv_cap)
    feats = e.project(e.vision(_px(G, px_key)))
    lg = e.lm_forward(kv, 0, torch.arange(L)[None], ids=ids, image_feats=feats, logits_rows=1)[:, 0]
    steps_logits = [lg]
    for t in range(1, n):
        cur = torch.tensor([int(ref_toks[t - 1])], device="cuda")
        steps_logits.append(e.decode(cur, kv, L + t - 1, L + t, graph=True).clone())
    ours = torch.cat(steps_logits, 0)                       # (n, V)
    ours_s = ours[:, sidx].cpu().numpy()
    top_idx = torch.from_numpy(gb["topk_idx"][:n]).cuda()
    ours_top = torch.gather(ours, 1, top_idx).cpu().numpy()
    # |delta| at the reference's top-8
    assert np.abs(ours_top - gb["topk_val"][:n]).max() <= 0.25
    # argmax agreement where the reference is decisive
    am = ours.argmax(-1).cpu().numpy()
    decisive = gb["margin"][:n] > 0.25
    assert np.array_equal(am[decisive], ref_toks[:n][decisive]), (am, ref_toks[:n])
    # per-step closeness to the reference bf16 (against its own fp32 floor) and our
    # error vs the fp32 truth relative to the reference's own bf16 error
    check_model_parity(f"{label}/teacher_forced_{n}", ours_s, gb["sample_vals"][:n], gf["sample_vals"][:n])


@torch.no_grad()
def test_teacher_forced_64_steps(eng224, G):
    _teacher_forced(eng224, G, G["bf16"], G["fp32"], 64)


@torch.no_grad()
def test_teacher_forced_256_steps(eng224, G):
    """configs[1] as BASELINE.json states it: 256 output tokens, KV length up to 544 (past the
    12-chunk register form of the o_proj prologue's attention combine)."""
    _teacher_forced(eng224, G, G["bf16_256"], G["fp32_256"], 256)


@pytest.mark.parametrize("n", [64, 256])
@torch.no_grad()
def test_free_running_greedy(eng224, G, n):
    gb = G["bf16"] if n == 64 else G["bf16_256"]
    ids = torch.from_numpy(gb["ids"]).cuda()
    toks = eng224.generate(ids, _px(G, "u8_0_224"), n, graph=True).cpu().numpy()[0]
    ref = gb["tokens"].reshape(-1)
    diff = np.nonzero(toks != ref)[0]
    if len(diff):
        # the first divergence must sit on a step where the reference itself is indecisive
        assert gb["margin"][diff[0]] < 0.25, (diff[0], toks[:diff[0] + 2], ref[:diff[0] + 2], gb["margin"][diff[0]])


@torch.no_grad()
def test_no_kv_cache_ablation(eng224, G):
    """BASELINE config 3: KV cache disabled, each step a full recompute over prompt + generated
    tokens (ablation_study_fixed.py:244-251), teacher-forced on the reference's tokens: top-8 and
    argmax as above, and SURVEY sec.8c's per-step rel-L2 rule over the 1,024 sampled logits against the
    reference bf16, with its fp32 truth (full_nokv_fp32.npz: the reference in fp32, teacher-forced on
    the same tokens) as the floor and the "<= 1.5x the reference's own error" bound."""
    g = G["nokv"]
    ids0 = torch.from_numpy(g["ids"]).cuda()
    ref = g["tokens"].reshape(-1)
    sidx = torch.from_numpy(g["sample_idx"]).cuda()
    px = _px(G, "u8_0_224")
    feats = eng224.project(eng224.vision(px))
    samples = []
    for t in range(len(ref)):
        ids = torch.cat([ids0, torch.tensor([ref[:t].tolist()], dtype=torch.int64, device="cuda")], 1)
        L = ids.shape[1]
        kv = eng224.scratch_kv(1, L)
        lg = eng224.lm_forward(kv, 0, torch.arange(L)[None], ids=ids, image_feats=feats, logits_rows=1)[0, 0]
        top = torch.gather(lg, 0, torch.from_numpy(g["topk_idx"][t]).cuda()).cpu().numpy()
        assert np.abs(top - g["topk_val"][t]).max() <= 0.25
        if g["margin"][t] > 0.25:
            assert int(lg.argmax()) == int(ref[t])
        samples.append(lg[sidx].cpu().numpy())
    check_model_parity("full224/no_kv", np.stack(samples), g["sample_vals"], G["nokv_fp32"]["sample_vals"])


@torch.no_grad()
def test_prefill_448(G):
    """BASELINE config 5: 1024 image tokens + 32 text tokens (L = 1056)."""
    g = G["448"]
    e = _engine(448, max_seq=1088, max_kv=1088)
    ids = torch.from_numpy(g["ids"]).cuda()
    L = ids.shape[1]
    feats = e.project(e.vision(_px(G, "u8_0_448")))
    # logits_rows 1 (every row's final hidden kept) and 2 (the generate loop's prefill: the last
    # layer past its K/V for the last row only) both meet the reference
    for rows in (1, 2):
        kv = e.new_kv(1, 1088)
        lg = e.lm_forward(kv, 0, torch.arange(L)[None], ids=ids, image_feats=feats, logits_rows=rows)[0, 0]
        top = torch.gather(lg, 0, torch.from_numpy(g["topk_idx"][0]).cuda()).cpu().numpy()
        assert np.abs(top - g["topk_val"][0]).max() <= 0.25, rows
        s = lg[torch.from_numpy(g["sample_idx"]).cuda()].cpu().numpy()
        # the fp32 truth of this prefill step is step 0 of full448_decode_fp32.npz (same ids, pixels
        # and weights: its bf16 step 0 equals this fixture exactly): the SURVEY sec.8c rule
        check_model_parity(f"full448/prefill_rows{rows}", s[None], g["sample_vals"][:1],
                           G["448d_fp32"]["sample_vals"][:1])
        if g["margin"][0] > 0.25:
            assert int(lg.argmax()) == int(g["topk_idx"][0, 0]), rows
    del e
    torch.cuda.empty_cache()


@torch.no_grad()
def test_decode_448_teacher_forced(G):
    """configs[4]'s shapes through the KV-cached decode loop: the 448 px prefill (L = 1056) and 15
    graph-replayed decode steps over 1057..1071 cached keys (17 flash-decoding chunks: past the
    12-chunk register form of the o_proj prologue's combine), teacher-forced on the reference's
    16 greedy tokens (tests/golden/full448_decode_*.npz), under the same rules as 224 px."""
    e = _engine(448, max_seq=1088, max_kv=1088)
    _teacher_forced(e, G, G["448d"], G["448d_fp32"], 16, px_key="u8_0_448", kv_cap=1088, label="full448")
