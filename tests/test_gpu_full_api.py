"""The drop-in PaliGemmaForConditionalGeneration at the FULL PaliGemma-3B / 224 px shapes, driven as
the reference's inference.py drives it (inference.py:55-78), against the reference's own outputs
(tests/golden/full256_bf16.npz, full_bf16.npz):

  * prefill logits of EVERY position at V = 257,216 (modeling_gemma.py:417-418), through the
    default lazy logits (last row eager, the rest materialised on first read) and through the
    eager all-row mode -- per row |delta| <= 0.25 at the reference's top-8, argmax where the
    reference's margin exceeds 0.25, sampled rel-L2 < 4e-2 on average / 6e-2 at most over every 8th row;
  * the inference.py greedy loop through forward() for 64 tokens (pixel_values re-passed, the
    attention mask grown by a float column per step, next_token.item() per token).
"""
import os

import numpy as np
import pytest
import torch

from oracle import weights as W
from tests_helpers import check_model_parity, pixels_from_u8

pytestmark = [pytest.mark.gpu, pytest.mark.slow]
SEED = 1234


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.fixture(scope="module")
def G(golden_dir):
    load = lambda n: np.load(os.path.join(golden_dir, n))  # noqa: E731
    return {"256": load("full256_bf16.npz"), "64": load("full_bf16.npz"), "64f": load("full_fp32.npz"),
            "px": load("pixels.npz")}


@pytest.fixture(scope="module")
def model():
    import modeling_gemma as MG
    import utils as U
    cfg = W.full_config(224)
    pcfg = MG.PaliGemmaConfig(**{k: v for k, v in cfg.items() if k not in ("bos_token_id", "eos_token_id")})
    m = U.build_model(pcfg, device="cuda")
    m.tie_weights()
    eng = m._pgmi_engine()               # binds the module tree to one engine slab
    eng.fill_synthetic(SEED, W.init_policy)  # the synthetic 3B weights, straight into that slab
    eng.prepare()
    yield m.eval()
    del m
    torch.cuda.empty_cache()


def _check_rows(lg, g):
    """lg: (L, V) fp32 prefill logits vs the reference's per-row summaries."""
    L = lg.shape[0]
    top = torch.gather(lg, 1, torch.from_numpy(g["rows_topk_idx"]).cuda()).cpu().numpy()
    assert np.abs(top - g["rows_topk_val"]).max() <= 0.25, np.abs(top - g["rows_topk_val"]).max()
    am = lg.argmax(-1).cpu().numpy()
    decisive = (g["rows_topk_val"][:, 0] - g["rows_topk_val"][:, 1]) > 0.25
    assert np.array_equal(am[decisive], g["rows_topk_idx"][decisive, 0])
    s = lg[::8][:, torch.from_numpy(g["sample_idx"]).cuda()].cpu().numpy()
    # two bf16 implementations, each ~2.4 % rel-L2 from the fp32 truth (full_fp32.npz ref_bf16_rel_l2:
    # mean 0.024, max 0.028), are expected ~sqrt(2) x 2.4 % ~ 3.4 % apart row by row
    per_row = [rel(s[i], g["rows_sample_vals"][i]) for i in range(L // 8)]
    assert np.mean(per_row) < 4e-2 and max(per_row) < 6e-2, (np.mean(per_row), max(per_row))
    # per-row energy (sum of squares over all 257,216 logits; the plain sum is dominated by
    # cancellation: sqrt(V) x per-logit noise ~ the sums themselves)
    sumsq = (lg.double() ** 2).sum(-1).cpu().numpy()
    assert np.abs(sumsq / g["rows_sumsq"] - 1).max() < 3e-2, np.abs(sumsq / g["rows_sumsq"] - 1).max()


@torch.no_grad()
def test_prefill_all_row_logits_full_vocab(model, G):
    import modeling_gemma as MG
    from pgmi.lazy_logits import LazyLogits
    g = G["256"]
    ids = torch.from_numpy(g["ids"]).cuda()
    px = torch.from_numpy(pixels_from_u8(G["px"]["u8_0_224"])[None]).cuda()
    L = ids.shape[1]
    V = W.full_config(224)["text_config"]["vocab_size"]
    out = model(input_ids=ids, pixel_values=px, attention_mask=torch.ones_like(ids), kv_cache=MG.KVCache())
    lz = out["logits"]
    assert isinstance(lz, LazyLogits) and tuple(lz.shape) == (1, L, V) and lz.dtype == torch.float32
    last = lz[:, -1, :]
    assert not lz.is_materialized
    top = torch.gather(last[0], 0, torch.from_numpy(g["topk_idx"][0]).cuda()).cpu().numpy()
    assert np.abs(top - g["topk_val"][0]).max() <= 0.25
    full = lz.materialize()
    assert tuple(full.shape) == (1, L, V)
    _check_rows(full[0], g)
    # the eager all-row mode (the reference's behaviour) runs the same lm_head GEMM: identical rows
    # 0..L-2; row L-1 is the lazy form's eager GEMV row (same values up to accumulation order)
    model.pgmi_prefill_logits = "all"
    try:
        eager = model(input_ids=ids, pixel_values=px, attention_mask=torch.ones_like(ids),
                      kv_cache=MG.KVCache())["logits"]
    finally:
        model.pgmi_prefill_logits = "lazy"
    assert isinstance(eager, torch.Tensor)
    assert torch.equal(eager[:, :-1], full[:, :-1])
    assert rel(eager[0, -1].cpu().numpy(), full[0, -1].cpu().numpy()) < 1e-3
    _check_rows(eager[0], g)


def _dropin_loop(model, G, n=64, forced=None):
    """inference.py:55-78 through the drop-in module (pixel_values re-passed, the float mask column appended,
    argmax of logits[:, -1, :], .item() per token; the greedy lookahead on, as by default).  forced: feed these
    tokens instead of the argmax (teacher forcing on the reference's path).  Returns the tokens chosen, the
    sampled logits of every step (the fixture's 1,024 vocabulary entries) and the cache."""
    import modeling_gemma as MG
    g = G["64"]
    ids = torch.from_numpy(g["ids"]).cuda()
    px = torch.from_numpy(pixels_from_u8(G["px"]["u8_0_224"])[None]).cuda()
    sidx = torch.from_numpy(g["sample_idx"]).cuda()
    mask = torch.ones_like(ids)
    kv = MG.KVCache()
    toks, vals = [], []
    for t in range(n):
        out = model(input_ids=ids, pixel_values=px, attention_mask=mask, kv_cache=kv)
        kv = out["kv_cache"]
        last = out["logits"][:, -1, :]
        vals.append(last[0, sidx].clone())
        nxt = torch.argmax(last, dim=-1, keepdim=True)
        assert nxt.size() == (1, 1)
        nxt = nxt.squeeze(0)
        toks.append(int(nxt.item()))
        if forced is not None:
            nxt = torch.tensor([int(forced[t])], device=ids.device)
        ids = nxt.unsqueeze(-1)
        mask = torch.cat([mask, torch.ones((1, 1), device=ids.device)], dim=-1)
    return np.array(toks), torch.stack(vals).cpu().numpy(), kv


@torch.no_grad()
def test_inference_loop_full_size(model, G):
    """inference.py:55-78 through the drop-in module, 64 greedy tokens vs the reference's, and every step's
    logits (through the lookahead's hits) held to SURVEY sec.8c's per-step rule against full_bf16.npz and its
    fp32 truth, up to the first step where the free-running tokens may part (the reference indecisive)."""
    g, f = G["64"], G["64f"]
    toks, vals, kv = _dropin_loop(model, G)
    ref = g["tokens"].reshape(-1)
    diff = np.nonzero(toks != ref)[0]
    upto = 64
    if len(diff):
        assert g["margin"][diff[0]] < 0.25, (diff[0], toks[:diff[0] + 2], ref[:diff[0] + 2])
        upto = int(diff[0]) + 1  # the step that chose the other token still ran on the reference's prefix
    check_model_parity("dropin_loop_free", vals[:upto], g["sample_vals"][:upto], f["sample_vals"][:upto])
    assert kv.num_items() == g["ids"].shape[1] + 63


@torch.no_grad()
def test_inference_loop_teacher_forced_full_size(model, G):
    """The same loop fed the reference's own tokens (so every step runs on the reference's path): all 64 steps'
    logits held to the per-step rule against full_bf16.npz and full_fp32.npz, with the greedy lookahead handing
    back the steps whose token it predicted (the reference's token equals our argmax wherever it is decisive)."""
    from pgmi.lookahead import lookahead_for
    g, f = G["64"], G["64f"]
    la = lookahead_for(model._pgmi_engine(), 1)
    hits = la.hits
    toks, vals, _ = _dropin_loop(model, G, forced=g["tokens"].reshape(-1))
    check_model_parity("dropin_loop_teacher_forced", vals, g["sample_vals"], f["sample_vals"])
    assert lookahead_for(model._pgmi_engine(), 1).hits - hits >= 32


@torch.no_grad()
def test_lookahead_bit_identical_greedy_and_forced(model, G):
    """The greedy lookahead of the drop-in decode step (pgmi/lookahead.py, on by default) returns exactly
    what the step run on demand returns: the inference.py loop for 24 tokens with the lookahead on and off,
    logits bit for bit, once greedy (every lookahead used) and once with every third token forced to the
    runner-up (a miss: the asked step runs behind the wasted lookahead, whose KV row is overwritten).  After
    two misses in a row the lookahead stands down for that cache."""
    import modeling_gemma as MG
    from pgmi.lookahead import lookahead_for
    g = G["64"]
    ids0 = torch.from_numpy(g["ids"]).cuda()
    px = torch.from_numpy(pixels_from_u8(G["px"]["u8_0_224"])[None]).cuda()

    def loop(lookahead, forced_every=0, n=24):
        model.pgmi_lookahead = lookahead
        try:
            ids, mask, kv = ids0, torch.ones_like(ids0), MG.KVCache()
            outs = []
            for t in range(n):
                out = model(input_ids=ids, pixel_values=px, attention_mask=mask, kv_cache=kv)
                lg = out["logits"][:, -1, :]
                outs.append(lg.clone())
                pick = 1 if forced_every and t % forced_every == forced_every - 1 else 0
                nxt = torch.topk(lg, 2, dim=-1).indices[:, pick:pick + 1]
                _ = int(nxt.item())
                ids = nxt
                mask = torch.cat([mask, torch.ones((1, 1), device=ids.device)], dim=-1)
            return torch.cat(outs, 0), kv
        finally:
            model.pgmi_lookahead = True

    eng = model._pgmi_engine()
    for forced in (0, 3):
        on, kv_on = loop(True, forced)
        off, kv_off = loop(False, forced)
        assert torch.equal(on, off), forced
        n = kv_on.num_items()
        assert n == kv_off.num_items() == ids0.shape[1] + 23
        assert torch.equal(kv_on._slab[:, :, :, :n], kv_off._slab[:, :, :, :n])
    la = lookahead_for(eng, 1)
    hits = la.hits
    # forced tokens on two steps in a row: the lookahead stands down for the cache
    ids, mask, kv = ids0, torch.ones_like(ids0), MG.KVCache()
    for t in range(8):
        out = model(input_ids=ids, pixel_values=px, attention_mask=mask, kv_cache=kv)
        ids = torch.topk(out["logits"][:, -1, :], 2, dim=-1).indices[:, 1:2]
        mask = torch.cat([mask, torch.ones((1, 1), device=ids.device)], dim=-1)
    assert la.hits == hits and la.pending is None


@torch.no_grad()
def test_lookahead_two_interleaved_caches(model, G):
    """Two sequences decoded in alternation on one model (two KVCaches, greedy): every step finds the pending
    lookahead on the other cache, runs behind it on the caller's stream and starts its own; each cache's
    logits and KV rows equal those of the same alternation with the lookahead off, and the lookahead stands
    down for both caches after two misses each."""
    import modeling_gemma as MG
    from pgmi.lookahead import lookahead_for
    g = G["64"]
    ids0 = torch.from_numpy(g["ids"]).cuda()
    px = [torch.from_numpy(pixels_from_u8(G["px"]["u8_0_224"])[None]).cuda(),
          torch.from_numpy(pixels_from_u8(G["px"]["u8_1_224"])[None]).cuda()]

    def alternate(lookahead, n=12):
        model.pgmi_lookahead = lookahead
        try:
            st = [{"ids": ids0, "mask": torch.ones_like(ids0), "kv": MG.KVCache(), "out": []} for _ in range(2)]
            for t in range(n):
                for j, s in enumerate(st):
                    out = model(input_ids=s["ids"], pixel_values=px[j], attention_mask=s["mask"], kv_cache=s["kv"])
                    lg = out["logits"][:, -1, :]
                    s["out"].append(lg.clone())
                    s["ids"] = torch.argmax(lg, dim=-1, keepdim=True)
                    _ = int(s["ids"].item())
                    s["mask"] = torch.cat([s["mask"], torch.ones((1, 1), device=lg.device)], dim=-1)
            return st
        finally:
            model.pgmi_lookahead = True

    on, off = alternate(True), alternate(False)
    for a, b in zip(on, off):
        assert torch.equal(torch.cat(a["out"]), torch.cat(b["out"]))
        n = a["kv"].num_items()
        assert n == b["kv"].num_items() == ids0.shape[1] + 11
        assert torch.equal(a["kv"]._slab[:, :, :, :n], b["kv"]._slab[:, :, :, :n])
        assert getattr(a["kv"], "_pgmi_misses", 0) >= 2
    assert lookahead_for(model._pgmi_engine(), 1).pending is None
