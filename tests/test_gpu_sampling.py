"""Nucleus sampling kernel (pgmi_sample_top_p, kernels_sample.hip) vs the oracle
(oracle/sampling_np.py, pinned to the reference's draws by tests/test_cpu_sampling.py).

Given the same probabilities, top_p and uniform u, the kernel's token must be the oracle's
inverse-CDF token (bit-exact index) wherever the oracle's decision margin exceeds 1e-6 (draws
closer to a cumulative-sum boundary may flip under another summation order; they are counted
and must be rare).  The kept mass Z must match to fp32 rounding."""
import os

import numpy as np
import pytest
import torch

from oracle import sampling_np as S
from oracle import weights as W

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from pgmi import Engine
    e = Engine(W.small_config(vision_layers=1, text_layers=1, vocab=1024), max_batch=1, max_seq=64, max_kv=64)
    e.prepare()
    return e


@pytest.fixture(scope="module")
def G(golden_dir):
    return np.load(os.path.join(golden_dir, "sampling.npz"))


def _check(eng, probs, top_p, us, temperature=None, logits=None):
    rows = len(us)
    x = logits if logits is not None else probs
    xt = torch.from_numpy(np.ascontiguousarray(np.broadcast_to(x, (rows, x.shape[-1])))).cuda()
    ut = torch.from_numpy(np.asarray(us, np.float32)).cuda()
    tok, kept = eng.sample_top_p(xt, top_p, temperature, u=ut, return_kept_mass=True)
    torch.cuda.synchronize()
    tok, kept = tok.cpu().numpy(), kept.cpu().numpy()
    bad, close = 0, 0
    for i, u in enumerate(us):
        ref, Z, margin = S.sample_top_p(probs, top_p, float(np.float32(u)))
        if margin <= 1e-6 * max(1.0, Z):
            close += 1
            continue
        bad += int(tok[i] != ref)
        assert abs(kept[i] - Z) <= 2e-6 * Z, (i, kept[i], Z)
    return bad, close


def test_fixture_rows_exact(eng, G):
    rng = np.random.default_rng(0)
    for i, name in enumerate(G["names"]):
        L = int(G["lengths"][i])
        p = G["probs"][i][:L].astype(np.float32)
        us = np.concatenate([rng.random(512), [0.0, 0.5, 1 - 2 ** -24]]).astype(np.float32)
        bad, close = _check(eng, p, float(G["top_p"][i]), us)
        assert bad == 0, name
        assert close <= 4, (name, close)


@pytest.mark.parametrize("V,temperature,top_p", [(257216, 0.8, 0.9), (257216, 1.0, 0.5), (4096, 0.3, 0.99),
                                                 (1000, 2.0, 1.0), (77, 0.8, 0.0)])
def test_logits_with_temperature(eng, V, temperature, top_p):
    rng = np.random.default_rng(V + int(top_p * 100))
    logits = (rng.standard_normal(V) * 3).astype(np.float32)
    probs = S.softmax_t(logits, temperature)
    us = rng.random(64).astype(np.float32)
    bad, close = _check(eng, probs, top_p, us, temperature=temperature, logits=logits)
    # the device softmax may differ from numpy's by an ulp per entry
    assert bad <= 1 and close <= 4, (bad, close)


def test_distribution_matches_reference_draws(eng, G):
    """Stratified u over [0, 1): the kernel's token frequencies are the kept distribution that
    the reference's multinomial draws fit (tests/test_cpu_sampling.py)."""
    m = 4096
    for i, name in enumerate(G["names"]):
        L = int(G["lengths"][i])
        p = G["probs"][i][:L].astype(np.float32)
        q = S.kept_distribution(p, float(G["top_p"][i]))
        xt = torch.from_numpy(np.ascontiguousarray(np.broadcast_to(p, (m, L)))).cuda()
        ut = torch.from_numpy(((np.arange(m) + 0.5) / m).astype(np.float32)).cuda()
        tok = eng.sample_top_p(xt, float(G["top_p"][i]), u=ut).cpu().numpy()
        freq = np.bincount(tok, minlength=L) / m
        assert np.array_equal(freq > 0, q > 0), name
        assert np.abs(freq - q).max() <= 2.0 / m, name


def test_generate_with_sampling_is_reproducible(eng):
    cfg = W.small_config(vision_layers=1, text_layers=1, vocab=1024)
    from pgmi import Engine
    e = Engine(cfg, max_batch=2, max_seq=300, max_kv=320)
    e.fill_synthetic(5, W.init_policy)
    e.prepare()
    n_img = W.num_image_tokens(cfg)
    ids = torch.tensor([[cfg["image_token_index"]] * n_img + [2, 17, 99, 108]] * 2).cuda()
    px = torch.rand((2, 3, 224, 224), device="cuda") * 2 - 1
    g1 = torch.Generator(device="cuda").manual_seed(11)
    g2 = torch.Generator(device="cuda").manual_seed(11)
    a = e.generate(ids, px, 8, do_sample=True, temperature=0.8, top_p=0.9, generator=g1)
    b = e.generate(ids, px, 8, do_sample=True, temperature=0.8, top_p=0.9, generator=g2)
    assert torch.equal(a, b)
    assert int(a.min()) >= 0 and int(a.max()) < cfg["text_config"]["vocab_size"]


def test_rejects_bad_arguments(eng):
    x = torch.rand((2, 10), device="cuda")
    with pytest.raises(ValueError):
        eng.sample_top_p(x, 0.9, u=torch.rand(3, device="cuda"))
    with pytest.raises(ValueError):
        eng.sample_top_p(x, -0.5)
