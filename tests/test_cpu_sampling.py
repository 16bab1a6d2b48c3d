"""Nucleus sampling oracle (oracle/sampling_np.py) vs the reference's own draws.

tests/golden/sampling.npz holds N multinomial draws of inference._sample_top_p
(inference.py:15-24) per probability row (tests/golden/make_sampling_golden.py).  The oracle's
kept set must be exactly the support of those draws, and its renormalised distribution must fit
the draw counts (chi-square).  The inverse-CDF draw of the oracle (the rule the HIP kernel
implements) must reproduce that distribution over a stratified u grid."""
import numpy as np
import pytest
from scipy import stats

from oracle import sampling_np as S


@pytest.fixture(scope="module")
def G(golden_dir):
    import os
    return np.load(os.path.join(golden_dir, "sampling.npz"))


def _rows(G):
    for i, name in enumerate(G["names"]):
        L = int(G["lengths"][i])
        yield str(name), G["probs"][i][:L], float(G["top_p"][i]), G["counts"][i][:L]


def test_kept_set_is_the_reference_support(G):
    for name, p, top_p, counts in _rows(G):
        q = S.kept_distribution(p, top_p)
        assert np.array_equal(q > 0, counts > 0), name


def test_kept_distribution_fits_reference_draws(G):
    n = int(G["n_draws"])
    for name, p, top_p, counts in _rows(G):
        q = S.kept_distribution(p, top_p)
        k = q > 0
        if k.sum() < 2:
            assert counts[k].sum() == n, name
            continue
        chi = stats.chisquare(counts[k], q[k] * n)
        assert chi.pvalue > 1e-4, (name, chi)


def test_inverse_cdf_draw_reproduces_the_distribution(G):
    m = 20000
    for name, p, top_p, counts in _rows(G):
        q = S.kept_distribution(p, top_p)
        us = (np.arange(m) + 0.5) / m
        toks = np.array([S.sample_top_p(p, top_p, u)[0] for u in us])
        freq = np.bincount(toks, minlength=len(p)) / m
        assert np.abs(freq - q).max() < 2.0 / m + 1e-9, name


def test_temperature_softmax_matches_torch():
    import torch
    rng = np.random.default_rng(3)
    x = (rng.standard_normal((3, 5000)) * 4).astype(np.float32)
    ref = torch.softmax(torch.from_numpy(x) / 0.8, -1).numpy()
    got = S.softmax_t(x, 0.8)
    assert np.abs(got - ref).max() <= 2e-6 * np.abs(ref).max()
