"""oracle/sampling_np.py -- TEST INFRASTRUCTURE ONLY.

CPU restatement (numpy) of the reference's nucleus sampling, inference.py:15-24
(_sample_top_p) and the temperature softmax in front of it (inference.py:65,
ablation_study_fixed.py:231-232).  The reference draws with torch.multinomial; here the draw is
an inverse-CDF pick on a caller-supplied uniform u, so one (probs, p, u) has one answer that
the HIP kernel (kernels_sample.hip) must reproduce exactly.  Distributional parity with the
reference's own multinomial draws is pinned by tests/golden/sampling.npz
(tests/golden/make_sampling_golden.py ran inference._sample_top_p).

Only tests/ may use this module; the product never imports it.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


def softmax_t(logits, temperature):
    """torch.softmax(logits / temperature, dim=-1) in fp32 (inference.py:65); the sum is taken
    in float64 and rounded once, as the kernel does."""
    z = np.asarray(logits, F32) / F32(temperature)
    m = z.max(axis=-1, keepdims=True)
    e = np.exp(z - m).astype(F32)
    s = e.astype(np.float64).sum(axis=-1, keepdims=True).astype(F32)
    return (e / s).astype(F32)


def sorted_order(p_row):
    """torch.sort(probs, descending=True) (inference.py:17); equal values in index order."""
    p_row = np.asarray(p_row, F32)
    return np.lexsort((np.arange(p_row.size), -p_row.astype(np.float64)))


def nucleus(p_row, top_p):
    """inference.py:17-21: the kept prefix of the descending order (mask = cumsum - p > top_p
    drops a token) and its mass Z.  Returns (order, k = number kept, cumsum, Z)."""
    order = sorted_order(p_row)
    ps32 = np.asarray(p_row, F32)[order]
    ps = ps32.astype(np.float64)
    c = np.cumsum(ps)  # torch's CPU cumsum of fp32 accumulates in double (acc_type) ...
    c32 = c.astype(F32)  # ... and stores fp32
    excl = (c32 - ps32).astype(F32)  # :19 in fp32: probs_sum - probs_sort > p (p cast to fp32)
    keep = excl <= F32(top_p)
    k = int(np.argmin(keep)) if not keep.all() else len(keep)  # the kept prefix
    k = max(k, 1)
    return order, k, c, float(c[k - 1])


def kept_distribution(p_row, top_p):
    """probs_sort after :20-21 scattered back to vocabulary order (what multinomial draws from)."""
    order, k, c, Z = nucleus(p_row, top_p)
    q = np.zeros(len(order), np.float64)
    q[order[:k]] = np.asarray(p_row, np.float64)[order[:k]] / Z
    return q


def sample_top_p(p_row, top_p, u):
    """:22-23 with the multinomial draw made by inverse CDF: the first sorted position whose
    cumulative kept mass exceeds u * Z.  Returns (token index, Z, margin) where margin is the
    distance of the draw target u*Z from the nearest cumulative sum -- draws with a tiny margin
    may legitimately differ under another summation order.  (The cut-off itself is decided by
    the reference's fp32 formula, which the kernel evaluates the same way.)"""
    order, k, c, Z = nucleus(p_row, top_p)
    r = float(u) * Z
    j = int(np.searchsorted(c[:k], r, side="right"))
    j = min(j, k - 1)
    margin = np.abs(c[:k] - r).min()
    return int(order[j]), Z, float(margin)
