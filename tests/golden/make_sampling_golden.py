"""Generate tests/golden/sampling.npz by running the REFERENCE's nucleus sampler,
inference._sample_top_p (inference.py:15-24), with torch's own multinomial.

Runs only in the survey container (imports /root/reference/inference.py; `fire` is stubbed
because it is not installed).  The fixture is data: probability rows, top_p, and the token
counts of N reference draws per row (torch.manual_seed per row), which pin the kept set and
the renormalised distribution the oracle (oracle/sampling_np.py) and the HIP kernel must match
in distribution.

    python tests/golden/make_sampling_golden.py
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, REF)
sys.modules.setdefault("fire", types.SimpleNamespace(Fire=lambda *a, **k: None))
import inference as RI  # noqa: E402

N_DRAWS = 20000


def rows():
    g = torch.Generator().manual_seed(7)
    out = []
    # peaked logits, temperature 0.8 (inference.py defaults), p = 0.9
    lg = torch.randn(64, generator=g) * 3.0
    out.append((torch.softmax(lg / 0.8, -1), 0.9, "peaked64_t0.8_p0.9"))
    # flat-ish over 512 tokens, p = 0.5
    lg = torch.randn(512, generator=g) * 0.5
    out.append((torch.softmax(lg, -1), 0.5, "flat512_p0.5"))
    # exact ties (quantised probabilities), p = 0.7
    q = torch.tensor([8, 8, 8, 4, 4, 2, 2, 2, 1, 1, 0, 0], dtype=torch.float32)
    out.append((q / q.sum(), 0.7, "ties12_p0.7"))
    # p small enough that only the top token survives
    lg = torch.randn(100, generator=g) * 2.0
    out.append((torch.softmax(lg, -1), 0.05, "top1_100_p0.05"))
    return out


def main():
    probs, ps, counts, names = [], [], [], []
    for i, (p, top_p, name) in enumerate(rows()):
        torch.manual_seed(1000 + i)
        batch = p[None].expand(N_DRAWS, -1).contiguous()
        tok = RI._sample_top_p(batch.clone(), top_p).reshape(-1).numpy()
        probs.append(p.numpy().astype(np.float32))
        ps.append(top_p)
        counts.append(np.bincount(tok, minlength=p.numel()).astype(np.int64))
        names.append(name)
    V = max(len(p) for p in probs)
    pad = lambda a, dt: np.stack([np.pad(x, (0, V - len(x))) for x in a]).astype(dt)  # noqa: E731
    np.savez_compressed(os.path.join(HERE, "sampling.npz"), probs=pad(probs, np.float32),
                        lengths=np.array([len(p) for p in probs]), top_p=np.array(ps, np.float64),
                        counts=pad(counts, np.int64), names=np.array(names), n_draws=N_DRAWS)
    print("wrote sampling.npz:", names)


if __name__ == "__main__":
    main()
