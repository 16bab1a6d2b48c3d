"""Probe: B-row greedy decode as one hipGraph launch per step (pgmi_decode) against n steps per launch
(pgmi_decode_steps), alternating on one engine and one KV cache (every pass restarts at KV row L, so
all passes decode the same token sequence).  Prints ms per step per form and whether the token
records agree bit for bit.

    python tools/probes/multistep_probe.py [--batch 1] [--steps 64] [--rounds 3] [--ns 4,8,16]
"""
import argparse
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "multimodal-financial-analysis-tool-using-paligemma_amd"))
from pgmi import Engine  # noqa: E402
from pgmi.synthetic import init_policy, paligemma_3b_config, prompt_ids  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--ns", default="4,8,16")
    a = ap.parse_args()
    ns = [int(x) for x in a.ns.split(",")]
    cfg = paligemma_3b_config(224)
    n_img = 256
    L = n_img + 32
    B = a.batch
    cap = (L + a.steps + 8 + 63) // 64 * 64
    eng = Engine(cfg, max_batch=B, max_seq=L, max_kv=cap)
    eng.fill_synthetic(1234, init_policy)
    eng.prepare()
    g = torch.Generator(device="cuda").manual_seed(5)
    px = (torch.rand((B, 3, 224, 224), generator=g, device="cuda") * 2 - 1).contiguous()
    ids = torch.from_numpy(prompt_ids(cfg["image_token_index"], n_img, cfg["text_config"]["vocab_size"])).cuda()
    ids = ids.expand(B, -1).contiguous()
    kv = eng.new_kv(B, cap)
    feats = eng.project(eng.vision(px))
    lg = eng.lm_forward(kv, 0, torch.arange(L).expand(B, L), ids=ids, image_feats=feats, logits_rows=2)
    first = eng.argmax(lg[:, 0])
    V = cfg["text_config"]["vocab_size"]
    logits = torch.empty((B, V), dtype=torch.float32, device="cuda")

    def single(n_total, rec):
        cur = first.clone()
        for t in range(n_total):
            eng.decode(cur, kv, L + t, L + t + 1, logits=logits, next_ids=cur, graph=True)
            if rec is not None:
                rec[t].copy_(cur)
        return cur

    recs = {}

    def multi(n_total, n, rec):
        cur = first.clone()
        t = 0
        while t < n_total:
            k = min(n, n_total - t)
            eng.decode_steps(cur, kv, L + t, L + t + 1, k, logits=logits, tokens=recs[n][t:t + k] if rec else None,
                             graph=True)
            t += k
        return cur

    for n in ns:
        recs[n] = torch.empty((a.steps, B), dtype=torch.int64, device="cuda")
    ref = torch.empty((a.steps, B), dtype=torch.int64, device="cuda")
    # capture every form's graphs (first call eager, second captured), token records from the same start
    single(a.steps, ref)
    for n in ns:
        for rec in (True, True, False, False):
            multi(a.steps, n, rec)
    single(a.steps, None)
    torch.cuda.synchronize()
    for n in ns:
        print(f"n={n}: token record equal to the one-step form: {bool(torch.equal(recs[n], ref))}", flush=True)

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / a.steps

    for r in range(a.rounds):
        row = [f"single {timed(lambda: single(a.steps, None)):.4f}"]
        for n in ns:
            row.append(f"n={n} {timed(lambda: multi(a.steps, n, False)):.4f}")
        print(f"round {r}: ms/step " + ", ".join(row), flush=True)


if __name__ == "__main__":
    main()
